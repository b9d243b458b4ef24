#!/bin/bash
# DFA-job census per rule (BJX_JOB_STATS) on cfg3 / cfg2 / cfg4 samples.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/${1:-jobs}; mkdir -p "$out"
for c in cfg3 cfg2 cfg4; do
  n=20000000; [ $c = cfg4 ] && n=2000000
  BJX_JOB_STATS=1 timeout -k 10 200 python tools/scan_stats.py $c $n 1 > "$out/$c.log" 2>&1 || exit $?
  grep -A16 BJX_JOB_STATS "$out/$c.log" | head -18
  tail -1 "$out/$c.log" | cut -c1-400
done
