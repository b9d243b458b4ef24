#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py for each config in CFGS
# (gpurun_out/trace_<cfg>/tr_kernel_stats.csv, tr_kernel_trace.csv)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in ${CFGS:-cfg3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$repo/gpurun_out/trace_$c" -o tr --output-format csv \
    -- python3 "$repo/bench.py" --config $c --no-cpu-baseline --bans-steps 0 > "$repo/gpurun_out/trace_$c.log" 2>&1 || exit $?
done
