#!/bin/bash
# Cold first batch (empty state tables): kernel trace of tools/scan_stats.py
# (state_clear before every batch) at cfg3 and cfg5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
mkdir -p gpurun_out/cold
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-cfg3 cfg5}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$repo/gpurun_out/cold/$cfg" -o tr --output-format csv \
    -- python3 "$repo/tools/scan_stats.py" $cfg ${LINES:-20000000} 2 > "$repo/gpurun_out/cold/$cfg.log" 2>&1 || exit $?
  tail -2 "$repo/gpurun_out/cold/$cfg.log" | cut -c1-600
done
