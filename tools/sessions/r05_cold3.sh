#!/bin/bash
# kernel trace of the default cfg3 bench's cold first step (and one warm step)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
mkdir -p gpurun_out/cold_full
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-cfg3}; do
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$repo/gpurun_out/cold_full/$cfg" -o tr --output-format csv \
  -- python3 "$repo/bench.py" --config $cfg --steps 1 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$repo/gpurun_out/cold_full/$cfg.log" 2>&1 || exit $?
done
