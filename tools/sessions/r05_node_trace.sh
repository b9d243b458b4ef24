#!/bin/bash
# kernel trace of the one-GPU two-engine node bench (cfg3, 2 x 125M lines): 1 warm-up + 1 timed step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
mkdir -p gpurun_out/node_trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$repo/gpurun_out/node_trace" -o tr --output-format csv \
  -- python3 "$repo/bench.py" --node-engines 2 --steps 1 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$repo/gpurun_out/node_trace/node2.log" 2>&1
