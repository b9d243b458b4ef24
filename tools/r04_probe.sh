#!/bin/bash
# Round-4 probe: counter list, cfg3 kernel trace on the current tree, and the
# instruction-cache counters of the match kernels (k_lines code size question).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
out=$repo/gpurun_out/r04_probe; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv \
  -- python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/trace.log" 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH \
  --kernel-include-regex "k_lines|k_scan|k_dfa" -d "$out/pmc_ic" -o pmc --output-format csv \
  -- python3 "$repo/bench.py" --steps 2 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/pmc_ic.log" 2>&1
echo "pmc rc=$?"
