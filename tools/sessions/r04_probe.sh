#!/bin/bash
# Round-4 probe: k_lines2 parity subset, then cfg3 kernel traces of k_lines
# (BJX_LINES=1) and k_lines2, and the instruction-cache counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
out=$repo/gpurun_out/r04_probe; mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan_templates.py tests/test_golden.py -x -q \
  --timeout 120 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 "$out/tests.log"
case $rc in 0|1) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
for L in 2 1; do
  BJX_LINES=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace$L" -o trace --output-format csv \
    -- python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/trace$L.log" 2>&1 || exit $?
  tail -1 "$out/trace$L.log" | cut -c1-300
done
timeout -s KILL 60 rocprofv3 -L > "$out/counters.txt" 2>&1 || true
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH \
  --kernel-include-regex "k_lines|k_scan|k_dfa" -d "$out/pmc_ic" -o pmc --output-format csv \
  -- python3 "$repo/bench.py" --steps 2 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/pmc_ic.log" 2>&1
echo "pmc rc=$?"
