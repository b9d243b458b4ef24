#!/bin/bash
# two-level grouping: the forced-path parity tests, then cfg3 / cfg4 / cfg1 benches (batch-size gate)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/sort2e
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py "tests/test_gpu_parity.py::test_two_level_grouping" > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for c in cfg3 cfg5 cfg4; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $o/b_$c.log; exit 1; }
done
python3 tools/bench_summary.py $o/b_cfg3.log $o/b_cfg5.log $o/b_cfg4.log
grep -o '"grouping": [0-9]*' $o/b_cfg3.log $o/b_cfg4.log || true
