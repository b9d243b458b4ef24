#!/bin/bash
# two-level grouping with the hot-key hold: hot-key + parity tests, then every config with it and without (BJX_SORT2=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
o=$repo/gpurun_out/sort2d
mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py tests/test_gpu_parity.py tests/test_gpu_state_growth.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for c in cfg3 cfg5 cfg5h cfg1 cfg2 cfg4; do
  w=3; [ $c = cfg5 ] && w=3
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup $w --no-cpu-baseline --bans-steps 0 > $o/b_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $o/b_$c.log; exit 1; }
  BJX_SORT2=0 timeout -k 10 300 python bench.py --config $c --steps 5 --warmup $w --no-cpu-baseline --bans-steps 0 > $o/bf_$c.log 2>&1 || { echo "bench $c full failed"; exit 1; }
  python3 tools/bench_summary.py $o/b_$c.log $o/bf_$c.log
done
