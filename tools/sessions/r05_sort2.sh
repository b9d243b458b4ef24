#!/bin/bash
# two-level event grouping (k_bucket_apply): GPU parity subset, then cfg3 / cfg5h / cfg2 benches with it and without (BJX_SORT2=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/sort2
o=gpurun_out/sort2
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py tests/test_gpu_parity.py tests/test_gpu_state_growth.py tests/test_gpu_node.py > $o/tests.log 2>&1; echo "tests rc=$?" | tee -a $o/rc.txt
tail -3 $o/tests.log
for c in cfg3 cfg5h cfg2; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $o/b_$c.log; exit 1; }
  BJX_SORT2=0 timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b0_$c.log 2>&1 || { echo "bench0 $c failed"; exit 1; }
done
python3 tools/bench_summary.py $o/b_cfg3.log $o/b0_cfg3.log $o/b_cfg5h.log $o/b0_cfg5h.log $o/b_cfg2.log $o/b0_cfg2.log 2>&1 | tee $o/summary.txt
