#!/bin/bash
# two-level grouping up to 7/8 of a bucket on average: node rehearsal with it and without, cfg3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/sort2f
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_node.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -30 $o/tests.log; exit 1; }
tail -1 $o/tests.log
timeout -k 10 400 python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline > $o/b_node2.log 2>&1 || { echo "node failed"; tail -5 $o/b_node2.log; exit 1; }
BJX_SORT2=0 timeout -k 10 400 python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline > $o/bf_node2.log 2>&1 || { echo "node full failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b_cfg3.log 2>&1 || { echo "cfg3 failed"; exit 1; }
python3 tools/bench_summary.py $o/b_node2.log $o/bf_node2.log $o/b_cfg3.log
grep -o '"grouping": [0-9]*' $o/b_node2.log $o/b_cfg3.log || true
