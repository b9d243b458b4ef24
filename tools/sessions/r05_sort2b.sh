#!/bin/bash
# two-level grouping, round 2: hot-key tests, cfg5h / cfg3 benches, kernel traces of both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
o=$repo/gpurun_out/sort2b
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -20 $o/tests.log; exit 1; }
tail -1 $o/tests.log
for c in cfg5h cfg3; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $o/b_$c.log; exit 1; }
done
python3 tools/bench_summary.py $o/b_cfg5h.log $o/b_cfg3.log
cd /tmp && export TMPDIR=/tmp
for c in cfg5h cfg3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/tr_$c -o tr --output-format csv -- python3 $repo/bench.py --config $c --steps 2 --warmup 2 --no-cpu-baseline --bans-steps 0 > $o/tr_$c.log 2>&1 || { echo "trace $c failed"; exit 1; }
done
echo done
