#!/bin/bash
# two-level grouping, variants: BJX_BKT=1 (records gathered into LDS) / 0 (walk through HBM) / BJX_SORT2=0 (full sort)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
o=$repo/gpurun_out/sort2c
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py > $o/tests.log 2>&1 || { echo "tests failed"; tail -20 $o/tests.log; exit 1; }
BJX_BKT=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py > $o/tests0.log 2>&1 || { echo "tests0 failed"; tail -20 $o/tests0.log; exit 1; }
tail -1 $o/tests.log $o/tests0.log
for c in cfg3 cfg5h; do
  for v in 1 0; do
    BJX_BKT=$v timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/b${v}_$c.log 2>&1 || { echo "bench $c $v failed"; tail -5 $o/b${v}_$c.log; exit 1; }
  done
  BJX_SORT2=0 timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline --bans-steps 0 > $o/bf_$c.log 2>&1 || { echo "bench $c full failed"; exit 1; }
done
python3 tools/bench_summary.py $o/b1_cfg3.log $o/b0_cfg3.log $o/bf_cfg3.log $o/b1_cfg5h.log $o/b0_cfg5h.log $o/bf_cfg5h.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  BJX_BKT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/tr$v -o tr --output-format csv -- python3 $repo/bench.py --config cfg3 --steps 2 --warmup 2 --no-cpu-baseline --bans-steps 0 > $o/tr$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
