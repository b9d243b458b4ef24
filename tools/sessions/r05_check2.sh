#!/bin/bash
# closing check of the final tree: the GPU suite, smoke, the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/check2
mkdir -p $o
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/suite.log 2>&1 || { echo "suite failed"; tail -30 $o/suite.log; exit 1; }
tail -1 $o/suite.log
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > $o/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 500 python bench.py > $o/bench.log 2>&1 || { echo "bench failed"; tail -20 $o/bench.log; exit 1; }
python3 tools/bench_summary.py $o/bench.log
