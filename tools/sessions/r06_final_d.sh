#!/bin/bash
# Round-6 closing evidence, part D: the ban log's pinned buffer reserved at a
# quarter of the batch on first use.  Emission tests, the driver's bench
# command, and the bench lines whose emission figures it moves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "bans_tests|300|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bans.py tests/test_gpu_node.py" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg3|500|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_cfg4|300|python3 bench.py --config cfg4 --no-cpu-baseline" \
  "bench_cfg5|400|python3 bench.py --config cfg5 --no-cpu-baseline --warmup 3" \
  "bench_cfg5h|400|python3 bench.py --config cfg5h --no-cpu-baseline --warmup 3"
