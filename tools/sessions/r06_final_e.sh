#!/bin/bash
# Round-6 closing evidence, part E: the pinned ban-log reserve at half the batch;
# emission tests, smoke, the driver's bench command.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "bans_tests|300|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bans.py" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg3|500|python3 bench.py --gpus 1 --steps 20 --warmup 5"
