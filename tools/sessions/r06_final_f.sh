#!/bin/bash
# Round-6 closing evidence, part F: the GPU suite on the final library, and the
# bench lines whose emission figures the last reserve change moves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "suite|800|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "bench_cfg4|300|python3 bench.py --config cfg4 --no-cpu-baseline" \
  "bench_cfg5|400|python3 bench.py --config cfg5 --no-cpu-baseline --warmup 3" \
  "bench_cfg5h|400|python3 bench.py --config cfg5h --no-cpu-baseline --warmup 3"
