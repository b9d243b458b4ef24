#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
tools/gpu_session.sh \
  "tests|700|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "cold_full|400|tools/r05_cold3.sh" \
  "b_cfg3|300|python bench.py --no-cpu-baseline > gpurun_out/bench/cfg3.json" \
  "b_cfg5|300|python bench.py --no-cpu-baseline --config cfg5 > gpurun_out/bench/cfg5.json"
