#!/bin/bash
# bench lines of the current tree: cfg3 (default), cfg5, cfg4, cfg2 (no CPU baseline)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
tools/gpu_session.sh \
  "b_cfg3|300|python bench.py --no-cpu-baseline > gpurun_out/bench/cfg3.json" \
  "b_cfg5|300|python bench.py --no-cpu-baseline --config cfg5 > gpurun_out/bench/cfg5.json" \
  "b_cfg4|300|python bench.py --no-cpu-baseline --config cfg4 > gpurun_out/bench/cfg4.json" \
  "b_cfg2|300|python bench.py --no-cpu-baseline --config cfg2 > gpurun_out/bench/cfg2.json"
