#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
tools/gpu_session.sh \
  "rl_tests|400|python -u -m pytest tests/test_gpu_state_growth.py tests/test_gpu_hotkey.py tests/test_gpu_parity.py tests/test_gpu_node.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'state or hot or collision or overflow or rollback or growth or workload or node'" \
  "cold_full|400|tools/r05_cold3.sh" \
  "b_cfg3|300|python bench.py --no-cpu-baseline > gpurun_out/bench/cfg3.json" \
  "b_cfg5|300|python bench.py --no-cpu-baseline --config cfg5 > gpurun_out/bench/cfg5.json"
