#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "rl_tests|400|python -u -m pytest tests/test_gpu_state_growth.py tests/test_gpu_hotkey.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'state or hot or collision or overflow or rollback or growth or workload'" \
  "cold|300|tools/r05_cold.sh"
