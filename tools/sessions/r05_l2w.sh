#!/bin/bash
# k_lines2 wide masks: parity tests, then cfg2 / cfg3 benches with the tables' sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "l2tests|600|python -u -m pytest tests/test_gpu_parity.py -k 'wide_masks or workload or stress or golden or bounded or shared or tile or overflow' -x -q --timeout 200 --timeout-method thread" \
  "golden|300|python -u -m pytest tests/test_golden.py -x -q --timeout 200 --timeout-method thread" \
  "cfg2|400|BJX_DEBUG_IMG=1 python bench.py --config cfg2 --no-cpu-baseline" \
  "cfg3|400|python bench.py --no-cpu-baseline"
