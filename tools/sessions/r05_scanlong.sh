#!/bin/bash
# k_scan long-line hit aggregation: scan parity tests, cfg4 / cfg3 / cfg2 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "tests|600|python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread -k 'tile or overflow or workload or long or lead or golden or self_loop or short'" \
  "b_cfg4|300|python bench.py --config cfg4 --no-cpu-baseline" \
  "b_cfg3|300|python bench.py --no-cpu-baseline" \
  "b_cfg2|300|python bench.py --config cfg2 --no-cpu-baseline"
