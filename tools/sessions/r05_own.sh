#!/bin/bash
# per-host anchored rules inlined: parity, then cfg3 / cfg5 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "tests|600|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan_templates.py tests/test_golden.py -x -q --timeout 200 --timeout-method thread" \
  "cfg3|400|BJX_DEBUG_IMG=1 python bench.py --no-cpu-baseline" \
  "cfg5|400|python bench.py --config cfg5 --no-cpu-baseline --warmup 3"
