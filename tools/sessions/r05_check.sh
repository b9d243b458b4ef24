#!/bin/bash
# GPU suite + smoke + default bench of the current tree (round 5 checkpoints).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "suite|700|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "smoke|180|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench|400|python bench.py --no-cpu-baseline"
