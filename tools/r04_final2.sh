#!/bin/bash
# Round-4 closing check of the final tree: the whole GPU suite, the parity
# workloads again with the IP pre-lookup on (opt-in path), smoke, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "final2_suite|600|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "final2_prelookup|300|BJX_IP_PRELOOKUP=1 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k 'workload or overflow or collisions'" \
  "final2_smoke|180|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "final2_bench|400|python bench.py"
