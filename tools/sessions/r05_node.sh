#!/bin/bash
# node checks: node + sharded + partition tests, the 2-engine node bench (2 warm-up steps), its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "nodetests|400|python -u -m pytest tests/test_gpu_node.py tests/test_gpu_parity.py -k 'node or sharded or partition or workload' -x -q --timeout 200 --timeout-method thread" \
  "nodebench|400|python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline" \
  "nodetrace|300|tools/r05_node_trace.sh"
