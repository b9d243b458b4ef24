#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bench
tools/gpu_session.sh \
  "img|120|BJX_DEBUG_IMG=1 python tools/scan_stats.py cfg3 200000 1 2>&1 | grep -i 'k_lines2'" \
  "tests|500|python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_nfa.py tests/test_gpu_plan_templates.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "b_cfg3|300|python bench.py --no-cpu-baseline > gpurun_out/bench/cfg3.json" \
  "b_cfg5|300|python bench.py --no-cpu-baseline --config cfg5 > gpurun_out/bench/cfg5.json" \
  "node_trace|400|tools/r05_node_trace.sh"
