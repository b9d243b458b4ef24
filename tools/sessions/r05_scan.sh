#!/bin/bash
# k_scan rework: parity of the scan-sensitive suites, then scan counters and ablation at cfg3 / cfg4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "scan_tests|500|python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "stats_cfg3|200|python tools/scan_stats.py cfg3 20000000 2" \
  "stats_cfg4|200|python tools/scan_stats.py cfg4 2000000 2" \
  "abl_cfg3|400|CFG=cfg3 LINES=20000000 tools/scan_ablation.sh" \
  "abl_cfg4|400|CFG=cfg4 LINES=2000000 tools/scan_ablation.sh" \
  "bench|400|python bench.py --no-cpu-baseline"
