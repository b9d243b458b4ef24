#!/bin/bash
# Round-5 starting point: k_scan ablation (BJX_DEBUG_SKIP bits) and scan counters, cfg3 and cfg4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "stats_cfg3|200|python tools/scan_stats.py cfg3 20000000 2" \
  "stats_cfg4|200|python tools/scan_stats.py cfg4 2000000 2" \
  "abl_cfg3|400|CFG=cfg3 LINES=20000000 tools/scan_ablation.sh" \
  "abl_cfg4|400|CFG=cfg4 LINES=2000000 tools/scan_ablation.sh"
