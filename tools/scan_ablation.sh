#!/bin/bash
# k_scan timing ablation (BJX_DEBUG_SKIP bits; results are NOT valid matches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in ${SKIPS:-0 1 2 8 4}; do
  echo "skip=$d $(BJX_DEBUG_SKIP=$d timeout -k 10 120 python tools/scan_stats.py ${CFG:-cfg3} ${LINES:-20000000} 2 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phases"]["scan"], d["scan_ms"], d["device_ms"])')"
done
