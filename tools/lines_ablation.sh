#!/bin/bash
# k_lines timing ablation (BJX_DEBUG_LINES bits; results are NOT valid matches)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 4 8 3 15; do
  echo "dbg=$d $(BJX_DEBUG_LINES=$d timeout -k 10 120 python tools/scan_stats.py cfg3 20000000 2 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phases"]["resolve"], d["device_ms"])')"
done
