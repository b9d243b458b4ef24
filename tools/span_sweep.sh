#!/bin/bash
# k_lines LDS staging span sweep (BJX_SPAN_BYTES; 0 = unstaged, max occupancy)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for sp in ${SPANS:-0 6144 8192 9216 12288}; do
  echo "span=$sp $(BJX_SPAN_BYTES=$sp timeout -k 10 120 python tools/scan_stats.py ${CFG:-cfg3} ${LINES:-20000000} 2 2>/dev/null | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["phases"]["resolve"], d["device_ms"])')"
done
