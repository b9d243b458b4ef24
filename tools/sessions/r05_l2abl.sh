#!/bin/bash
# k_lines2 ablation (timing only, results wrong): BJX_DEBUG_L2 bits over 20M cfg3 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 0 1 2 4 8 15; do
  echo "== BJX_DEBUG_L2=$b"
  BJX_DEBUG_L2=$b timeout -k 10 200 python tools/scan_stats.py cfg3 20000000 3 2>&1 | grep '^{' | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['phases']['resolve'], d['kernel_ms'])"
done
