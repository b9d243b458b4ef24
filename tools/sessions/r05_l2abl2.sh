#!/bin/bash
# k_lines2 per-lane anchored walk: 20M cfg3 lines (resolve phase and kernel times), then the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python tools/scan_stats.py cfg3 20000000 3 2>&1 | grep '^{' | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['phases']['resolve'], d['kernel_ms'])" && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_cfg3.log 2>&1 && \
timeout -k 10 300 python bench.py --config cfg5 --warmup 3 --no-cpu-baseline > gpurun_out/b_cfg5.log 2>&1
