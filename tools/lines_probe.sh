#!/bin/bash
# k_lines diagnostics at cfg3: lookup-image section sizes (BJX_DEBUG_IMG),
# per-segment wave clocks (BJX_PROF_LINES) and the kernel-time ablation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/lines_probe; mkdir -p $o
BJX_DEBUG_IMG=1 BJX_PROF_LINES=1 timeout -k 10 120 python -u tools/scan_stats.py cfg3 ${LINES:-40000000} 2 > $o/prof.log 2>&1 || exit $?
grep "\[bjx\]" $o/prof.log
DBGS="${DBGS:-0 16 32 64 8}" LINES=${LINES:-40000000} tools/lines_ablation2.sh
