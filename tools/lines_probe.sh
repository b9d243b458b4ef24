#!/bin/bash
# k_lines diagnostics at cfg3: lookup-image and plan-class sizes (BJX_DEBUG_IMG),
# per-segment wave clocks (BJX_PROF_LINES; only with a library built with
# BJX_PROF=1, e.g. `BJX_PROF=1 python -m banjax_amd.build --force`, and PROF=1
# here) and the kernel-time ablation (tools/lines_ablation2.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/lines_probe; mkdir -p $o
if [ "${PROF:-0}" = 1 ]; then export BJX_PROF_LINES=1; fi
BJX_DEBUG_IMG=1 timeout -k 10 120 python -u tools/scan_stats.py cfg3 ${LINES:-40000000} 2 > $o/prof.log 2>&1 || exit $?
grep "\[bjx\]" $o/prof.log
DBGS="${DBGS:-0 16 32 64 8}" LINES=${LINES:-40000000} tools/lines_ablation2.sh
