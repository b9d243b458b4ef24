#!/bin/bash
# Round-4 k_scan session: parity subset, scan ablation (BJX_DEBUG_SKIP), then a
# cfg3 kernel trace of the bench.
#   tools/r04_scan.sh <tag> [tests|notests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-scan}; repo=$PWD
out=$repo/gpurun_out/$tag; mkdir -p "$out"
if [ "${2:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
CFG=cfg3 LINES=${LINES:-40000000} SKIPS="${SKIPS:-0 1 2 8 4}" bash tools/scan_ablation.sh > "$out/ablation.log" 2>&1 || exit $?
cat "$out/ablation.log"
timeout -k 10 200 python tools/scan_stats.py cfg3 ${LINES:-40000000} 2 > "$out/stats.log" 2>&1 || exit $?
tail -1 "$out/stats.log" | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv \
  -- python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/trace.log" 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/trace.log" | tr '\n' ' '; echo
