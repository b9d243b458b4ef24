#!/bin/bash
# Round-4 GPU session: GPU suite (default path), then cfg3 kernel traces with
# k_lines2 (default) and k_lines (BJX_LINES=1).
#   tools/r04_run.sh <tag> [suite|nosuite]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-run}; repo=$PWD
out=$repo/gpurun_out/$tag; mkdir -p "$out"
if [ "${2:-suite}" = suite ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/suite.log" 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 "$out/suite.log"
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
cd /tmp && export TMPDIR=/tmp
for L in 2 1; do
  BJX_LINES=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace$L" -o trace --output-format csv \
    -- python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/trace$L.log" 2>&1 || exit $?
  grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/trace$L.log" | tr '\n' ' '; echo
done
