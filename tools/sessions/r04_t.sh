#!/bin/bash
# Round-4 session: a GPU test subset (TESTS), then a cfg3 kernel trace of the
# bench (and of BENCH2 args when set).
#   TESTS="tests/test_gpu_parity.py ..." tools/r04_t.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-t}; repo=$PWD
out=$repo/gpurun_out/$tag; mkdir -p "$out"
if [ -n "${TESTS:-tests}" ] && [ "${TESTS}" != none ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 200 --timeout-method thread > "$out/tests.log" 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o trace --output-format csv \
  -- python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline ${BENCH_ARGS:-} > "$out/trace.log" 2>&1 || exit $?
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/trace.log" | tr '\n' ' '; echo
python3 - "$out" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/trace_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-48s %4s %8.3f" % (r["Name"][:48], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
if [ -n "${BENCH2:-}" ]; then
  timeout -k 10 300 python3 "$repo/bench.py" --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline $BENCH2 > "$out/bench2.log" 2>&1 || exit $?
  grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/bench2.log" | tr '\n' ' '; echo
fi
