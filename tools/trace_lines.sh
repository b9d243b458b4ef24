#!/bin/bash
# kernel trace of tools/scan_stats.py (cfg3, $LINES lines, 2 batches) -> gpurun_out/tl_$1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD; o=$repo/gpurun_out/tl_$1; mkdir -p $o
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $o -o t --output-format csv -- python3 $repo/tools/scan_stats.py ${WL:-cfg3} ${LINES:-40000000} 2 > $o/run.log 2>&1 || exit $?
python3 - $o <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/t_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r['Name'] for k in ('k_lines', 'k_scan', 'k_dfa', 'k_nl_count')):
        print("%-48s %8.3f ms" % (r['Name'].replace('void (anonymous namespace)::', '').split('(')[0][:48], float(r['AverageNs']) / 1e6))
PY
