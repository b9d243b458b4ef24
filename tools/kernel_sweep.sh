#!/bin/bash
# Kernel time of the match kernels under settings of one env variable
# (rocprofv3 kernel trace of tools/scan_stats.py cfg3).
#   VAR=BJX_DFA_CHUNKS VALS="1 4 16" LINES=40000000 tools/kernel_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
out=$repo/gpurun_out/sweep_$VAR; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/v$v -o t --output-format csv -- python3 $repo/tools/scan_stats.py ${WL:-cfg3} ${LINES:-40000000} 2 > $out/v$v.log 2>&1 || exit $?
  f=$(find $out/v$v -name "t_kernel_stats.csv" | head -1)
  echo "$VAR=$v $(python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    n = r['Name'].replace('void (anonymous namespace)::','').replace('(anonymous namespace)::','').split('(')[0]
    if any(k in n for k in ('k_lines', 'k_dfa', 'k_scan', 'k_nl_count')): print(n, round(float(r['AverageNs'])/1e6,3), end='  ')
")"
done
