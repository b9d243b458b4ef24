#!/bin/bash
# k_lines timing ablation on the plan path (BJX_DEBUG_LINES bits 16/32/64;
# results are NOT valid matches): rocprofv3 kernel time of k_lines per setting
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
repo=$PWD
out=$repo/gpurun_out/lines_abl2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for d in ${DBGS:-0 16 32 48 64 112 8}; do
  BJX_DEBUG_LINES=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/d$d -o t --output-format csv -- python3 $repo/tools/scan_stats.py cfg3 ${LINES:-40000000} 2 > $out/d$d.log 2>&1
  f=$(find $out/d$d -name "t_kernel_stats.csv" | head -1)
  echo "dbg=$d $(python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'k_lines' in r['Name'] or 'k_dfa' in r['Name']: print(r['Name'].replace('void (anonymous namespace)::','').split('(')[0], round(float(r['AverageNs'])/1e6,3), end='  ')
")"
done
