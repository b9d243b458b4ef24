#!/bin/bash
# k_lines diagnostics (BJX_PROF=1 library): segment clocks of the generic
# kernel, then kernel times of hit-mask vs generic at 40M cfg3 lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/lp; mkdir -p $o
BJX_DEBUG_IMG=1 BJX_PROF_LINES=1 timeout -k 10 120 python -u tools/scan_stats.py cfg3 40000000 2 > $o/prof.log 2>&1 || exit $?
[ "${PROF_ONLY:-0}" = 1 ] && exit 0
repo=$PWD
cd /tmp && export TMPDIR=/tmp
for v in hm nohm; do
  if [ $v = nohm ]; then export BJX_NO_HM=1; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $repo/$o/$v -o t --output-format csv -- python3 $repo/tools/scan_stats.py cfg3 40000000 2 > $repo/$o/$v.log 2>&1 || exit $?
done
