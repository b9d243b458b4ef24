#!/bin/bash
# Time library variants side by side: tools/scan_stats.py over one workload for
# the in-tree library (base) and each exp_libs/lib_<v>.so (VARIANTS), printing
# the last repeat's kernel times and phases.  k_lines2 segment profiles
# (BJX_PROF_L2 builds) print on stderr.
#   VARIANTS="a b" tools/variant_times.sh [workload] [lines] [repeats]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
wl=${1:-cfg3}; n=${2:-20000000}; r=${3:-3}
for v in base ${VARIANTS}; do
  if [ "$v" = base ]; then lib=""; else lib=$PWD/exp_libs/lib_$v.so; fi
  echo "== $v $wl $n"
  BJX_LIB_PATH=$lib timeout -k 10 240 python tools/scan_stats.py "$wl" "$n" "$r" > gpurun_out/vt_$v.log 2> gpurun_out/vt_$v.err
  rc=$?
  grep '^\[bjx\] k_lines2 segments' gpurun_out/vt_$v.err | tail -1
  tail -1 gpurun_out/vt_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['device_ms'], d['kernel_ms'], d['phases'])"
  [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 gpurun_out/vt_$v.err; exit $rc; }
done
exit 0
