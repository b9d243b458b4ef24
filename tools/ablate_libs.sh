#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in ${VARIANTS:-base}; do
  BJX_LIB_PATH=$PWD/exp_libs/lib_$v.so tools/trace_lines.sh abl_$v > gpurun_out/abl_$v.txt 2>&1 || exit $?
  echo "== $v"; grep -E "k_lines|k_scan|k_dfa" gpurun_out/abl_$v.txt
done
