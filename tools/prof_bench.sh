#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py (+ optional PMC passes on the scan
# kernel); outputs under gpurun_out/prof_<tag>/.
# usage: tools/prof_bench.sh <tag> [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; shift
out=$PWD/gpurun_out/prof_$tag
mkdir -p $out
repo=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 $repo/bench.py "$@" > $out/trace.log 2>&1
if [ -n "$BJX_PMC" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_scan" -d $out/pmc_fetch -o pmc --output-format csv -- python3 $repo/bench.py "$@" > $out/pmc_fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_scan" -d $out/pmc_write -o pmc --output-format csv -- python3 $repo/bench.py "$@" > $out/pmc_write.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_scan|k_lines|k_dfa" -d $out/pmc_sq -o pmc --output-format csv -- python3 $repo/bench.py "$@" > $out/pmc_sq.log 2>&1
fi
find $out -name "*.csv" | sort
