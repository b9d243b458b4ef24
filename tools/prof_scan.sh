#!/bin/bash
# PMC + kernel-trace passes over tools/scan_stats.py (one workload); outputs under gpurun_out/prof_<tag>/
# usage: tools/prof_scan.sh <tag> <workload> <lines>
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; wl=$2; n=$3
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o trace --output-format csv -- python3 tools/scan_stats.py $wl $n 2 > $out/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-include-regex "k_scan|k_lines|k_dfa" -d $out/pmc1 -o pmc1 --output-format csv -- python3 tools/scan_stats.py $wl $n 1 > $out/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_scan|k_lines|k_dfa" -d $out/pmc2 -o pmc2 --output-format csv -- python3 tools/scan_stats.py $wl $n 1 > $out/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT --kernel-include-regex "k_scan|k_lines|k_dfa" -d $out/pmc3 -o pmc3 --output-format csv -- python3 tools/scan_stats.py $wl $n 1 > $out/pmc3.log 2>&1
find $out -name "*.csv" | head -20
