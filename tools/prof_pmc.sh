#!/bin/bash
# PMC passes (one counter group per run) on kernels matching $1 over bench.py.
# usage: tools/prof_pmc.sh <tag> <kernel-regex> [bench args...]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; rx=$2; shift 2
out=$PWD/gpurun_out/pmc_$tag
mkdir -p $out
repo=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$rx" -d $out/p$i -o pmc --output-format csv -- python3 $repo/bench.py "$@" > $out/p$i.log 2>&1
done
find $out -name "*counter_collection.csv" | sort
