#!/bin/bash
# Two SQ counter passes (issue / instruction mix, LDS and memory instructions)
# over tools/scan_stats.py for kernels matching PMC_REGEX, one pass per run,
# for the in-tree library and each exp_libs/lib_<v>.so in VARIANTS.
#   PMC_REGEX=k_lines2 VARIANTS="r5" tools/pmc_kernel.sh <tag> [workload] [lines]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=$1; wl=${2:-cfg3}; n=${3:-20000000}
repo=$PWD
out=$repo/gpurun_out/pmck_$tag; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
g1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
g2="SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU"
for v in base ${VARIANTS}; do
  if [ "$v" = base ]; then lib=""; else lib=$repo/exp_libs/lib_$v.so; fi
  i=0
  for g in "$g1" "$g2"; do
    i=$((i+1))
    BJX_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $g --kernel-include-regex "${PMC_REGEX:-k_lines2}" -d "$out/${v}_p$i" -o pmc \
      --output-format csv -- python3 "$repo/tools/scan_stats.py" "$wl" "$n" 1 > "$out/${v}_p$i.log" 2>&1 || { echo "pass $v $i failed"; exit 1; }
  done
done
echo done
