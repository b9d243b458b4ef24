#!/bin/bash
# PMC passes over k_scan alone (tools/scan_stats.py, cfg3 20M lines and cfg4 2M
# lines, one batch each after a warm-up batch): one counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
tag=${1:-scan}
out=$repo/gpurun_out/pmc_$tag; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
  "SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
for cfg in ${CFGS:-cfg3 cfg4}; do
  n=20000000; [ $cfg = cfg4 ] && n=2000000
  i=0
  for g in "${groups[@]}"; do
    i=$((i+1))
    echo "$cfg pass $i: $g"
    timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "${PMC_REGEX:-k_scan|k_lines2}" -d "$out/${cfg}_p$i" -o pmc --output-format csv \
      -- python3 "$repo/tools/scan_stats.py" $cfg $n 2 > "$out/${cfg}_p$i.log" 2>&1 || { echo "pass failed rc=$?"; exit 1; }
  done
done
echo done
