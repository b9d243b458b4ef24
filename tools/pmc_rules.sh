set -e
cd "${GRAFT_REPO_ROOT}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=$PWD/gpurun_out/pmc_rules; mkdir -p $out; repo=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_BUSY_CYCLES" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "k_rules|k_scan" -d $out/p$i -o pmc --output-format csv -- python3 $repo/bench.py --steps 2 --warmup 0 --no-cpu-baseline > $out/p$i.log 2>&1
done
