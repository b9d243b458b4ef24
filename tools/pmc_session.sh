#!/bin/bash
# rocprofv3 PMC passes over the default cfg3 bench for every engine kernel
# (k_*): one counter group per run, within gfx950's per-pass slots (8 SQ,
# 4 TCC: FETCH_SIZE costs 3, WRITE_SIZE 2).  Output: gpurun_out/pmc_<tag>/p<i>/
#   bash tools/pmc_session.sh <tag> [bench args...]
# env: PASSES="1 2" (subset of the groups), PMC_REGEX (kernel filter, default k_)
set -e
tag=${1:-cur}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
repo=$PWD
out=$repo/gpurun_out/pmc_$tag; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
groups=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
  "SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VALU"
  "FETCH_SIZE"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
)
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4} " in *" $i "*) ;; *) continue;; esac
  echo "pass $i: $g"
  timeout -s KILL 150 rocprofv3 --pmc $g --kernel-include-regex "${PMC_REGEX:-k_}" -d "$out/p$i" -o pmc --output-format csv \
    -- python3 "$repo/bench.py" --steps 2 --warmup 1 --bans-steps 0 --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
done
echo done
