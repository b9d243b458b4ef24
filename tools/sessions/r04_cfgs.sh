#!/bin/bash
# Round-4 other-config session: bench lines for cfg4, cfg5 (steady state),
# cfg5h, cfg2, then a kernel trace of --node-engines 2 (two engines of the
# node API on one GPU) and of two single-engine steps' worth (cfg3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-cfgs}; repo=$PWD
out=$repo/gpurun_out/$tag; mkdir -p "$out"
for c in ${CFGS:-cfg4 cfg5 cfg5h cfg2}; do
  w=1; case $c in cfg5|cfg5h) w=3;; esac
  timeout -k 10 400 python bench.py --config $c --steps 3 --warmup $w --bans-steps 0 --no-cpu-baseline > "$out/bench_$c.log" 2>&1 || exit $?
  echo "$c $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/bench_$c.log" | tr '\n' ' ')"
done
if [ -n "${NODE:-1}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/node" -o trace --output-format csv \
    -- python3 "$repo/bench.py" --node-engines 2 --steps 3 --warmup 1 --bans-steps 0 --no-cpu-baseline > "$out/node.log" 2>&1 || exit $?
  echo "node2 $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*' "$out/node.log" | tr '\n' ' ')"
fi
