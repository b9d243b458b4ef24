#!/bin/bash
# node rehearsal: the two-level grouping forced (BJX_SORT2=2) against the default gate
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/sort2g
mkdir -p $o
BJX_SORT2=2 timeout -k 10 400 python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline > $o/b2_node2.log 2>&1 || { echo "node forced failed"; tail -5 $o/b2_node2.log; exit 1; }
python3 tools/bench_summary.py $o/b2_node2.log
grep -o '"grouping": [0-9]*\|"states": [0-9]*\|"state_table_slots": [0-9]*' $o/b2_node2.log || true
