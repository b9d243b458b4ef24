#!/bin/bash
# inline automata for every small rule (BJX_INLINE_ALL) vs anchored only: jobs and kernel times
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 1; do
  for c in cfg3 cfg4; do
    n=20000000; [ $c = cfg4 ] && n=2000000
    if [ $v = 1 ]; then export BJX_INLINE_ALL=1; else unset BJX_INLINE_ALL; fi
    echo "== inline_all=$v $c"
    timeout -k 10 200 python tools/scan_stats.py $c $n 3 2>&1 | grep '^{' | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['phases']['resolve'], d['kernel_ms'], d['stats']['dfa_jobs'])" || exit 1
  done
done
