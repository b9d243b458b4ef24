#!/bin/bash
# Round-5 closing evidence on one box: GPU suite, smoke, the default bench
# (with the CPU baselines), every config's bench line, the 2-engine node
# rehearsal, a kernel trace of the default bench and the PMC passes behind
# profiles/pmc_traffic.json.  Logs under gpurun_out/ (copied to profiles/r05_final).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "suite|800|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg3|500|python bench.py" \
  "bench_cfg1|300|python bench.py --config cfg1 --no-cpu-baseline" \
  "bench_cfg2|300|python bench.py --config cfg2 --no-cpu-baseline" \
  "bench_cfg4|300|python bench.py --config cfg4 --no-cpu-baseline" \
  "bench_cfg5|400|python bench.py --config cfg5 --no-cpu-baseline --warmup 3" \
  "bench_cfg5h|400|python bench.py --config cfg5h --no-cpu-baseline --warmup 3" \
  "bench_node2|400|python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline" \
  "trace_cfg3|400|CFGS=cfg3 tools/r05_trace.sh" \
  "pmc_cfg3|700|bash tools/pmc_session.sh r05"
