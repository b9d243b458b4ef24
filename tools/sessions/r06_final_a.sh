#!/bin/bash
# Round-6 closing evidence, part A: GPU suite, smoke, the driver's bench command
# (with the CPU baselines), a kernel trace of the default bench, the PMC passes
# behind profiles/pmc_traffic.json.  Logs under gpurun_out/ (copied to profiles/r06_final).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "suite|800|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg3|500|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "trace_cfg3|400|CFGS=cfg3 bash tools/trace_bench.sh" \
  "pmc_cfg3|700|bash tools/pmc_session.sh r06"
