#!/bin/bash
# Round-4 closing session: the whole GPU suite, smoke, the default bench line
# (with the CPU baselines), and a kernel trace of the cfg3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
repo=$PWD
exec_steps=(
  "final_suite|600|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
  "final_smoke|180|python -c 'import __graft_entry__ as g; g.smoke()'"
  "final_bench|400|python bench.py"
  "final_trace|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -d $repo/gpurun_out/final_trace -o trace --output-format csv -- python3 $repo/bench.py --steps 3 --warmup 2 --bans-steps 0 --no-cpu-baseline"
)
tools/gpu_session.sh "${exec_steps[@]}"
