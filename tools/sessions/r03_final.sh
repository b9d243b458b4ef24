#!/bin/bash
# Round-3 closing measurements: GPU suite, default bench (cfg3 + CPU
# baselines), kernel trace, PMC passes over the default bench, other configs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "suite|500|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "bench|300|python -u bench.py" \
  "trace|300|tools/prof_bench.sh r03f --steps 5 --warmup 2 --no-cpu-baseline" \
  "pmc|700|bash tools/pmc_session.sh r03f" \
  "cfg4|200|python -u bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline" \
  "cfg2|200|python -u bench.py --config cfg2 --steps 5 --warmup 2 --no-cpu-baseline" \
  "cfg1|200|python -u bench.py --config cfg1 --steps 10 --warmup 2 --no-cpu-baseline" \
  "cfg5|250|python -u bench.py --config cfg5 --steps 3 --warmup 3 --no-cpu-baseline" \
  "cfg5h|250|python -u bench.py --config cfg5h --steps 3 --warmup 2 --no-cpu-baseline"
