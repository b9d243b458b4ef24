#!/bin/bash
# every config's bench line on the current tree, then the k_scan / k_lines2 PMC passes (cfg3, cfg4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "b_cfg1|300|python bench.py --config cfg1 --no-cpu-baseline" \
  "b_cfg4|300|python bench.py --config cfg4 --no-cpu-baseline" \
  "b_cfg5h|400|python bench.py --config cfg5h --no-cpu-baseline --warmup 3" \
  "pmc_scan|600|bash tools/r05_pmc_scan.sh scan5"
