#!/bin/bash
# Round 6: rulesets whose every scope is past 128 positions skip the line pass
# (the wide per-line kernel takes every line).  GPU suite, cfg2k times against
# the previous commit's library, the cfg2k bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "suite|900|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "vt2k|400|VARIANTS='prev' bash tools/variant_times.sh cfg2k 20000000 3" \
  "bench_cfg2k|400|python3 bench.py --config cfg2k --no-cpu-baseline --bans-steps 0"
