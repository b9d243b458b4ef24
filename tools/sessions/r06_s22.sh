#!/bin/bash
# Round 6: per-line masks word-major (word w of line j at w * stride + j).
# GPU suite, then cfg2k / cfg2 / cfg3 times against the previous commit's library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "suite|900|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "vt2k|400|VARIANTS='prev' bash tools/variant_times.sh cfg2k 20000000 3" \
  "vt2|400|VARIANTS='prev' bash tools/variant_times.sh cfg2 20000000 3" \
  "bench_cfg3|300|python3 bench.py --no-cpu-baseline --bans-steps 0"
