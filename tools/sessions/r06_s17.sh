#!/bin/bash
# Round 6: ban log written in chunks with its D2H on a side stream (emission
# tests, cfg5 emission per step, cfg5/cfg3 bench lines) and the cfg2 k_scan
# SQ counter passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "bans_tests|300|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bans.py" \
  "emit_cfg5|400|python3 tools/emit_bench.py cfg5 4 6" \
  "bench_cfg5|400|python3 bench.py --config cfg5 --no-cpu-baseline --warmup 3" \
  "bench_cfg3|400|python3 bench.py --no-cpu-baseline" \
  "pmc_cfg2_scan|300|PMC_REGEX=k_scan tools/pmc_kernel.sh cfg2scan cfg2 20000000"
