#!/bin/bash
# Round 6: table counters read with the match phase's last counts and with the
# state claims' flags (three fewer host syncs per batch).  GPU suite, small
# batches A/B against the previous commit's library, cfg3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "suite|900|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests" \
  "sb_new|200|python3 tools/small_batch.py cfg3 1700000 12" \
  "sb_prev|200|BJX_LIB_PATH=exp_libs/lib_prev.so python3 tools/small_batch.py cfg3 1700000 12" \
  "sb_new2|200|python3 tools/small_batch.py cfg3 1700000 12" \
  "bench_cfg3|300|python3 bench.py --no-cpu-baseline --bans-steps 0"
