#!/bin/bash
# Round 6: cfg3 emission per step (where the trip bursts fall and what they cost
# with the full log, first time and again).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "emit_cfg3|400|python3 tools/emit_bench.py cfg3 2 36"
