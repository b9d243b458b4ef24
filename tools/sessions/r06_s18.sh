#!/bin/bash
# Round 6: k_bucket_apply sorts (low key << 12 | position) words without a
# value array; its tests, then cfg3 bench A/B against the previous commit's
# library (exp_libs/lib_prev.so), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "grouping_tests|400|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_hotkey.py tests/test_gpu_parity.py -k 'two_level or hot_key or rollback or record_forms or workload'" \
  "ab_new1|300|python3 bench.py --no-cpu-baseline --bans-steps 0 --steps 10" \
  "ab_prev1|300|BJX_LIB_PATH=exp_libs/lib_prev.so python3 bench.py --no-cpu-baseline --bans-steps 0 --steps 10" \
  "ab_new2|300|python3 bench.py --no-cpu-baseline --bans-steps 0 --steps 10" \
  "ab_prev2|300|BJX_LIB_PATH=exp_libs/lib_prev.so python3 bench.py --no-cpu-baseline --bans-steps 0 --steps 10"
