#!/bin/bash
# Round 6: fewer host syncs per batch (job count read with the line-pass
# counters; IP-claim flags, table counters and collision count in one read).
# Parity tests, then small batches A/B against the previous commit's library
# and a kernel trace of the new one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "parity|600|python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_hotkey.py" \
  "sb_new|200|python3 tools/small_batch.py cfg3 1700000 12" \
  "sb_prev|200|BJX_LIB_PATH=exp_libs/lib_prev.so python3 tools/small_batch.py cfg3 1700000 12" \
  "sb_new2|200|python3 tools/small_batch.py cfg3 1700000 12" \
  "sb_trace|300|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/sb6 -o sb --output-format csv -- python3 \$GRAFT_REPO_ROOT/tools/small_batch.py cfg3 1700000 6"
