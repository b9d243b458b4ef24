#!/bin/bash
# tail bench: slots and batch size
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "tail256s2|300|python tools/tail_bench.py cfg3 20000000 256 /tmp 2" \
  "tail256s3|300|python tools/tail_bench.py cfg3 20000000 256 /tmp 3" \
  "tail128s4|300|python tools/tail_bench.py cfg3 20000000 128 /tmp 4" \
  "tail512s3|300|python tools/tail_bench.py cfg3 20000000 512 /tmp 3" \
  "tailtest|300|python -u -m pytest tests/test_tailer.py -x -q --timeout 200 --timeout-method thread"
