#!/bin/bash
# default bench, tail bench (256 MiB and 1 GiB batches), node bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "bench|400|python bench.py --no-cpu-baseline" \
  "tail256|300|python tools/tail_bench.py cfg3 20000000 256 /tmp" \
  "tail1024|300|python tools/tail_bench.py cfg3 20000000 1024 /tmp" \
  "nodebench|400|python bench.py --node-engines 2 --steps 4 --warmup 2 --bans-steps 0 --no-cpu-baseline"
