#!/bin/bash
# Round-6 closing evidence, part C (after the last code changes; part A's suite,
# smoke, trace and PMC passes ran on the same library): the driver's bench
# command again (emission warmed over as many steps as the plain run), every
# other config's bench line, the node rehearsal, the 1,000-global-rule shape,
# emission per step at cfg5, small batches and the tail-inclusive rate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "bench_cfg3|500|python3 bench.py --gpus 1 --steps 20 --warmup 5" \
  "bench_cfg1|300|python3 bench.py --config cfg1 --no-cpu-baseline" \
  "bench_cfg2|300|python3 bench.py --config cfg2 --no-cpu-baseline" \
  "bench_cfg4|300|python3 bench.py --config cfg4 --no-cpu-baseline" \
  "bench_cfg5|400|python3 bench.py --config cfg5 --no-cpu-baseline --warmup 3" \
  "bench_cfg5h|400|python3 bench.py --config cfg5h --no-cpu-baseline --warmup 3" \
  "bench_cfg2k|400|python3 bench.py --config cfg2k --no-cpu-baseline --bans-steps 0" \
  "bench_node2|400|python3 bench.py --node-engines 2 --steps 4 --warmup 3 --bans-steps 0 --no-cpu-baseline" \
  "emit_cfg5|400|python3 tools/emit_bench.py cfg5 4 6" \
  "small_batch|300|python3 tools/small_batch.py cfg3 1700000 12" \
  "tail|500|python3 tools/tail_bench.py cfg3 20000000 256 /tmp 2"
