#!/bin/bash
# GPU session: new GPU tests, the default bench (cfg3) with CPU baselines and the
# decision-emission figure, then cfg1 / cfg5 / cfg5h bench lines.  Each step has
# its own time limit; the first failure ends the session.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
o=gpurun_out/r02s; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_state_growth.py tests/test_gpu_hotkey.py -x -v --timeout 300 --timeout-method thread > $o/tests.log 2>&1
timeout -k 10 300 python -u bench.py > $o/bench_cfg3.json 2> $o/bench_cfg3.err
timeout -k 10 200 python -u bench.py --config cfg1 --steps 10 --warmup 2 > $o/bench_cfg1.json 2> $o/bench_cfg1.err
timeout -k 10 300 python -u bench.py --config cfg5 --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_cfg5.json 2> $o/bench_cfg5.err
timeout -k 10 300 python -u bench.py --config cfg5h --steps 3 --warmup 1 --no-cpu-baseline > $o/bench_cfg5h.json 2> $o/bench_cfg5h.err
echo session-ok
