bash tools/gpu_session.sh \
 "b3|300|python3 bench.py --steps 10 --warmup 5 --bans-steps 0 --no-cpu-baseline" \
 "b3ns|300|BJX_NO_SHRINK=1 python3 bench.py --steps 10 --warmup 5 --bans-steps 0 --no-cpu-baseline" \
 "b5|300|python3 bench.py --config cfg5 --steps 6 --warmup 5 --bans-steps 0 --no-cpu-baseline" \
 "b5ns|300|BJX_NO_SHRINK=1 python3 bench.py --config cfg5 --steps 6 --warmup 5 --bans-steps 0 --no-cpu-baseline" \
 "tst|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_state_growth.py tests/test_gpu_hotkey.py tests/test_gpu_parity.py -k \"growth or rollback or hot_key or two_level or workload\""
