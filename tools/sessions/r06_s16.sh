bash tools/gpu_session.sh \
 "wide|600|python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k \"stress or wide_scope or fallback or consume_line\"" \
 "b2k|400|python3 bench.py --config cfg2k --no-cpu-baseline --bans-steps 0"
