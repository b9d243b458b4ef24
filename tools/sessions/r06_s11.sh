bash tools/gpu_session.sh \
 "bans|400|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bans.py tests/test_golden.py" \
 "emit|500|python tools/emit_bench.py cfg5 4 3" \
 "emtrace|500|cd /tmp && rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/em2_trace -o em --output-format csv -- python3 \$GRAFT_REPO_ROOT/tools/emit_bench.py cfg5 3 2"
