bash tools/gpu_session.sh \
 "vt|400|VARIANTS=\"r5 nouni prof\" bash tools/variant_times.sh cfg3 20000000 3" \
 "par|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_plan_templates.py -k \"golden or workload_parity or lines2 or tile_geometry or short_line or edge or template or inline or lead\"" \
 "sb|300|python tools/small_batch.py cfg3 1700000 12" \
 "sbtrace|300|cd /tmp && rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/sb_trace -o sb --output-format csv -- python3 \$GRAFT_REPO_ROOT/tools/small_batch.py cfg3 1700000 6" \
 "c5bans|400|cd /tmp && rocprofv3 --kernel-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/c5_trace -o c5 --output-format csv -- python3 \$GRAFT_REPO_ROOT/bench.py --config cfg5 --bans 1 --steps 2 --warmup 1 --bans-steps 0 --no-cpu-baseline"
