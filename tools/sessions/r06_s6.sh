bash tools/gpu_session.sh \
 "vt3|300|VARIANTS=\"prev\" bash tools/variant_times.sh cfg3 20000000 3" \
 "vt2|300|VARIANTS=\"prev\" bash tools/variant_times.sh cfg2 20000000 3" \
 "par|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden.py tests/test_gpu_parity.py -k \"golden or workload_parity or tile_geometry or short_line or overflow_hits or edge or regex_corpus or bounded_lead\"" \
 "emit|500|python tools/emit_bench.py cfg5 4 3" \
 "emtrace|500|cd /tmp && rocprofv3 --kernel-trace --memory-copy-trace --stats -d \$GRAFT_REPO_ROOT/gpurun_out/em_trace -o em --output-format csv -- python3 \$GRAFT_REPO_ROOT/tools/emit_bench.py cfg5 3 2"
