bash tools/gpu_session.sh \
 "vt3|300|VARIANTS=\"prev nopj prof\" bash tools/variant_times.sh cfg3 20000000 3" \
 "vt5|300|VARIANTS=\"prev\" bash tools/variant_times.sh cfg5 20000000 3" \
 "par|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_golden.py tests/test_gpu_parity.py tests/test_gpu_plan_templates.py -k \"golden or workload_parity or lines2 or template or inline or lead or edge\""
