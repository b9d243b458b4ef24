bash tools/gpu_session.sh \
 "vt3|300|VARIANTS=\"wpe3\" bash tools/variant_times.sh cfg3 20000000 3" \
 "vt2|300|VARIANTS=\"wpe3\" bash tools/variant_times.sh cfg2 20000000 3" \
 "vt4|300|VARIANTS=\"wpe3\" bash tools/variant_times.sh cfg4 2000000 3"
