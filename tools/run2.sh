tools/gpu_session.sh \
 "stats|400|python tools/scan_stats.py cfg3 20000000 3 && python tools/scan_stats.py cfg2 20000000 2 && python tools/scan_stats.py cfg4 2000000 2 && python tools/scan_stats.py cfg5 20000000 2 && python tools/scan_stats.py cfg1 1000000 2" \
 "bench_full|500|python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
