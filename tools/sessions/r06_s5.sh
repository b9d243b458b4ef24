bash tools/gpu_session.sh \
 "sb|300|python tools/small_batch.py cfg3 1700000 12" \
 "vt|400|VARIANTS=\"prof\" bash tools/variant_times.sh cfg3 20000000 3" \
 "abl3|400|CFG=cfg3 bash tools/scan_ablation.sh" \
 "abl2|400|CFG=cfg2 bash tools/scan_ablation.sh" \
 "c5|600|python3 bench.py --config cfg5 --warmup 4 --steps 3 --bans-steps 2 --no-cpu-baseline" \
 "suite|900|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu"
