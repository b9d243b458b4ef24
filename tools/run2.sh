tools/gpu_session.sh "pytest_gpu|400|python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120" 
for k in 0 1; do echo "skip=$k"; BJX_DEBUG_SKIP=$k timeout -k 10 120 python tools/scan_stats.py cfg3 20000000 2 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['scan_ms'], d['phases'], d['stats'])"; done
for w in cfg2 cfg4 cfg5; do timeout -k 10 120 python tools/scan_stats.py $w 10000000 2 2>&1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['workload'], d['scan_ms'], d['phases'], d['stats'])"; done
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
