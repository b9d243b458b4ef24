tools/gpu_session.sh \
 "pytest_gpu|400|python -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120" \
 "prof|600|tools/prof_scan.sh cfg3v3 cfg3 10000000"
