bash tools/gpu_session.sh \
 "b3|300|python3 bench.py --steps 6 --warmup 4 --bans-steps 0 --no-cpu-baseline" \
 "b3nosort|300|BJX_LIB_PATH=\$GRAFT_REPO_ROOT/exp_libs/lib_nosort.so python3 bench.py --steps 6 --warmup 4 --bans-steps 0 --no-cpu-baseline"
