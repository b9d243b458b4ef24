#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# fault-like exit status (timeout, abort, segfault, kill).  Test failures
# (pytest exit 1) do not stop later steps.
# usage: tools/gpu_session.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc in $(( $(date +%s) - start )) s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139|143) echo "fault-like exit $rc: stopping"; exit $rc;;
  esac
done
