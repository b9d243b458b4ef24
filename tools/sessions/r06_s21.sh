#!/bin/bash
# Round 6: wide-scope fallback takes the fast timestamp parse first.  Wide-scope
# parity tests, then cfg2k times: base, the previous commit's library, and a
# timing-only variant without decide_wide (the fallback's parse alone).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "wide_tests|600|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k 'wide or stress or slow or exotic or timestamp'" \
  "vt2k|600|VARIANTS='prev nodec' bash tools/variant_times.sh cfg2k 20000000 3"
