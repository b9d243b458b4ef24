#!/bin/bash
# Round 6: the wide per-line kernel parses with 16-B loads (find_spaces) and
# starts a lead rule's automaton at the first hit of its literals.  Wide-scope
# and fallback parity tests, then cfg2k times against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "wide_tests|600|python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests -k 'wide or stress or slow or exotic or timestamp or fallback or edge or corpus or golden'" \
  "vt2k|400|VARIANTS='prev' bash tools/variant_times.sh cfg2k 20000000 3"
