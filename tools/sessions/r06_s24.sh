#!/bin/bash
# Round 6: where the wide per-line kernel's time goes (cfg2k): timing-only
# variants without automaton runs, without literal hits, without decide_wide;
# SQ counter passes of k_parse_match.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tools/gpu_session.sh \
  "vt2k|400|VARIANTS='noeval nohits nodec' bash tools/variant_times.sh cfg2k 20000000 3" \
  "pmc_wide|300|PMC_REGEX=k_parse_match tools/pmc_kernel.sh wide cfg2k 20000000"
