#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu_session.sh \
  "scan_tests|500|python -u -m pytest tests/test_golden.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread" \
  "abl_cfg3|400|CFG=cfg3 LINES=20000000 tools/scan_ablation.sh" \
  "abl_cfg4|400|CFG=cfg4 LINES=2000000 tools/scan_ablation.sh" \
  "pmc|600|tools/r05_pmc_scan.sh scan1"
