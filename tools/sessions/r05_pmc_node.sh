#!/bin/bash
# PMC passes over the exchange kernels of the one-GPU 2-engine node bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PASSES="1 2 3 4" PMC_REGEX="k_pack|k_part_count|k_unpack_lines|k_ip_claim|k_st_claim" bash tools/pmc_session.sh node --node-engines 2
