#!/bin/bash
# Round-4 PMC session: k_lines2 LDS sizing (BJX_DEBUG_IMG), then the four PMC
# passes of tools/pmc_session.sh over the default cfg3 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
tag=${1:-r04p}
mkdir -p gpurun_out/pmc_$tag
BJX_DEBUG_IMG=1 timeout -k 10 120 python tools/scan_stats.py cfg3 2000000 1 > gpurun_out/pmc_$tag/img.log 2>&1 || exit $?
grep "k_lines2" gpurun_out/pmc_$tag/img.log | head -3
bash tools/pmc_session.sh $tag
