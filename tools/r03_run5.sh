#!/bin/bash
# line_bench with the store-coalescing modes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03e}
mkdir -p $O
timeout -k 10 120 ./tools/line_bench 10 > $O/line.log 2>&1; echo "line exit $?"; cat $O/line.log
