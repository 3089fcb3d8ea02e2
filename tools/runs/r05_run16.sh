#!/bin/bash
# Round 5: where the dispatcher leg's time goes -- kernel + memory-copy trace
# of the 1-shard dispatcher leg (sync and async modes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05p}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/dtrace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --dispatch-shards 1 --dispatch-bundles 4 > $O/dtrace.log 2>&1 || exit $?
ls $O/dtrace
