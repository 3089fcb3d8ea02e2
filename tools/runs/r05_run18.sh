#!/bin/bash
# Round 5: dispatcher pipeline depth 8 (experiment) -- the dispatcher leg
# (1 shard) and a copy trace of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05r}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --no-e2e --dispatch-shards 1 > $O/bench_dispatch_1.log 2>&1 || exit $?
tail -1 $O/bench_dispatch_1.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); [print(k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle'], v['all_accepted']) for k,v in j['dispatch'].items()]"
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/dtrace -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --dispatch-shards 1 --dispatch-bundles 4 > $O/dtrace.log 2>&1 || exit $?
