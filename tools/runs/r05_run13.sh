#!/bin/bash
# Round 5: asynchronous dispatcher host bundles -- the bench's dispatcher leg
# (1 shard: sync / async / copy / registered; then 2 shards), and the
# dispatcher tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05m}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_dispatch_async.py tests/test_dispatcher.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for sh in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --no-cpu --no-e2e --dispatch-shards $sh > $O/bench_dispatch_$sh.log 2>&1 || exit $?
  tail -1 $O/bench_dispatch_$sh.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value']/1e6); [print(k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle'], v['all_accepted']) for k,v in j['dispatch'].items()]"
done
