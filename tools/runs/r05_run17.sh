#!/bin/bash
# Round 5: packed per-packet copies for chunk-sized pipeline bundles --
# pipeline / aggregator / dispatcher tests, the dispatcher leg (1 and 2
# shards), sync_bench queue and agg_bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05q}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline.py tests/test_aggregator.py tests/test_dispatch_async.py tests/test_dispatcher.py tests/test_rawpacket.py tests/test_single_packet.py tests/test_jni_shim.py tests/test_small_bundles.py tests/test_host_memory.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for sh in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --dispatch-shards $sh > $O/bench_dispatch_$sh.log 2>&1 || exit $?
  tail -1 $O/bench_dispatch_$sh.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); e=j.get('e2e') or {}; print('e2e', e.get('directional_pps'), e.get('pcie_gbps_h2d_plus_d2h')); [print(k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle'], v['all_accepted']) for k,v in j['dispatch'].items()]"
done
SYNC_AGG=16384,24,8 SYNC_DEPTH=256 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/sync_queue.jsonl || exit $?
cat $O/sync_queue.jsonl
timeout -k 10 120 ./tools/agg_bench > $O/agg_bench.log 2>&1 || exit $?
tail -4 $O/agg_bench.log
