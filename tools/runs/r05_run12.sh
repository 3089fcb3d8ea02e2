#!/bin/bash
# Round 5: the look-back second sort pass (batched retries) and asynchronous
# dispatcher host bundles -- parity subset + dispatcher tests, A/B against the
# HEAD build, and the bench's dispatcher leg (1 shard: sync / async / copy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05l}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_dispatch_async.py tests/test_dispatcher.py tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_config5_sharded.py > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --steps 20 --no-cpu --no-e2e --dispatch-shards 1 > $O/bench_dispatch.log 2>&1 || exit $?
tail -1 $O/bench_dispatch.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print(j['value']/1e6); [print(k, v['directional_pps']/1e6, v['ms_per_bundle'], v['host_ms_per_bundle'], v['all_accepted']) for k,v in j['dispatch'].items()]"
