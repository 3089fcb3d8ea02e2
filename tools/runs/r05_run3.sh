#!/bin/bash
# Round 5: pipelined aggregator lanes (two bundles in flight): the per-packet
# GPU tests, then sync_bench's queue / one / arrayq points and agg_bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5TAG:-r05c}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_jni_shim.py \
  tests/test_aggregator.py tests/test_single_packet.py tests/test_rawpacket.py tests/test_pipeline.py > $O/tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for cfg in "4096,8,6 64" "4096,8,6 256" "16384,24,8 256"; do
  set -- $cfg
  SYNC_AGG=$1 SYNC_DEPTH=$2 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
  python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['agg']='$1'; j['depth']=$2; print(json.dumps(j))" >> $O/sync.jsonl
done
SYNC_AGG=4096,8,6 SYNC_DEPTH=256 timeout -k 10 60 ./tools/sync_bench 2 queue 0 8 rt >> $O/sync.jsonl || exit $?
for p in "one 0 1 rt" "one 0 64 rt" "arrayq 0 8" "arrayq 8 8" "arrayq 0 64"; do
  timeout -k 10 60 ./tools/sync_bench 2 $p >> $O/sync.jsonl || exit $?
done
timeout -k 10 120 ./tools/agg_bench > $O/agg_bench.log 2>&1 || exit $?
