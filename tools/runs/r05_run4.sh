#!/bin/bash
# Round 5: per-packet GPU tests, then the aggregator with and without the
# pipelined second bundle (libjitsi_amd/variants/nopipe: SRTP_AGG_PIPE=1), A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5TAG:-r05d}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_jni_shim.py \
  tests/test_aggregator.py tests/test_single_packet.py tests/test_rawpacket.py tests/test_pipeline.py > $O/tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for rep in 1 2; do
  for v in default nopipe; do
    if [ $v = nopipe ]; then export LD_LIBRARY_PATH=$PWD/libjitsi_amd/variants/nopipe; else unset LD_LIBRARY_PATH; fi
    for cfg in "4096,8,6 64" "16384,24,8 256"; do
      set -- $cfg
      SYNC_AGG=$1 SYNC_DEPTH=$2 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
      python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['agg']='$1'; j['depth']=$2; j['lib']='$v'; print(json.dumps(j))" >> $O/sync.jsonl
    done
    timeout -k 10 60 ./tools/sync_bench 2 one 0 64 rt > $O/q.tmp || exit $?
    python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['lib']='$v'; print(json.dumps(j))" >> $O/sync.jsonl
    timeout -k 10 120 ./tools/agg_bench > $O/agg_$v.$rep.log 2>&1 || exit $?
  done
done
unset LD_LIBRARY_PATH
