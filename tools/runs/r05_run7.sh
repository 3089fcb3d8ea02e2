#!/bin/bash
# Round 5: the JNI queue test, and the aggregator's callback path over a
# one-shard dispatcher with and without the pipelined second bundle, A/B x3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5TAG:-r05g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu tests/test_jni_shim.py > $O/tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for rep in 1 2 3; do
  for v in default nopipe; do
    if [ $v = nopipe ]; then export LD_LIBRARY_PATH=$PWD/libjitsi_amd/variants/nopipe; else unset LD_LIBRARY_PATH; fi
    for sh in 0 1; do
      timeout -k 10 60 ./tools/agg_bench 2 0 $sh 16 > $O/a.tmp 2>&1 || exit $?
      python3 -c "import json; j=json.loads([l for l in open('$O/a.tmp') if l.startswith('{')][0]); j['lib']='$v'; print(json.dumps(j))" >> $O/agg.jsonl
    done
    SYNC_AGG=16384,24,8 SYNC_DEPTH=256 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
    python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['lib']='$v'; print(json.dumps(j))" >> $O/agg.jsonl
  done
done
unset LD_LIBRARY_PATH
