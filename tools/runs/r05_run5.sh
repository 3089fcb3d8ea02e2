#!/bin/bash
# Round 5: the queue test, then kernel + copy traces of the aggregator's
# bundles with and without the pipelined second bundle, and bundle sizing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/${R5TAG:-r05e}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -s --timeout 120 --timeout-method thread -m gpu tests/test_jni_shim.py > $O/tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
for cfg in "8192,12,8 64" "8192,12,8 256" "16384,24,8 128"; do
  set -- $cfg
  SYNC_AGG=$1 SYNC_DEPTH=$2 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
  python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['agg']='$1'; j['depth']=$2; print(json.dumps(j))" >> $O/sync.jsonl
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/agg_pipe -o t -- $R/tools/agg_bench 1 0 1 16 > $R/$O/agg_pipe.log 2>&1 || exit $?
LD_LIBRARY_PATH=$R/libjitsi_amd/variants/nopipe timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/agg_nopipe -o t -- $R/tools/agg_bench 1 0 1 16 > $R/$O/agg_nopipe.log 2>&1 || exit $?
SYNC_AGG=16384,24,8 SYNC_DEPTH=256 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/$O/queue -o t -- $R/tools/sync_bench 1 queue 0 64 rt > $R/$O/queue.log 2>&1 || exit $?
