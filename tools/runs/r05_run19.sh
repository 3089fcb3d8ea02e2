#!/bin/bash
# Round 5: dispatcher pipeline depth -- 8 slots of 32768 packets (default) vs
# 16 slots of 16384 (libjitsi_amd/variants/libsrtp_d16.so), dispatcher leg
# at 1 and 2 shards, twice each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05s}
O=gpurun_out/$T
mkdir -p $O
for r in 1 2; do
  for lib in default libjitsi_amd/variants/libsrtp_d16.so; do
    if [ "$lib" = default ]; then unset SRTP_MI355X_LIB; else export SRTP_MI355X_LIB=$PWD/$lib; fi
    timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --no-e2e --dispatch-shards 1 > $O/b.log 2>&1 || exit $?
    tail -1 $O/b.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); [print('$lib'.split('/')[-1], k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle']['wait_ms']) for k,v in j['dispatch'].items()]"
  done
done
unset SRTP_MI355X_LIB
