#!/bin/bash
# Round 5: the queued per-packet path (sync_bench queue) against the library
# before the dispatcher-depth commit (old5c8) and with the packed-copy limit
# back at 8192 (kpack13), alternating on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05q
mkdir -p $O
: > $O/q.jsonl
for rep in 1 2 3; do
  for v in cur kpack13 old5c8; do
    for cfg in "16384,24,8 256" "4096,8,6 64"; do
      set -- $cfg
      if [ $v = cur ]; then LP=; else LP=$PWD/libjitsi_amd/variants/$v; fi
      LD_LIBRARY_PATH=$LP SYNC_AGG=$1 SYNC_DEPTH=$2 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
      python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); print(json.dumps({'lib': '$v', 'agg': '$1', 'depth': $2, 'calls_per_s': j['calls_per_s'], 'p50': j['lat_us']['p50'], 'p99': j['lat_us'].get('p99')}))" | tee -a $O/q.jsonl
    done
  done
done
