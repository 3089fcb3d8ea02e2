#!/bin/bash
# Round 5: the asynchronous queue path's throughput against bundle sizing,
# slot count and per-thread depth, and a kernel trace of one point.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05b
mkdir -p $O
for cfg in "4096,8,6" "16384,24,4" "16384,24,8" "8192,12,8"; do
  for d in 64 256; do
    SYNC_AGG=$cfg SYNC_DEPTH=$d timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
    python3 -c "import json,sys; j=json.loads(open('$O/q.tmp').read()); j['agg']='$cfg'; j['depth']=$d; print(json.dumps(j))" >> $O/queue_sweep.jsonl
  done
done
SYNC_AGG=16384,24,8 SYNC_DEPTH=256 timeout -k 10 60 ./tools/sync_bench 2 queue 0 8 rt >> $O/queue_sweep.jsonl || exit $?
cd /tmp && export TMPDIR=/tmp
SYNC_AGG=4096,8,6 SYNC_DEPTH=64 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o q64 -- $GRAFT_REPO_ROOT/tools/sync_bench 1 queue 0 64 rt > $GRAFT_REPO_ROOT/$O/prof.log 2>&1
