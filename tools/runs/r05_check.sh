#!/bin/bash
# Round 5 checkpoint on one GPU: the whole GPU suite, smoke, the default bench
# as the driver runs it, and the per-packet / aggregator benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5TAG:-r05chk}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || exit $?
for p in "one 0 1 rt" "one 0 64 rt" "arrayq 0 64" "arrayq 8 8" "array 8 8"; do
  timeout -k 10 60 ./tools/sync_bench 2 $p >> $O/sync.jsonl || exit $?
done
for cfg in "4096,8,6 64" "16384,24,8 256"; do
  set -- $cfg
  SYNC_AGG=$1 SYNC_DEPTH=$2 timeout -k 10 60 ./tools/sync_bench 2 queue 0 64 rt > $O/q.tmp || exit $?
  python3 -c "import json; j=json.loads(open('$O/q.tmp').read()); j['agg']='$1'; j['depth']=$2; print(json.dumps(j))" >> $O/sync.jsonl
done
timeout -k 10 120 ./tools/agg_bench > $O/agg_bench.log 2>&1 || exit $?
# the dispatcher leg (1 shard; the asynchronous mode's per-operation times)
timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --no-e2e --dispatch-shards 1 > $O/bench_dispatch.log 2>&1 || exit $?
# --gpus 8 without torchrun: one process per side, all on device 0 (gloo)
timeout -k 10 300 env SRTP_BENCH_ONE_DEVICE=1 python bench.py --gpus 8 --backend gloo --steps 20 --no-cpu --no-e2e --no-dispatch > $O/rehearsal8.log 2>&1 || exit $?
