#!/bin/bash
# Round-3 measurement pass on one GPU: the deployment paths (aggregator
# throughput, in-process 8-GPU and 2-rank rehearsals on device 0), the skewed
# and stream-count bench points, then the profile evidence (tools/r03_prof.sh).
# Test failures continue; a crash or time limit (exit >= 124) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03b}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -3 $O/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
t agg_bench 240 ./tools/agg_bench 2
SRTP_BENCH_ONE_DEVICE=1 t bench_inproc8 600 python bench.py --gpus 8 --steps 10 --no-cpu --e2e-bundles 6 --dispatch-bundles 4
SRTP_BENCH_ONE_DEVICE=1 t bench_2rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --no-cpu --backend gloo --e2e-bundles 8
t bench_zipf 300 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --zipf 1.1
t bench_one 300 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --ssrcs 1
t bench_100k 300 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --ssrcs 100000
t bench_steps20 300 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch
R03_TAG=${R03_TAG:-r03b}/prof ./tools/r03_prof.sh
echo done
