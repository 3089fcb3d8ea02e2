#!/bin/bash
# Round-3 GPU pass 2: the tests that failed in pass 1 (fixed), 1M streams over
# 8 shards, then the deployment paths (aggregator throughput, in-process
# 8-GPU and 2-rank rehearsals on device 0), the skewed and stream-count bench
# points and the split AES-CM / HMAC micro-benchmark.  Test failures continue;
# a crash or time limit (exit >= 124) ends the script.
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
PT="python -u -m pytest --timeout 200 --timeout-method thread -p no:cacheprovider"
t fixed 200 $PT -v tests/test_aggregator.py tests/test_lifecycle.py -m gpu
t c5 300 $PT -x -v -s tests/test_config5_sharded.py --timeout 280
t agg_bench 120 ./tools/agg_bench 2
SRTP_BENCH_ONE_DEVICE=1 t bench_inproc8 150 python bench.py --gpus 8 --steps 10 --no-cpu --e2e-bundles 6 --dispatch-bundles 4
SRTP_BENCH_ONE_DEVICE=1 t bench_2rank 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --no-cpu --backend gloo --e2e-bundles 8
t bench_zipf 90 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --zipf 1.1
t bench_one 90 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --ssrcs 1
t bench_100k 90 python bench.py --steps 20 --no-cpu --no-e2e --no-dispatch --ssrcs 100000
t split 90 ./tools/split_bench 20
echo done
