#!/bin/bash
# Round-end evidence of the committed tree: the GPU suite, smoke, the bench
# line as the driver runs it and at the default step count, every BASELINE
# config, mixed key sets, the per-packet path (sync_bench) and aggregator
# throughput, then the profile passes (tools/prof.sh: kernel traces, PMC,
# calibration, timeline).  TAG names the gpurun_out/ subdirectory.
# A crash or time limit (exit >= 124) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -2 $O/$name.log | cut -c1-400
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
t gpu 300 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu
t smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
t bench20 180 python bench.py --gpus 1 --steps 20 --warmup 5
t bench100 180 python bench.py
t configs 300 python -u tools/config_bench.py --out $O/configs.json
t keysets16 180 python bench.py --steps 20 --keysets 16 --no-cpu --no-e2e --no-dispatch
t keysets1000 180 python bench.py --steps 20 --keysets 1000 --no-cpu --no-e2e --no-dispatch
t ssrcs100k 180 python bench.py --steps 20 --ssrcs 100000 --no-cpu --no-e2e --no-dispatch
t sync_bench 300 ./tools/sync_bench 2
t agg_bench 120 ./tools/agg_bench 1.5
# --gpus 8 without torchrun: one process per side, all on device 0 here (gloo
# for the timing reductions); host enqueue per step is in each line
t rehearsal8 300 env SRTP_BENCH_ONE_DEVICE=1 python bench.py --gpus 8 --backend gloo --steps 20 --no-cpu --no-e2e --no-dispatch
[ -n "$PROF" ] && TAG=${TAG:-final}/prof ./tools/prof.sh
echo final done
