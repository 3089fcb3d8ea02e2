#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_ab2
for v in default new; do
  e=0; [ $v = new ] && e=1
  for k in 20 100; do
    SRTP_BENCH_NEW_STREAM_A=$e timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu --no-e2e > gpurun_out/r02_ab2/$v.$k.log 2>&1 || exit $?
    echo "$v $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_ab2/$v.$k.log)"
  done
done
for p in join lag1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --pipe $p > gpurun_out/r02_ab2/$p.20.log 2>&1 || exit $?
  echo "$p 20 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_ab2/$p.20.log)"
done
