#!/bin/bash
# bench stream-coupling variants at 20 and 100 steps
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_pipe
for p in free join; do
  for k in "20 5" "100 5" "20 30"; do
    set -- $k
    timeout -k 10 200 python bench.py --steps $1 --warmup $2 --no-cpu --no-e2e --pipe $p > gpurun_out/r02_pipe/$p.$1.$2.log 2>&1 || exit $?
    echo "$p $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_pipe/$p.$1.$2.log)"
  done
done
