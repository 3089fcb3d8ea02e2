#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_walk
for d in 0 1 2 0 1 2; do
  SRTP_DEBUG=$d timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --no-e2e > gpurun_out/r02_walk/$d.log 2>&1 || exit $?
  echo "debug=$d $(grep -o '"stage_ms": {[^}]*}' gpurun_out/r02_walk/$d.log)"
done
