#!/bin/bash
# A/B of engine diagnostic builds on the default bench (free pipe)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_ab
for v in cur noev nocount none cur; do
  lib=""; [ "$v" != cur ] && lib="$PWD/libjitsi_amd/diag/lib_$v.so"
  for k in 20 100; do
    SRTP_MI355X_LIB=$lib timeout -k 10 200 python bench.py --steps $k --warmup 5 --no-cpu --no-e2e > gpurun_out/r02_ab/$v.$k.log 2>&1 || exit $?
    echo "$v $k $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r02_ab/$v.$k.log)"
  done
done
