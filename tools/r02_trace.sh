#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02_trace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/join20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --pipe join > $O/t1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/free20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --pipe free > $O/t2.log 2>&1
echo rc $?
