#!/bin/bash
# Round 2: why does a 20-step bench read lower than a 100-step one?
# Bench lines at both step counts, then a kernel trace of the 20-step run.
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/r02_steps
mkdir -p $P
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > $P/b20a.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu --no-e2e > $P/b100.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > $P/b20b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $P/trace20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e > $P/t20.log 2>&1
echo rc $?
