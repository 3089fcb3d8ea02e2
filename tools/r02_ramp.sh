#!/bin/bash
# Is the 20-step shortfall a ramp-up? Longer warmup, and a kernel trace of a
# 20-step join run (per-step durations over time).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r02_ramp
mkdir -p $O
for w in 5 30 100; do
  timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu --no-e2e --pipe join > $O/join.w$w.log 2>&1 || exit $?
  echo "join w$w $(grep -o '"ms_per_step": [0-9.]*' $O/join.w$w.log)"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 30 --no-cpu --no-e2e --pipe free > $O/free.w30.log 2>&1 || exit $?
echo "free w30 $(grep -o '"ms_per_step": [0-9.]*' $O/free.w30.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --pipe join > $O/t.log 2>&1
echo rc $?
