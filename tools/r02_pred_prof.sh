#!/bin/bash
# ROC prediction cost: 100-step bench line, then a kernel trace of the serial pass
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/r02_predprof
mkdir -p $P
timeout -k 10 300 python bench.py --steps 100 --no-cpu --no-e2e > $P/bench.log 2>&1 &&
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' $P/bench.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --serial > $P/t2.log 2>&1
echo rc $?
f=$(ls $P/trace/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -d, -f1-6 "$f"
exit 0
