#!/bin/bash
# Round 5: the look-back second sort pass (no count launch) -- GPU suite,
# A/B against the HEAD build (libjitsi_amd/variants/libsrtp_head.so), and a
# two-stream kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05j}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch > $O/trace.log 2>&1 || exit $?
python3 tools/timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 10 > $O/timeline.txt && head -14 $O/timeline.txt
