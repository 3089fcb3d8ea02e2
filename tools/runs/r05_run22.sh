#!/bin/bash
# Round 5: k_unprotect saves the walk's re-check state only for contexts with
# a packet far from s_l (BundleArgs::far) -- GPU suite, A/B against the
# save-always build, serial trace; and the dispatcher's two-in-flight mode
# from Python with / without other engines alive.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05v}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_savestate.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial > $O/trace.log 2>&1 || exit $?
grep -E "k_unprotect|k_protect|k_parse" $(find $O/trace -name "*kernel_stats.csv" | head -1) | cut -d, -f1-4
timeout -k 10 300 python3 tools/dispatch_async_py.py 16 > $O/dispatch_async_py.jsonl 2>&1 || exit $?
cat $O/dispatch_async_py.jsonl
