#!/bin/bash
# Round 5: walk passes in one launch (k_walk2), re-check state only for
# contexts whose ROC could change in-bundle, asynchronous dispatcher host
# bundles -- the whole GPU suite, A/B against the save-always build, the
# dispatcher leg, a two-stream trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05o}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; [ $rc -gt 1 ] && exit $rc
grep -E "FAILED|ERROR" $O/gpu_suite.log | head -5
AB_TAG=$T/ab REPS=2 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_savestate.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
for sh in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --no-e2e --dispatch-shards $sh > $O/bench_dispatch_$sh.log 2>&1 || exit $?
  tail -1 $O/bench_dispatch_$sh.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); [print(k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle'], v['all_accepted']) for k,v in j['dispatch'].items()]"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch > $O/trace.log 2>&1 || exit $?
python3 tools/timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 10 > $O/timeline.txt && head -14 $O/timeline.txt
