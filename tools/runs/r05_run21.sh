#!/bin/bash
# Round 5: the MSD two-digit sort (high-digit pass + per-bucket low-digit
# sort, no count launch) -- the whole GPU suite, A/B against the LSD build
# (libjitsi_amd/variants/libsrtp_lsd.so), skewed bundles, two-stream trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05u}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; tail -3 $O/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_lsd.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
for z in "--zipf 1.1" "--ssrcs 1"; do
  for lib in default libjitsi_amd/variants/libsrtp_lsd.so; do
    if [ "$lib" = default ]; then unset SRTP_MI355X_LIB; else export SRTP_MI355X_LIB=$PWD/$lib; fi
    timeout -k 10 300 python3 bench.py --steps 20 --no-cpu --no-e2e --no-dispatch $z > $O/skew.log 2>&1 || exit $?
    grep -a '^{' $O/skew.log | tail -1 | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$z', '$lib'.split('/')[-1], round(j['value']/1e6,1), j['stage_ms'])"
  done
done
unset SRTP_MI355X_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch > $O/trace.log 2>&1 || exit $?
python3 tools/timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) 10 > $O/timeline.txt && head -14 $O/timeline.txt
# dispatcher host bundles without Python: synchronous and two in flight
timeout -k 10 120 ./tools/dispatch_bench 16 1 > $O/dispatch_bench.jsonl 2>&1 || exit $?
cat $O/dispatch_bench.jsonl
