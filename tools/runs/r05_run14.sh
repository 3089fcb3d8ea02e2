#!/bin/bash
# Round 5: k_unprotect saves the walk's re-check state only for contexts whose
# ROC could change within the bundle (per-context SEQ range from k_parse) --
# parity subset, A/B against the save-always build
# (libjitsi_amd/variants/libsrtp_savestate.so), serial kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05n}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_config5_sharded.py tests/test_fuzz_parity.py tests/test_single_packet.py > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_savestate.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial > $O/trace.log 2>&1 || exit $?
grep -E "k_unprotect|k_protect|k_parse" $O/trace/run_kernel_stats.csv | cut -d, -f1-4
