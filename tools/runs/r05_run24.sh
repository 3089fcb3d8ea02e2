#!/bin/bash
# Round 5: k_unprotect's received tag loaded ahead of the last SHA-1 blocks --
# parity subset, A/B against the build without it (variants/libsrtp_notagpf.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05x}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_fuzz_parity.py > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=$T/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_notagpf.so > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
