#!/bin/bash
# Round 5: k_unprotect's tag compare from aligned 16-B pieces (tag_matches_at):
# parity of the new default on the subset with forged tags and odd lengths,
# then A/B against the previous library (variants/libsrtp_head.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05tg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_fuzz_parity.py tests/test_single_packet.py > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=r05tg/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so
