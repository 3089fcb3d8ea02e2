#!/bin/bash
# Round 5: k_protect's word-store trailer: every tag length 1..12 (new test),
# the parity subset, then A/B against the previous library (variants/libsrtp_head.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05tw2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tag_lengths.py tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_fuzz_parity.py tests/test_single_packet.py tests/test_rawpacket.py > $O/parity.log 2>&1
rc=$?; tail -3 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=r05tw2/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so
