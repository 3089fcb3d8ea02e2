#!/bin/bash
# Round 5: {g0, auth_ok} packed per packet (one 8-B gather in the walk):
# parity subset of the new default, then A/B against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05gok
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tag_lengths.py tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py tests/test_small_bundles.py tests/test_fuzz_parity.py tests/test_single_packet.py tests/test_skein.py tests/test_twofish.py tests/test_aes256.py > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=r05gok/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so
