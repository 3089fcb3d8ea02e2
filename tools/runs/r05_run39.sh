#!/bin/bash
# Round 5: the trailer's first two words as one 8-B store: tag-length and
# parity subset on the new default, then A/B (4 reps) against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05t8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_tag_lengths.py tests/test_gpu_parity.py tests/test_golden.py tests/test_small_bundles.py tests/test_fuzz_parity.py tests/test_single_packet.py > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=r05t8/ab REPS=4 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so
