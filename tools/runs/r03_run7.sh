#!/bin/bash
# Parity of the tree (GPU suites touching the crypto kernels), then an A/B of
# the default build against SRTP_TAIL_STEP=0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03g}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_fuzz_parity.py tests/test_pipeline.py -m gpu > $O/parity.log 2>&1; rc=$?
echo "parity exit $rc: $(tail -1 $O/parity.log)"
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $O/parity.log | head -30; exit $rc; }
R03_TAG=r03g/ab REPS=3 ./tools/r03_ab.sh default libjitsi_amd/variants/libsrtp_notail.so
