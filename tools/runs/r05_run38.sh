#!/bin/bash
# Round 5: the walk's result as one 16-B record per packet: the whole GPU
# suite on the new default, then A/B against the previous library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05wo
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ > $O/gpu_suite.log 2>&1
rc=$?; tail -2 $O/gpu_suite.log; [ $rc -ne 0 ] && exit $rc
AB_TAG=r05wo/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_head.so
