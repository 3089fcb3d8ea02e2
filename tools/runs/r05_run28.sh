#!/bin/bash
# Round 5: k_protect's last partial chunk in one more fused step (SRTP_PROTECT_TAIL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05pt/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_ptail.so
