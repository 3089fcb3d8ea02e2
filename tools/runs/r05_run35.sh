#!/bin/bash
# Round 5: non-temporal chunk stores in the fused loops (SRTP_NT_STORES variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05nt/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_nt.so
