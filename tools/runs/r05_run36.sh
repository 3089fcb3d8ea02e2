#!/bin/bash
# Round 5: k_unprotect's context loads after the T-table fill (SRTP_CTX_AFTER_FILL variant).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05caf/ab REPS=4 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_caf.so
