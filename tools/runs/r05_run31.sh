#!/bin/bash
# Round 5 diagnostic: what k_unprotect's tag compare and long-chain check cost
# (variants wrong on forged tags / long chains; timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05dg/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_notag.so libjitsi_amd/variants/libsrtp_nolng.so
