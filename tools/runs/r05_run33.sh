#!/bin/bash
# Round 5 diagnostic: what k_protect's byte-wise tag write costs (variant
# writes no tag: wrong output, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05tw/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_notagw.so
