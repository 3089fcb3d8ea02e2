#!/bin/bash
# Round 5: k_parse workgroup size (global count atomics per sort tile: 8 / 4 / 2 workgroups).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
AB_TAG=r05pb/ab REPS=3 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_pb512.so libjitsi_amd/variants/libsrtp_pb1024.so
