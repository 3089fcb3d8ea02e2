#!/bin/bash
# Round 5: crypto-kernel variants A/B (lean16 default vs the round-4 schedule,
# 3 waves/SIMD without spills, no re-check state stores), and the dispatcher's
# FIFO lock under 8 array callers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5TAG:-r05h}
mkdir -p $O
AB_TAG=${R5TAG:-r05h}/ab REPS=2 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_lean0.so \
  libjitsi_amd/variants/libsrtp_occ3.so libjitsi_amd/variants/libsrtp_notail.so > $O/ab.txt 2>&1 || exit $?
for p in "array 8 8" "arrayq 8 8" "arrayq 8 1" "array 8 1"; do
  timeout -k 10 60 ./tools/sync_bench 2 $p >> $O/sync.jsonl || exit $?
done
