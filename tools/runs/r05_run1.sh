#!/bin/bash
# Round 5, first GPU call: the asynchronous per-packet path (GPU tests of the
# shim / aggregator / per-packet paths, sync_bench's queue / arrayq points),
# then the lean-register AES round variants A/B'd against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_jni_shim.py \
  tests/test_aggregator.py tests/test_single_packet.py tests/test_rawpacket.py > $O/tests.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc  # test failures (1) still leave the benches to run
for p in "queue 0 8 rt" "queue 0 16 rt" "queue 0 64 rt" "queue 8 16 rt" "one 0 64 rt" "array 0 8" "arrayq 0 8" \
         "array 8 8" "arrayq 8 8" "arrayq 0 64"; do
  timeout -k 10 90 ./tools/sync_bench 3 $p >> $O/sync.jsonl || exit $?
done
AB_TAG=r05a/ab REPS=2 bash tools/ab.sh default libjitsi_amd/variants/libsrtp_lean16.so \
  libjitsi_amd/variants/libsrtp_lean20.so libjitsi_amd/variants/libsrtp_lean24.so > $O/ab.txt 2>&1
