#!/bin/bash
# Walk tile size A/B: GPU parity + skew tests on the variant build, then the
# uniform, Zipf and one-SSRC bench points of the default build and the variant.
# Usage: tools/r02_walkspan.sh <variant .so>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_walkspan
mkdir -p $O
V=$1
SRTP_MI355X_LIB=$PWD/$V timeout -k 10 600 python -u -m pytest tests/test_skew.py tests/test_gpu_parity.py tests/test_fuzz_parity.py -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  for mode in "" "--zipf 1.1" "--ssrcs 1"; do
    for lib in libjitsi_amd/libsrtp_mi355x.so $V; do
      SRTP_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e $mode > $O/b.log 2>&1 || exit 1
      python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$lib', '$mode', round(j['value']/1e6,1), j['stage_ms']['walk'], j['stage_ms']['sort'])"
    done
  done
done
