#!/bin/bash
# GPU parity / skew tests of the default build, then the uniform, Zipf and
# one-SSRC bench points of each build given (alternating, twice).
# Usage: tools/r02_ab4.sh lib1 lib2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_ab4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_skew.py tests/test_gpu_parity.py tests/test_fuzz_parity.py tests/test_rawpacket.py -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do
  for mode in "" "--zipf 1.1" "--ssrcs 1"; do
    for lib in "$@"; do
      SRTP_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e $mode > $O/b.log 2>&1 || { tail -3 $O/b.log; exit 1; }
      python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$lib'.split('/')[-1], '$mode', round(j['value']/1e6,1), j['stage_ms']['walk'], j['slow_path_per_bundle']['long_walked'])"
    done
  done
done
