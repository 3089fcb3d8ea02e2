#!/bin/bash
# A/B of engine builds on the default bench point: each build given (a path to
# a variant .so, or "default"), alternating, REPS times; prints value and the
# crypto kernels' per-launch times.  Then a short parity check of each variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${AB_TAG:-ab}
mkdir -p $O
REPS=${REPS:-2}
for rep in $(seq $REPS); do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset SRTP_MI355X_LIB; else export SRTP_MI355X_LIB=$PWD/$lib; fi
    timeout -k 10 120 python bench.py --steps 30 --no-cpu --no-e2e --no-dispatch > $O/b.log 2>&1 || { echo "bench failed: $lib"; tail -5 $O/b.log; exit 1; }
    python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); s=j['stage_ms']; print('$lib'.split('/')[-1], round(j['value']/1e6,1), s)"
  done
done
unset SRTP_MI355X_LIB
for lib in "$@"; do
  [ "$lib" = default ] && continue
  SRTP_MI355X_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py tests/test_golden.py tests/test_skew.py tests/test_repairs.py -m gpu > $O/parity_$(basename $lib).log 2>&1; rc=$?
  echo "parity $lib exit $rc: $(tail -1 $O/parity_$(basename $lib).log)"
  [ $rc -ge 124 ] && exit $rc
done
echo done
