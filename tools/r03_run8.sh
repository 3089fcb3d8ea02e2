#!/bin/bash
# Length-class lane order: the whole GPU suite, then C3/C4 with and without it,
# then the default bench A/B (one length class: must not regress).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03k}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu.log 2>&1; rc=$?
echo "gpu suite exit $rc: $(tail -1 $O/gpu.log)"
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $O/gpu.log | head -30; exit $rc; }
for lib in default libjitsi_amd/variants/libsrtp_nolen.so; do
  if [ "$lib" = default ]; then unset SRTP_MI355X_LIB; else export SRTP_MI355X_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/config_bench.py --configs C3,C4 > $O/cfg_$(basename $lib).log 2>&1 || { echo "config_bench failed $lib"; tail -5 $O/cfg_$(basename $lib).log; exit 1; }
  echo "== $lib"; grep '^{' $O/cfg_$(basename $lib).log | python -c "import sys,json
for l in sys.stdin:
    j=json.loads(l); print(j['config'], {k: j[k] for k in ('unprotect_pps','protect_pps','round_trips_per_s','stage_ms_per_bundle','all_ok') if k in j})"
done
unset SRTP_MI355X_LIB
R03_TAG=r03k/ab REPS=2 ./tools/r03_ab.sh default libjitsi_amd/variants/libsrtp_nolen.so
