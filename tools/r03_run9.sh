#!/bin/bash
# Repair fan-out: the GPU suite, then C3 (faults) and C2 stage times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03l}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q -x --timeout 150 --timeout-method thread -p no:cacheprovider tests -m gpu > $O/gpu.log 2>&1; rc=$?
echo "gpu suite exit $rc: $(tail -1 $O/gpu.log)"
[ $rc -ne 0 ] && { grep -E "^E |FAILED|Error" $O/gpu.log | head -30; exit $rc; }
timeout -k 10 300 python -u tools/config_bench.py --configs C3,C4 > $O/cfg.log 2>&1 || { tail -5 $O/cfg.log; exit 1; }
grep '^{' $O/cfg.log | python -c "import sys,json
for l in sys.stdin:
    j=json.loads(l); print(j['config'], {k: j[k] for k in ('unprotect_pps','protect_pps','round_trips_per_s','stage_ms_per_bundle','all_ok','statuses') if k in j})"
timeout -k 10 200 python bench.py --steps 30 --no-cpu --no-e2e --no-dispatch > $O/bench.log 2>&1 && grep '^{' $O/bench.log | python -c "import sys,json; j=json.loads(sys.stdin.read()); print(round(j['value']/1e6,1), j['stage_ms'])"
