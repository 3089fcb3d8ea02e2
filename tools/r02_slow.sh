#!/bin/bash
# Slow-path counters (packets per bundle walked by walk_long, repaired, ROC
# re-checks) and walk stage time of the uniform, Zipf and one-SSRC bench points.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_slow
mkdir -p $O
for mode in "" "--zipf 1.1" "--ssrcs 1"; do
  timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e $mode > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$mode', round(j['value']/1e6,1), j['stage_ms'], j['slow_path_per_bundle'])"
done
