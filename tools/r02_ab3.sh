#!/bin/bash
# A/B of engine builds (SRTP_MI355X_LIB): stage timings and bench value,
# alternating, twice each.  Usage: tools/r02_ab3.sh lib1 lib2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_ab3
mkdir -p $O
for rep in 1 2; do
  for lib in "$@"; do
    SRTP_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 50 --warmup 3 --no-cpu --no-e2e > $O/b.log 2>&1 || { echo "$lib failed"; tail -3 $O/b.log; exit 1; }
    python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$lib', round(j['value']/1e6,1), j['stage_ms'])"
  done
done
