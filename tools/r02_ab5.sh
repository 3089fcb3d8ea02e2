#!/bin/bash
# Skewed bench points (one SSRC, Zipf 1.1) of each build given, alternating, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_ab5
mkdir -p $O
for rep in 1 2; do
  for mode in "--ssrcs 1" "--zipf 1.1"; do
    for lib in "$@"; do
      SRTP_MI355X_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e $mode > $O/b.log 2>&1 || { tail -3 $O/b.log; exit 1; }
      python -c "import json; l=[x for x in open('$O/b.log') if x.startswith('{')][-1]; j=json.loads(l); print('$lib'.split('/')[-1], '$mode', round(j['value']/1e6,1), j['stage_ms']['walk'], j['stage_ms']['parse'])"
    done
  done
done
