#!/bin/bash
# Walk-stage diagnostics: stage_ms of the serial bench under SRTP_DEBUG modes
# (1: the walk returns after staging its records; 2: trivial per-record step;
# results wrong by design, timing only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_walkdiag
mkdir -p $O
for d in 0 1 2 0; do
  SRTP_DEBUG=$d timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $O/d$d.log 2>&1 || { echo "debug $d failed rc=$?"; tail -3 $O/d$d.log; exit 1; }
  python -c "import json,sys; l=[x for x in open('$O/d$d.log') if x.startswith('{')][-1]; j=json.loads(l); print('debug', $d, j['value']/1e6, j['stage_ms'])"
done
