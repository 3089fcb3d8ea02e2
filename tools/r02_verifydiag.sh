#!/bin/bash
# k_unprotect diagnostics: stage timing with SRTP_DEBUG=3 (no midstate / ROC-block
# ciphertext stores; results wrong by design) against the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_verifydiag
mkdir -p $O
for d in 0 3 0 3; do
  SRTP_DEBUG=$d timeout -k 10 200 python bench.py --steps 50 --warmup 3 --no-cpu --no-e2e > $O/d$d.log 2>&1 || { echo "debug $d failed"; tail -3 $O/d$d.log; exit 1; }
  python -c "import json; l=[x for x in open('$O/d$d.log') if x.startswith('{')][-1]; j=json.loads(l); print('debug', $d, round(j['value']/1e6,1), j['stage_ms'])"
done
