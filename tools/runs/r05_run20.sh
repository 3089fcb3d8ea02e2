#!/bin/bash
# Round 5: the dispatcher leg's asynchronous mode against the number of
# bundles (4 / 8 / 16), 1 shard.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05t}
O=gpurun_out/$T
mkdir -p $O
for nb in 4 8 16 4; do
  timeout -k 10 400 python3 bench.py --steps 5 --no-cpu --no-e2e --dispatch-shards 1 --dispatch-bundles $nb > $O/b$nb.log 2>&1 || exit $?
  grep -a '^{' $O/b$nb.log | tail -1 | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); [print($nb, k, round(v['directional_pps']/1e6,2), v['ms_per_bundle'], v['host_ms_per_bundle']) for k,v in j['dispatch'].items()]"
done
