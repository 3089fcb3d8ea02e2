#!/bin/bash
# Round-3 pass 6: aggregator tests and throughput after the per-thread block
# rewrite, then the profile evidence of the tree (tools/r03_prof.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R03_TAG:-r03f}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -3 $O/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
t agg 200 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_aggregator.py tests/test_rawpacket.py -m gpu
t agg_bench 120 ./tools/agg_bench 1.5
R03_TAG=${R03_TAG:-r03f}/prof ./tools/r03_prof.sh
