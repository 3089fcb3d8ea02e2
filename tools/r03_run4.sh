#!/bin/bash
# Round-3 GPU pass 4: line_bench with the coalesced LDS-DMA modes; the
# dispatcher tests and the bench's dispatch leg with the copy-helper pool.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R03_TAG:-r03d}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -3 $O/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest --timeout 200 --timeout-method thread -p no:cacheprovider"
t line 120 ./tools/line_bench 10
t disp 200 $PT -q tests/test_dispatcher.py tests/test_aggregator.py tests/test_rawpacket.py -m gpu
t bench_disp 150 python bench.py --steps 10 --no-cpu --no-e2e --dispatch-bundles 6
echo done
