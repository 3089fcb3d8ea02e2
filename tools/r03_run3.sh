#!/bin/bash
# Round-3 GPU pass 3: aggregator tests after the lock-free rewrite, the
# aggregator throughput tool, the line-staging memory micro-benchmark (times,
# then FETCH_SIZE / WRITE_SIZE per dispatch).  Test failures continue; a crash
# or time limit (exit >= 124) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R03_TAG:-r03c}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -3 $O/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest --timeout 200 --timeout-method thread -p no:cacheprovider"
t agg 200 $PT -v tests/test_aggregator.py tests/test_rawpacket.py tests/test_dispatcher.py -m gpu
t agg_bench 120 ./tools/agg_bench 1.5
t line 120 ./tools/line_bench 10
t line_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/line_fetch -o run -- ./tools/line_bench 2
t line_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/line_write -o run -- ./tools/line_bench 2
echo done
