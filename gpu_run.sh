#!/bin/bash
# GPU-box driver for one measurement round: tests, smoke, bench, profile.
# Stops at the first crash/timeout (exit >= 124 or signal); test failures
# (exit 1) still let the smoke/bench steps run so the numbers are recorded.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
mkdir -p gpurun_out
step() {  # step <name> <timeout-s> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*" ; date
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ] || [ "$MODE" = diag ]; then
  step pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py --steps 20 --warmup 3
fi
if [ "$MODE" = diag ]; then
  step diag 600 python tools_diag.py
fi
if [ "$MODE" = prof ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu
fi
exit 0
