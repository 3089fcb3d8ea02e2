#!/bin/bash
# Round-2 GPU steps.  Usage: tools/gpu_r02.sh <mode> [pytest -k expr]
#   test   -m gpu suite (optionally -k), then smoke
#   bench  default bench line + 20-step line
#   both   test then bench
# Every GPU step runs under its own timeout; the script stops at the first
# crash / timeout (exit >= 124) so nothing else touches a faulted GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02
O=gpurun_out/r02
MODE=${1:-test}
K=${2:-}
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -4 "$O/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
if [ "$MODE" = test ] || [ "$MODE" = both ]; then
  if [ -n "$K" ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "$K"
  else
    run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider
  fi
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = bench ] || [ "$MODE" = both ]; then
  run bench20 300 python bench.py --steps 20 --warmup 5
  run bench100 300 python bench.py --steps 100 --no-cpu --no-e2e
fi
exit 0
