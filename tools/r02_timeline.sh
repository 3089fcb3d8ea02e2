#!/bin/bash
# GPU tests, then a kernel trace (start/end per dispatch) of the default
# two-stream bench for the step timeline (tools/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_tl
mkdir -p $O
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -4 "$O/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return $rc
}
if [ "${1:-all}" != notest ]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
fi
run trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e
exit 0
