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
  step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
  step bench 600 python bench.py
fi
if [ "$MODE" = quick ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  step bench 300 python bench.py --no-cpu
  export TMPDIR=/tmp
  step rocprof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu
fi
if [ "$MODE" = valu ]; then
  step valu_bench 120 ./tools/valu_bench
fi
if [ "$MODE" = probe ]; then
  step probe 300 python tools/walk_probe.py
fi
if [ "$MODE" = one ]; then
  step pytest_one 600 python -m pytest tests -m gpu -q -x --timeout 300 -p no:cacheprovider -k "${2:-malformed}"
fi
if [ "$MODE" = diag2 ]; then
  step diag2 300 python tools/twin_diag.py
fi
if [ "$MODE" = diag ]; then
  step diag 600 python tools/bench_loop_diag.py
fi
if [ "$MODE" = micro ]; then
  step sort_bench 120 ./tools/sort_bench
fi
if [ "$MODE" = micro ]; then
  export TMPDIR=/tmp
  step calib 120 ./tools/pmc_calib
  step calib_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/calib/trace -o run -- ./tools/pmc_calib
  step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run -- ./tools/pmc_calib
  step calib_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/write -o run -- ./tools/pmc_calib
fi
if [ "$MODE" = prof ] || [ "$MODE" = profall ]; then
  export TMPDIR=/tmp
  B="python3 bench.py --steps 5 --warmup 1 --no-cpu"
  P=gpurun_out/prof
  step rocprof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $B
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $B
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $B
  step pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/sq -o run -- $B
  step pmc_sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq2 -o run -- $B
fi
if [ "$MODE" = profall ]; then
  step calib 120 ./tools/pmc_calib
  step calib_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/calib/trace -o run -- ./tools/pmc_calib
  step calib_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib/fetch -o run -- ./tools/pmc_calib
  step calib_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/calib/write -o run -- ./tools/pmc_calib
fi
if [ "$MODE" = golden ]; then
  step pytest_golden 600 python -u -m pytest tests/test_golden.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
fi
exit 0
