#!/bin/bash
# Profile evidence of the committed tree: rocprofv3 kernel traces
# (serial and default two-stream bench), PMC passes (serial, as the roofline's
# stage timing), the PMC summary (writes profiles/pmc_traffic.json), and the
# FETCH_SIZE / WRITE_SIZE calibration of the kernels' access pattern
# (tools/pmc_calib).  Each GPU step has its own time limit; the first failure
# ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/${TAG:-prof}
mkdir -p $P
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$P/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -2 "$P/$name.log"
  return $rc
}
S="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-dispatch --serial"
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial &&
run fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $S &&
run write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $S &&
run sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/sq -o run -- $S &&
run sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq2 -o run -- $S &&
run calib_trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d $P/calib/trace -o run -- ./tools/pmc_calib &&
run calib_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/calib/fetch -o run -- ./tools/pmc_calib &&
run calib_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/calib/write -o run -- ./tools/pmc_calib &&
run calib_factor 60 python tools/pmc_calib_factor.py $P/calib &&
run pmc_summary 120 python tools/pmc_summary.py $P --calib $P/calib/factor.json --out $P/summary &&
run trace_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_default -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch &&
python tools/timeline.py $(find $P/trace_default -name "*kernel_trace.csv" | head -1) 10 > $P/timeline.txt && head -12 $P/timeline.txt || exit 1
# Per-variant counters (profiles/r04/kernel_experiments.md): the candidate
# builds of tools/build_variant.sh, same serial bench, trace + SQ passes.
for V in ${VARIANTS:-}; do
  L=libjitsi_amd/variants/libsrtp_$V.so
  [ -f $L ] || { echo "no $L"; exit 1; }
  export SRTP_MI355X_LIB=$L
  run ${V}_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$V/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial &&
  run ${V}_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/$V/sq -o run -- $S &&
  run ${V}_sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/$V/sq2 -o run -- $S &&
  run ${V}_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/$V/fetch -o run -- $S &&
  run ${V}_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/$V/write -o run -- $S &&
  python tools/pmc_summary.py $P/$V > $P/$V/pmc_summary.txt || exit 1
  unset SRTP_MI355X_LIB
done
echo done
