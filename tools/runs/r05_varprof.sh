#!/bin/bash
# Round 5: per-variant counters (serial bench trace + SQ passes) of the
# occupancy / schedule variants, for profiles/r05/kernel_experiments.md.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/r05var
mkdir -p $P
S="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-dispatch --serial"
for V in lean0 occ3; do
  export SRTP_MI355X_LIB=libjitsi_amd/variants/libsrtp_$V.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/$V/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial > $P/${V}_trace.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/$V/sq -o run -- $S > $P/${V}_sq.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/$V/sq2 -o run -- $S > $P/${V}_sq2.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/$V/fetch -o run -- $S > $P/${V}_fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/$V/write -o run -- $S > $P/${V}_write.log 2>&1 || exit $?
  unset SRTP_MI355X_LIB
done
