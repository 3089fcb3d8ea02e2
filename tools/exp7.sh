# PMC passes of the 160-B workload (serial): k_protect vs k_unprotect
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/exp7
mkdir -p $P
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial --len 160"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $B > $P/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $B > $P/f.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $B > $P/w.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/sq -o run -- $B > $P/s.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq2 -o run -- $B > $P/s2.log 2>&1
echo rc $?
