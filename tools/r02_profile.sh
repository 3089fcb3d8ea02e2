# Round-2 evidence: default bench line, rocprofv3 kernel traces (default and
# --serial) and PMC passes (serial: each kernel alone on the GPU, as in the
# bench's stage-timing pass that the roofline uses).
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/r02prof
mkdir -p $P
S="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial"
timeout -k 10 400 python bench.py > $P/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_default -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e > $P/t1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --serial > $P/t2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $S > $P/f.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $S > $P/w.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/sq -o run -- $S > $P/s.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq2 -o run -- $S > $P/s2.log 2>&1
echo rc $?
