# default vs non-temporal-store kernel build: bench + HBM traffic passes
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/exp5
mkdir -p $P
NT=$PWD/libjitsi_amd/libsrtp_mi355x_nt.so
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b_def.log 2>&1 &&
SRTP_MI355X_LIB=$NT timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b_nt.log 2>&1 &&
SRTP_MI355X_LIB=$NT timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial > $P/t.log 2>&1 &&
SRTP_MI355X_LIB=$NT timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial > $P/f.log 2>&1 &&
SRTP_MI355X_LIB=$NT timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial > $P/w.log 2>&1
echo rc $?
