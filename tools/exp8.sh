# k_unprotect workgroup size variants: bench at 1200 B and 160 B
cd "${GRAFT_REPO_ROOT}"
P=gpurun_out/exp8
mkdir -p $P
V=$PWD/libjitsi_amd/libsrtp_mi355x_768.so
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b_def.log 2>&1 &&
SRTP_MI355X_LIB=$V timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b_768.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --len 160 > $P/b_def160.log 2>&1 &&
SRTP_MI355X_LIB=$V timeout -k 10 300 python bench.py --no-cpu --no-e2e --len 160 > $P/b_768_160.log 2>&1
echo rc $?
