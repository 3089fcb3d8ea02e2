# walk span variants (records per lane 2 / 4 / 8)
cd "${GRAFT_REPO_ROOT}"
P=gpurun_out/exp10
mkdir -p $P
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b4.log 2>&1 &&
SRTP_MI355X_LIB=$PWD/libjitsi_amd/libsrtp_mi355x_w8.so timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b8.log 2>&1 &&
SRTP_MI355X_LIB=$PWD/libjitsi_amd/libsrtp_mi355x_w2.so timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b2.log 2>&1 &&
SRTP_MI355X_LIB=$PWD/libjitsi_amd/libsrtp_mi355x_w8.so timeout -k 10 300 python bench.py --no-cpu --no-e2e --ssrcs 100000 > $P/b8_100k.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --ssrcs 100000 > $P/b4_100k.log 2>&1
echo rc $?
