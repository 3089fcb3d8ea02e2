# k_protect chunk prefetch variant vs default (bench twice each, alternating)
cd "${GRAFT_REPO_ROOT}"
P=gpurun_out/exp13
mkdir -p $P
V=$PWD/libjitsi_amd/libsrtp_mi355x_pf.so
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/def_$r.log 2>&1 || exit $?
  SRTP_MI355X_LIB=$V timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/pf_$r.log 2>&1 || exit $?
done
echo done
