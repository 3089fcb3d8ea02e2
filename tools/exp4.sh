# packet-size / profile sweep of the bench workload (10k SSRCs, 2^18-packet bundles)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp4
timeout -k 10 300 python bench.py --no-cpu --no-e2e --len 160 > gpurun_out/exp4/b_160.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --len 400 > gpurun_out/exp4/b_400.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --policy AES_CM_128_HMAC_SHA1_32 > gpurun_out/exp4/b_32.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --policy F8_128_HMAC_SHA1_80 --steps 20 > gpurun_out/exp4/b_f8.log 2>&1
echo rc $?
