# F8 parity tests + F8 bench after the two-packets-per-lane k_f8
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/exp6/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --policy F8_128_HMAC_SHA1_80 --steps 20 > gpurun_out/exp6/b_f8.log 2>&1
echo rc $?
