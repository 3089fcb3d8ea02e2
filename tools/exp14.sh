# F8 with the HMAC folded into the chain loop: GPU tests + F8 bench
cd "${GRAFT_REPO_ROOT}"
P=gpurun_out/exp14
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $P/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --policy F8_128_HMAC_SHA1_80 --steps 20 > $P/b_f8.log 2>&1
echo rc $?
