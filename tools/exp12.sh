cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp12
timeout -k 10 600 python -u -m pytest tests/test_fuzz_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/exp12/pytest.log 2>&1
echo rc $?
