# parse with early loads: GPU tests + bench
cd "${GRAFT_REPO_ROOT}"
P=gpurun_out/exp11
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $P/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b.log 2>&1
echo rc $?
