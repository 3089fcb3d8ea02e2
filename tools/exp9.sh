# after the unprotect round-key reload fix: GPU tests, bench at 1200 / 160 B, traffic passes
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/exp9
mkdir -p $P
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $P/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e > $P/b.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu --no-e2e --len 160 > $P/b160.log 2>&1 &&
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $B > $P/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $B > $P/f.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $B > $P/w.log 2>&1
echo rc $?
