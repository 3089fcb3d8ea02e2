cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp1
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu > gpurun_out/exp1/b_streams.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 100 --warmup 5 --no-cpu --serial > gpurun_out/exp1/b_serial.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp1/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --serial > gpurun_out/exp1/t.log 2>&1
echo done $?
