# FETCH_SIZE / WRITE_SIZE passes of a short bench run (separate --pmc passes)
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
P=gpurun_out/pq
B="python3 bench.py --steps 5 --warmup 1 --no-cpu --serial"
mkdir -p $P
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- $B > $P/t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $B > $P/f.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $B > $P/w.log 2>&1
echo rc $?
