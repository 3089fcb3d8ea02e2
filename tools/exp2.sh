# stream-count sweep of the bench workload (1200-B packets, 2^18-packet bundles)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp2
for s in 100000 1000000; do
  timeout -k 10 400 python bench.py --no-cpu --no-e2e --ssrcs $s > gpurun_out/exp2/b_$s.log 2>&1 || exit $?
done
echo done
