# new GPU parity test + 2-rank rehearsal of the multi-GPU bench path on one GPU (gloo)
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/exp3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "config5 or full_size" > gpurun_out/exp3/pytest.log 2>&1 || exit $?
SRTP_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --backend gloo > gpurun_out/exp3/dist2.log 2>&1
echo rc $?
