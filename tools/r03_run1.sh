#!/bin/bash
# Round-3 first GPU pass: new parity tests (forced chain stall, bounded
# dispatcher rollback, 1M streams over 8 shards), the whole GPU suite, the
# default bench line, and a 2-GPU in-process rehearsal on device 0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03a
mkdir -p $O
t() { local name=$1 lim=$2; shift 2; echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name exit $rc"; tail -3 $O/$name.log; return $rc; }
t new 400 python -u -m pytest tests/test_skew.py tests/test_dispatcher.py tests/test_aggregator.py tests/test_rawpacket.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -k "forced or bounded or lanes or forwards or raw_abi" &&
t c5 600 python -u -m pytest tests/test_config5_sharded.py -x -v -s --timeout 550 --timeout-method thread -p no:cacheprovider &&
t gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_config5_sharded.py &&
t bench 600 python bench.py &&
SRTP_BENCH_ONE_DEVICE=1 t bench_inproc2 600 python bench.py --gpus 2 --steps 20 --no-cpu --ssrcs 10000
