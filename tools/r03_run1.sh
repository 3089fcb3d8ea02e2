#!/bin/bash
# Round-3 GPU pass: new parity tests (forced chain stall, bounded dispatcher
# rollback, aggregator lanes, raw RawPacket ABI), 1M streams over 8 shards,
# the whole GPU suite, the default bench line, and a 2-GPU in-process
# rehearsal on device 0.  Test failures (exit 1) let the next steps run; a
# crash, abort or time limit (exit >= 124) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R03_TAG:-r03a}
mkdir -p $O
t() {
  local name=$1 lim=$2; shift 2
  echo "== $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?
  echo "== $name exit $rc"; tail -4 $O/$name.log
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return 0
}
PT="python -u -m pytest --timeout 240 --timeout-method thread -p no:cacheprovider"
t new 400 $PT -v tests/test_skew.py tests/test_dispatcher.py tests/test_aggregator.py tests/test_rawpacket.py -k "forced or bounded or lanes or forwards or raw_abi"
t c5 600 $PT -x -v -s tests/test_config5_sharded.py --timeout 550
t gpu 900 $PT -q tests -m gpu --deselect tests/test_config5_sharded.py
t bench 600 python bench.py
SRTP_BENCH_ONE_DEVICE=1 t bench_inproc2 600 python bench.py --gpus 2 --steps 20 --no-cpu
t split 120 ./tools/split_bench 20
echo done
