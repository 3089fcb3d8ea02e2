#!/bin/bash
# Round-3 GPU pass: new parity tests (forced chain stall, bounded dispatcher
# rollback, aggregator lanes, raw RawPacket ABI), 1M streams over 8 shards,
# the whole GPU suite and the default bench line.  Test failures (exit 1) let
# the next steps run; a crash, abort or time limit (exit >= 124) ends the
# script.  The step limits sum to under gpurun's 1200 s.
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
PT="python -u -m pytest --timeout 200 --timeout-method thread -p no:cacheprovider"
t new 240 $PT -v tests/test_skew.py tests/test_dispatcher.py tests/test_aggregator.py tests/test_rawpacket.py -k "forced or bounded or lanes or forwards or raw_abi"
t c5 420 $PT -x -v -s tests/test_config5_sharded.py --timeout 400
t gpu 300 $PT -q tests -m gpu --deselect tests/test_config5_sharded.py::test_config5_1m_streams_8_shards
t bench 180 python bench.py
echo done
