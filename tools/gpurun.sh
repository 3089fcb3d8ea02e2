#!/bin/bash
# One runner for the GPU box (round 6 on): `gpurun -- bash tools/gpurun.sh
# <recipe> [<recipe> ...]`, each recipe a step with its own time limit, all
# output under gpurun_out/$TAG/.  The first failing step ends the call (a GPU
# fault, abort or time limit must not be followed by more GPU work).
# (The one-off per-call scripts of rounds 1-5 are under tools/runs/, which
# does not travel to the box.)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${TAG:-run}
mkdir -p "$O"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
BENCH="python bench.py --no-cpu --no-e2e --no-dispatch"

step() {  # step <name> <seconds> <cmd...>: output in $O/<name>.log
    local name=$1 t=$2
    shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
    local rc=$?
    echo "== $name exit $rc"
    tail -4 "$O/$name.log"
    return $rc
}

recipe() {
    case "$1" in
    suite)        step suite 900 $PYT tests -m gpu ;;
    # the parity-bearing tests with every engine on the split path / on the fused kernels
    parity_wide)  SRTP_TEST_DEBUG=2 step parity_wide 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_golden.py \
                      tests/test_small_bundles.py tests/test_repairs.py tests/test_skew.py tests/test_fuzz_parity.py \
                      tests/test_tag_lengths.py tests/test_context_export.py tests/test_lifecycle.py ;;
    parity_fused) SRTP_TEST_DEBUG=4 step parity_fused 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_golden.py \
                      tests/test_skew.py tests/test_repairs.py ;;
    dispatch_tests) step dispatch_tests 600 $PYT -m gpu tests/test_host_memory.py tests/test_dispatcher.py \
                      tests/test_dispatch_async.py tests/test_config5_sharded.py tests/test_rawpacket.py ;;
    # the dispatcher leg alone (host bundles, 1/2/4 shards on one GPU), in its torch-free child
    bench_dispatch) step bench_dispatch 600 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e &&
                    tail -1 "$O/bench_dispatch.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())
for k, v in (d["dispatch"] or {}).items():
    if isinstance(v, dict): print(k, v.get("directional_pps"), v.get("host_ms_per_bundle"))' | tee "$O/dispatch.txt" ;;
    smoke)        step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)        step bench 300 $BENCH --steps 20 --warmup 5 && tail -1 "$O/bench.log" > "$O/bench.json" ;;
    bench_fused)  SRTP_TEST_DEBUG=4 step bench_fused 300 $BENCH --steps 20 --warmup 5 ;;
    bench_serial) step bench_serial 300 $BENCH --steps 20 --warmup 5 --serial ;;
    bench_default) step bench_default 600 python bench.py && tail -1 "$O/bench_default.log" > "$O/bench_default.json" ;;
    trace)        step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
                      python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial ;;
    trace_default) step trace_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_default" \
                      -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch &&
                   python tools/timeline.py "$(find "$O/trace_default" -name '*kernel_trace.csv' | head -1)" 10 \
                      > "$O/timeline.txt" && head -14 "$O/timeline.txt" ;;
    # bundle-size sweep, serial (one stream), of the split path (debug 2), the
    # fused / small-bundle path (debug 4) and the default
    size_sweep)   for n in ${SWEEP_SIZES:-1024 4096 8192 16384 32768 65536 131072 262144}; do
                      for d in 4 2; do
                          SRTP_TEST_DEBUG=$d step sweep_${n}_$d 200 $BENCH --steps 20 --warmup 3 --serial --packets $n \
                              --ssrcs $(( n < 10000 ? n : 10000 )) || return 1
                          echo "n=$n dbg=$d $(tail -1 $O/sweep_${n}_$d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"])')" >> $O/sweep.txt
                      done
                  done; cat $O/sweep.txt ;;
    # counters of one build's crypto kernels on the serial bench (separate --pmc
    # passes); PROF_DEBUG=2 profiles the split path on the full bundle
    prof)         local S="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --no-dispatch --serial"
                  local P="$O/prof"
                  export SRTP_TEST_DEBUG=${PROF_DEBUG:-0}
                  step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$P/trace" -o run -- \
                      python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch --serial &&
                  step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$P/fetch" -o run -- $S &&
                  step prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$P/write" -o run -- $S &&
                  step prof_sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
                      SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$P/sq" -o run -- $S &&
                  step prof_sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
                      SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE \
                      --output-format csv -d "$P/sq2" -o run -- $S
                  local rc=$?
                  unset SRTP_TEST_DEBUG
                  return $rc ;;
    # the split path on the full bundle, serial stage timings: this build and
    # each variant in $VARIANTS (libjitsi_amd/variants/libsrtp_<v>.so), twice
    ab_wide)      for k in 1 2; do
                      SRTP_TEST_DEBUG=2 step ab_wide_cur_$k 200 $BENCH --steps 20 --warmup 3 --serial || return 1
                      for v in ${VARIANTS:-}; do
                          SRTP_TEST_DEBUG=2 SRTP_MI355X_LIB=libjitsi_amd/variants/libsrtp_$v.so \
                              step ab_wide_${v}_$k 200 $BENCH --steps 20 --warmup 3 --serial || return 1
                      done
                  done
                  for f in $O/ab_wide_*.log; do
                      echo "$(basename $f .log) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["stage_ms"])')"
                  done | tee $O/ab_wide.txt ;;
    *) echo "unknown recipe $1"; return 2 ;;
    esac
}

for r in "$@"; do
    recipe "$r" || { echo "recipe $r failed: stopping"; exit 1; }
done
echo "all done"
