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
    # small bundles on the multi-kernel chain (k_small off: SRTP_DEBUG_NO_SMALL)
    parity_nosmall) SRTP_TEST_DEBUG=8 step parity_nosmall 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_golden.py \
                      tests/test_small_bundles.py tests/test_single_packet.py tests/test_fuzz_parity.py ;;
    dispatch_tests) step dispatch_tests 600 $PYT -m gpu tests/test_host_memory.py tests/test_dispatcher.py \
                      tests/test_dispatch_async.py tests/test_config5_sharded.py tests/test_rawpacket.py ;;
    # the dispatcher leg alone (host bundles, 1/2/4 shards on one GPU), in its torch-free child
    bench_dispatch) step bench_dispatch 600 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e &&
                    tail -1 "$O/bench_dispatch.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())
for k, v in (d["dispatch"] or {}).items():
    if isinstance(v, dict): print(k, v.get("directional_pps"), v.get("host_ms_per_bundle"))' | tee "$O/dispatch.txt" ;;
    # the per-packet drop-in path (tools/sync_bench): a lone caller and 64
    # synchronous callers (protect + unprotect round trips), arrays through
    # the aggregator, and the queued path at the JNI shim's sizing and larger
    sync)         : > "$O/sync.jsonl"
                  # points as path_shards_threads[_rt]
                  for p in ${SYNC_POINTS:-one_0_1_rt one_0_64_rt arrayq_0_64}; do
                      step sync_pt 90 ./tools/sync_bench 2 ${p//_/ } && cat "$O/sync_pt.log" >> "$O/sync.jsonl" || return 1
                  done
                  for cfg in ${SYNC_CFGS:-"4096,8,6 64" "4096,8,6 256" "16384,24,8 64" "16384,24,8 256"}; do
                      set -- ${cfg//_/ }
                      SYNC_AGG=$1 SYNC_DEPTH=$2 step sync_q 90 ./tools/sync_bench 2 queue 0 64 ${SYNC_QMODE:-rt} || return 1
                      python3 -c "import json; j=json.loads(open('$O/sync_q.log').read().strip().splitlines()[-1]); j['agg']='$1'; j['depth']=$2; j['path'] += '${SYNC_DEBUG:+_dbg$SYNC_DEBUG}' + ('_${SYNC_QMODE}' if '${SYNC_QMODE:-rt}' != 'rt' else ''); print(json.dumps(j))" >> "$O/sync.jsonl"
                  done
                  python3 -c "
import json
for l in open('$O/sync.jsonl'):
    j = json.loads(l); print(j['path'], j['threads'], j.get('agg', ''), j.get('depth', ''), 'calls/s', j['calls_per_s'], 'p50', j['lat_us']['p50'], 'pkts/bundle', j.get('packets_per_bundle'))" ;;
    # the same points for this build and each aggregator variant in $AGG_VARIANTS
    # (tools/build_agg_variant.sh: libjitsi_amd/variants/agg_<v>/, swapped in by LD_LIBRARY_PATH)
    agg_ab)       : > "$O/agg_ab.jsonl"
                  for v in cur ${AGG_VARIANTS:-}; do
                      local lp=""; [ "$v" != cur ] && lp="libjitsi_amd/variants/agg_$v"
                      for p in ${SYNC_POINTS:-one_0_64_rt one_0_256_rt}; do
                          LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} SYNC_AGG=${PT_AGG:-} step ab_pt 90 ./tools/sync_bench 2 ${p//_/ } || return 1
                          python3 -c "import json; j=json.loads(open('$O/ab_pt.log').read().strip().splitlines()[-1]); j['variant']='$v'; j['agg']='${PT_AGG:-}'; print(json.dumps(j))" >> "$O/agg_ab.jsonl"
                      done
                      for cfg in ${SYNC_CFGS:-"16384,24,8 64" "16384,24,8 256"}; do
                          set -- ${cfg//_/ }
                          LD_LIBRARY_PATH=$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} SYNC_AGG=$1 SYNC_DEPTH=$2 \
                              step ab_q 90 ./tools/sync_bench 2 queue 0 64 rt || return 1
                          python3 -c "import json; j=json.loads(open('$O/ab_q.log').read().strip().splitlines()[-1]); j['agg']='$1'; j['depth']=$2; j['variant']='$v'; print(json.dumps(j))" >> "$O/agg_ab.jsonl"
                      done
                  done
                  python3 -c "
import json
for l in open('$O/agg_ab.jsonl'):
    j = json.loads(l); print(j['variant'], j['path'], j['threads'], j.get('agg', ''), j.get('depth', ''), 'calls/s', j['calls_per_s'], 'p50', j['lat_us']['p50'], 'pkts/bundle', j.get('packets_per_bundle'))" | tee "$O/agg_ab.txt" ;;
    # the default bench step (two streams), this build against each $VARIANTS
    # library, alternating, three times each
    ab_bench)     for k in 1 2 3; do
                      step ab_bench_cur_$k 200 $BENCH --steps 50 --warmup 5 || return 1
                      for v in ${VARIANTS:-}; do
                          SRTP_MI355X_LIB=libjitsi_amd/variants/libsrtp_$v.so \
                              step ab_bench_${v}_$k 200 $BENCH --steps 50 --warmup 5 || return 1
                      done
                  done
                  for f in $O/ab_bench_*.log; do
                      echo "$(basename $f .log) $(tail -1 $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["stage_ms"])')"
                  done | tee $O/ab_bench.txt ;;
    # a kernel + copy trace of one synchronous caller (the lone call's chain)
    # (TRACE_LIBDIR: a directory holding another libsrtp_mi355x.so to trace instead)
    trace_lone)   LD_LIBRARY_PATH=${TRACE_LIBDIR:-}${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH} \
                  step trace_lone 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
                      -d "$O/trace_lone" -o run -- ./tools/sync_bench 1 one 0 1 rt &&
                  python3 tools/lone_chain.py "$O/trace_lone" | tee "$O/lone_chain.txt" ;;
    small_tests)  step small_tests 600 $PYT -m gpu tests/test_k_small.py tests/test_small_bundles.py \
                      tests/test_gpu_parity.py tests/test_single_packet.py tests/test_aggregator.py ;;
    # kernel statistics of one sync_bench point (TRACE_ARGS, default: 256
    # synchronous callers), and the GPU's busy fractions over the window
    trace_sync)   step trace_sync 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
                      -d "$O/trace_sync" -o run -- ./tools/sync_bench 1 ${TRACE_ARGS:-one 0 256 rt} &&
                  f=$(find "$O/trace_sync" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -20 &&
                  python3 tools/trace_busy.py "$O/trace_sync" > "$O/trace_sync_busy.txt" 2>&1; cat "$O/trace_sync_busy.txt" | tail -25 ;;
    agg_tests)    step agg_tests 600 $PYT -m gpu tests/test_aggregator.py tests/test_single_packet.py tests/test_jni_shim.py \
                      tests/test_rawpacket.py tests/test_pipeline.py ;;
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
