#!/bin/bash
# Round-2 final evidence of the committed tree: GPU tests, smoke, the serial
# line, skew / stream-count bench points, rocprofv3 kernel traces (default and
# --serial) and PMC passes (serial, as the roofline's stage timing).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=gpurun_out/r02c
mkdir -p $P
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "$P/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc"; tail -2 "$P/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP after $name ($rc)"; exit $rc; fi
  return $rc
}
S="python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial"
run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
run trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --serial || exit 1
run fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o run -- $S || exit 1
run write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o run -- $S || exit 1
run sq 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $P/sq -o run -- $S || exit 1
run sq2 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq2 -o run -- $S || exit 1
run pmc_summary 120 python tools/pmc_summary.py $P --out $P/summary || exit 1  # also writes profiles/pmc_traffic.json, read by the bench line
run bench 400 python bench.py || exit 1
run bench_steps20 300 python bench.py --steps 20 --no-cpu --no-e2e || exit 1
run bench_zipf 300 python bench.py --steps 20 --no-cpu --no-e2e --zipf 1.1 || exit 1
run bench_one 300 python bench.py --steps 20 --no-cpu --no-e2e --ssrcs 1 || exit 1
run bench_100k 300 python bench.py --steps 20 --no-cpu --no-e2e --ssrcs 100000 || exit 1
run trace_default 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace_default -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e || exit 1
python tools/timeline.py $(find $P/trace_default -name "*kernel_trace.csv" | head -1) 10 > $P/timeline.txt; cat $P/timeline.txt | head -12
echo all done
