#!/bin/bash
# Round 5: the bench's stream-ordering events with a device-scope release
# against torch.cuda.Event (system scope), alternating on one box, and a
# two-stream kernel trace with the device-scope events.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R5TAG:-r05i}
mkdir -p $O
B="python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --no-dispatch"
for r in 1 2; do
  for ev in device torch; do
    timeout -k 10 200 $B --events $ev > $O/bench_${ev}_$r.log 2>&1 || exit $?
    tail -1 $O/bench_${ev}_$r.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$ev', j['value']/1e6, j['ms_per_step'], j['all_accepted'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_dev -o run -- python3 bench.py --steps 20 --warmup 2 --no-cpu --no-e2e --no-dispatch > $O/trace_dev.log 2>&1 || exit $?
python3 tools/timeline.py $(find $O/trace_dev -name "*kernel_trace.csv" | head -1) 10 > $O/timeline_dev.txt && head -14 $O/timeline_dev.txt
