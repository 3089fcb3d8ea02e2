#!/bin/bash
# Round 5: the driver's default bench invocation, timed.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05def
mkdir -p $O
s=$(date +%s.%N)
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
e=$(date +%s.%N)
python3 -c "print('wall_s', round($e - $s, 1))" | tee $O/wall.txt
python3 -c "
import json; d = json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'steps', d['steps'], 'frac', d['roofline']['frac'], 'stale', d['roofline'].get('traffic_stale'))
print('dispatch 1', d['dispatch']['1']['directional_pps'], '1_async', d['dispatch']['1_async']['directional_pps'])
"
