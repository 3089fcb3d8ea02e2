#!/bin/bash
# Per-kernel durations of the skewed bench points (serial run: one engine at a time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02_skewprof
mkdir -p $O
for m in one zipf; do
  a="--ssrcs 1"; [ $m = zipf ] && a="--zipf 1.1"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$m -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --serial $a > $O/$m.log 2>&1 || exit 1
  f=$(find $O/$m -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    print('$m', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
