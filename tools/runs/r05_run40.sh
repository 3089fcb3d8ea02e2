#!/bin/bash
# Round 5: the in-process multi-device bench (two sides on device 0) with the
# torch-free dispatcher child over two shards.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05inproc
mkdir -p $O
SRTP_BENCH_INPROC=1 SRTP_BENCH_ONE_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --no-e2e --dispatch-shards 2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'n_gpus', d['n_gpus'])
print({k: (v.get('directional_pps') if isinstance(v, dict) else v) for k, v in d['dispatch'].items()})
print({k: (v.get('directional_pps') if isinstance(v, dict) else v) for k, v in (d['dispatch_in_torch_process'] or {}).items()})
"
