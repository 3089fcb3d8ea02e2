#!/bin/bash
# Round 5: the bench's dispatcher leg in its torch-free child process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05z}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-e2e > $O/bench_child.json 2> $O/bench_child.err || { tail -20 $O/bench_child.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_child.json').read().strip().splitlines()[-1])
print('value', d['value'])
for k in ('dispatch', 'dispatch_in_torch_process'):
    for m, v in (d[k] or {}).items():
        print(k, m, v if not isinstance(v, dict) else (v.get('directional_pps'), v.get('async_ops'), v.get('all_accepted')))
"
# the headline step from C++ on /opt/rocm's runtime and on torch's
TL=$(python3 -c "import importlib.util, os; print(os.path.join(os.path.dirname(importlib.util.find_spec('torch').origin), 'lib'))")
H=/tmp/hip70_$$
mkdir -p $H
for f in libamdhip64.so libhsa-runtime64.so libamd_comgr.so librocprofiler-register.so; do ln -sf $TL/$f $H/$f; done
ln -sf $TL/libamdhip64.so $H/libamdhip64.so.7
for r in 1 2; do
timeout -k 10 180 ./tools/device_bench > $O/device_hip72_$r.json 2>&1 || { cat $O/device_hip72_$r.json; exit 1; }
LD_LIBRARY_PATH=$H timeout -k 10 180 ./tools/device_bench > $O/device_hip70_$r.json 2>&1 || { cat $O/device_hip70_$r.json; exit 1; }
done
cat $O/device_hip7*.json
