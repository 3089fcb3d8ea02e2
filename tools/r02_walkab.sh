#!/bin/bash
# Walk hand-off A/B: GPU parity suite, then stage timings and the default bench
# line of the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02_walkab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
[ $rc -ne 0 ] && exit 1
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 100 --no-cpu --no-e2e > $O/bench$k.log 2>&1 || exit 1
  python -c "import json; l=[x for x in open('$O/bench$k.log') if x.startswith('{')][-1]; j=json.loads(l); print(j['value']/1e6, j['ms_per_step'], j['stage_ms'])"
done
timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e --zipf 1.1 > $O/zipf.log 2>&1 && python -c "import json; l=[x for x in open('$O/zipf.log') if x.startswith('{')][-1]; j=json.loads(l); print('zipf', j['value']/1e6, j['stage_ms'])"
timeout -k 10 200 python bench.py --steps 20 --no-cpu --no-e2e --ssrcs 1 > $O/one.log 2>&1 && python -c "import json; l=[x for x in open('$O/one.log') if x.startswith('{')][-1]; j=json.loads(l); print('one', j['value']/1e6, j['stage_ms'])"
exit 0
