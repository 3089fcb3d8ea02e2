#!/bin/bash
# A/B: default engine vs a variant build (tools/ab/libsrtp_<v>.so) on the default bench
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_prio
for v in cur "$@" cur "$@"; do
  lib=""; [ "$v" != cur ] && lib="$PWD/tools/ab/libsrtp_$v.so"
  SRTP_MI355X_LIB=$lib timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-e2e > gpurun_out/r02_prio/$v.log 2>&1 || exit $?
  python - "$v" gpurun_out/r02_prio/$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], d["ms_per_step"], d["stage_ms"], d["roofline"]["kernel"], d["roofline"]["frac"])
PY
done
