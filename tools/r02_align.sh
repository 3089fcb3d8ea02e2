#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r02_align
for a in 16 128 256 16 128 256; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-e2e --align $a > gpurun_out/r02_align/$a.log 2>&1 || exit $?
  python - "$a" gpurun_out/r02_align/$a.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[1], d["value"], d["ms_per_step"], d["stage_ms"])
PY
done
