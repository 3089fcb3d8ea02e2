#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02_skew
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "" "--zipf 1.1" "--ssrcs 1" "--ssrcs 100"; do
  name=$(echo "x$cfg" | tr -d ' -')
  timeout -k 10 250 python bench.py --steps 20 --warmup 5 --no-cpu --no-e2e $cfg > $O/$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.]*\|"stage_ms": {[^}]*}' $O/$name.log | tr '\n' ' ')"
done
