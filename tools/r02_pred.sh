#!/bin/bash
# long-chain ROC guess check: parity subset, then bench points (uniform and skewed)
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/r02_pred
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_skew.py tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "" "--zipf 1.1" "--ssrcs 1" "--ssrcs 100" ""; do
  name=$(echo "x$cfg" | tr -d ' -')
  timeout -k 10 250 python bench.py --steps 50 --warmup 5 --no-cpu --no-e2e $cfg > $O/$name.log 2>&1 || exit $?
  echo "$name $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' $O/$name.log | tr '\n' ' ')"
done
