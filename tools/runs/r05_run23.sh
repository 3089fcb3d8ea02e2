#!/bin/bash
# Round 5: dispatcher two-in-flight mode -- C++ vs Python, with and without torch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05w}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 120 ./tools/dispatch_bench 16 1 > $O/dispatch_bench.jsonl 2>&1 || exit $?
cat $O/dispatch_bench.jsonl
timeout -k 10 300 python3 tools/dispatch_async_py.py 16 --no-torch > $O/py_notorch.jsonl 2>&1 || exit $?
cat $O/py_notorch.jsonl
timeout -k 10 300 python3 tools/dispatch_async_py.py 16 > $O/py_torch.jsonl 2>&1 || exit $?
cat $O/py_torch.jsonl
