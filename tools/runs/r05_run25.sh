#!/bin/bash
# Round 5: is the Python two-in-flight slowdown torch's bundled HIP runtime
# (ROCm 7.0, torch/lib/libamdhip64.so)?  torch loaded first, libsrtp_mi355x's
# NEEDED libamdhip64.so.7 resolves to torch's copy (same SONAME).
#  1. the C++ dispatch_bench on torch's runtime (symlinked as libamdhip64.so.7)
#  2. the Python probe with torch first (shared 7.0 runtime)
#  3. the Python probe with libsrtp_mi355x loaded first (it keeps /opt/rocm's 7.2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${R5TAG:-r05y}
O=gpurun_out/$T
mkdir -p $O
TL=$(python3 -c "import importlib.util, os; print(os.path.join(os.path.dirname(importlib.util.find_spec('torch').origin), 'lib'))")
H=/tmp/hip70_$$
mkdir -p $H
for f in libamdhip64.so libhsa-runtime64.so libamd_comgr.so librocprofiler-register.so; do ln -sf $TL/$f $H/$f; done
ln -sf $TL/libamdhip64.so $H/libamdhip64.so.7
LD_LIBRARY_PATH=$H ldd tools/dispatch_bench | grep -E "hip|hsa" > $O/cpp_hip70_ldd.txt
LD_LIBRARY_PATH=$H timeout -k 10 120 ./tools/dispatch_bench 16 1 > $O/cpp_hip70.jsonl 2>&1 || exit $?
cat $O/cpp_hip70_ldd.txt $O/cpp_hip70.jsonl
timeout -k 10 120 ./tools/dispatch_bench 16 1 > $O/cpp_hip72.jsonl 2>&1 || exit $?
cat $O/cpp_hip72.jsonl
timeout -k 10 300 python3 tools/dispatch_async_py.py 16 > $O/py_torch_torchfirst.jsonl 2>&1 || exit $?
cat $O/py_torch_torchfirst.jsonl
timeout -k 10 300 python3 tools/dispatch_async_py.py 16 --lib-first > $O/py_torch_libfirst.jsonl 2>&1 || exit $?
cat $O/py_torch_libfirst.jsonl
