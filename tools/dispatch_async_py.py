"""Dispatcher host bundles from Python, synchronous and two in flight, with
and without two other engines (and their streams) alive in the process --
the bench's dispatcher leg runs after the headline's sender and receiver
engines.  Prints one JSON line per (extra engines, mode).

    python tools/dispatch_async_py.py [bundle operations per mode] [--no-torch] [--lib-first]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from libjitsi_amd import (HostBuffer, SRTPContextFactory, SRTPDispatcher, SRTPEngine,  # noqa: E402
                          SRTPTransformer, profile_policies, synth)


def hip_runtime():
    """The libamdhip64 this process mapped: torch's wheel ships its own (ROCm
    7.0) with the same SONAME as /opt/rocm's, so whichever loads first serves
    both torch and libsrtp_mi355x."""
    with open("/proc/self/maps") as f:
        paths = {ln.split()[-1] for ln in f if "libamdhip64" in ln}
    return sorted(paths)


def run(ops, extra, use_torch=True):
    if use_torch:
        import torch
        torch.cuda.init()
    keep = [SRTPEngine(device=0, max_contexts=1 << 14, max_batch=1 << 18) for _ in range(extra)]
    pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
    b = synth.rtp_bundle(1 << 18, 10000, 1200, seed=synth.SEED_BASE + 2)
    d = SRTPDispatcher([0], check_replay=False, max_contexts=1 << 15, max_factories=8, max_transformers=8)
    (k, s), = synth.keys(2, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=d))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=d))
    hbs = [HostBuffer(b.seg.nbytes), HostBuffer(b.seg.nbytes)]
    bufs = []
    for hb in hbs:
        hb.array[:] = b.seg
        bufs.append((hb.array, b.length.copy()))
    for sg, ln in bufs:  # warm
        d.transform_host(False, snd.tid, sg, b.off, ln, b.cap)
        d.transform_host(True, rcv.tid, sg, b.off, ln, b.cap)
    out = []
    t0 = time.perf_counter()
    for i in range(ops):
        sg, ln = bufs[0]
        st = d.transform_host(bool(i & 1), (rcv if i & 1 else snd).tid, sg, b.off, ln, b.cap)
        assert not st.any()
    dt = time.perf_counter() - t0
    out.append({"torch": use_torch, "hip": hip_runtime(), "extra_engines": extra, "mode": "sync", "pps_per_direction": round(ops * b.n / dt, 1),
                "ms_per_op": round(dt / ops * 1e3, 3)})
    pending, t_sub = [], []
    t0 = time.perf_counter()
    for i in range(ops):
        rev = bool((i >> 1) & 1)
        sg, ln = bufs[i & 1]
        if len(pending) == 2:
            assert not pending.pop(0).wait().any()
        a = time.perf_counter()
        pending.append(d.submit_host(rev, (rcv if rev else snd).tid, sg, b.off, ln, b.cap))
        t_sub.append(time.perf_counter() - a)
    for tk in pending:
        assert not tk.wait().any()
    dt = time.perf_counter() - t0
    out.append({"torch": use_torch, "extra_engines": extra, "mode": "async2", "pps_per_direction": round(ops * b.n / dt, 1),
                "ms_per_op": round(dt / ops * 1e3, 3), "submit_ms_p50": round(float(np.median(t_sub)) * 1e3, 3)})
    d.close()
    for hb in hbs:
        hb.close()
    for e in keep:
        e.close()
    return out


if __name__ == "__main__":
    ops = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    use_torch = "--no-torch" not in sys.argv
    if "--lib-first" in sys.argv:  # libsrtp_mi355x (and /opt/rocm's HIP runtime) before torch
        from libjitsi_amd import _native
        _native.lib()
    for extra in (0, 2):
        for line in run(ops, extra, use_torch):
            print(json.dumps(line), flush=True)
