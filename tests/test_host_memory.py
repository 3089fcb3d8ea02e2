"""GPU: registered and engine-pinned host memory (srtp_host_register /
srtp_host_alloc, round 4) -- the ranges the dispatcher moves by DMA in place.

The registry's rules: ranges may not overlap, unregister takes the registered
pointer, an engine-allocated range is freed (not unregistered), and a bundle
wholly inside one range counts as registered.  Then a bundle in a HostBuffer
through one and two shards, bit for bit against the oracle (the in-place DMA
path and, over two shards, the copy path for chunks whose packets are not
back to back).
"""
import ctypes as C

import numpy as np
import pytest

from libjitsi_amd import (HostBuffer, SRTPDispatcher, host_is_registered, host_register, host_unregister,
                          profile_policies, synth)
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
EINVAL = -1  # SRTP_EINVAL


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")


def test_registry_rules():
    _gpu()
    L = N.lib()
    a = np.zeros(1 << 20, np.uint8)
    assert not host_is_registered(a)
    host_register(a)
    try:
        assert host_is_registered(a)
        assert L.srtp_host_is_registered(a.ctypes.data + 4096, 1000) == 1
        assert L.srtp_host_is_registered(a.ctypes.data + a.nbytes - 8, 16) == 0  # runs past the end
        # an overlapping range and a second registration are refused
        assert L.srtp_host_register(C.c_void_p(a.ctypes.data + 4096), 4096) == EINVAL
        assert L.srtp_host_register(C.c_void_p(a.ctypes.data), a.nbytes) == EINVAL
        # unregister takes the registered pointer only
        assert L.srtp_host_unregister(C.c_void_p(a.ctypes.data + 16)) == EINVAL
    finally:
        host_unregister(a)
    assert not host_is_registered(a)
    assert L.srtp_host_unregister(C.c_void_p(a.ctypes.data)) == EINVAL
    assert L.srtp_host_register(None, 16) == EINVAL
    # engine-allocated: registered, freed with srtp_host_free, not unregistered
    hb = HostBuffer(1 << 16)
    try:
        assert host_is_registered(hb.array)
        assert L.srtp_host_unregister(C.c_void_p(hb.array.ctypes.data)) == EINVAL
    finally:
        p = hb.array.ctypes.data
        hb.close()
    assert L.srtp_host_is_registered(C.c_void_p(p), 16) == 0
    assert L.srtp_host_free(C.c_void_p(p)) == EINVAL


class _InHostBuffer:
    """The dispatcher with every call's segment copied into a HostBuffer first
    (and the results copied out), as a caller whose packets live in the
    engine's pinned pool would run it."""

    def __init__(self, d):
        self._d = d

    def __getattr__(self, k):
        return getattr(self._d, k)

    def transform_host(self, reverse, tid, seg, off, length, cap, flags=None):
        hb = HostBuffer(seg.nbytes)
        try:
            hb.array[:] = seg
            st = self._d.transform_host(reverse, tid, hb.array, off, length, cap, flags)
            seg[:] = hb.array
            return st
        finally:
            hb.close()


@pytest.mark.parametrize("shards", [1, 2])
def test_dispatch_from_engine_pinned_memory(oracle, shards):
    _gpu()
    d = SRTPDispatcher([0] * shards, max_contexts=1 << 14, max_factories=16, max_transformers=16)
    try:
        twin = Twin(_InHostBuffer(d))
        (k, s), = synth.keys(91, 1)
        fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        b = synth.rtp_bundle(50000, 300, (60, 700), seed=92)  # two 2^15-packet chunks on one shard
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
        assert (st == N.STATUS_OK).all()
        seg = seg.copy()
        seg[int(b.off[40000]) + 20] ^= 1
        twin.run(rcv, True, seg, b.off, ln, b.cap)
    finally:
        d.close()


class _InRegistered:
    """The dispatcher with every call's segment in pageable memory registered
    for the call (srtp_host_register: mapped for the GPU too)."""

    def __init__(self, d):
        self._d = d

    def __getattr__(self, k):
        return getattr(self._d, k)

    def transform_host(self, reverse, tid, seg, off, length, cap, flags=None):
        buf = np.zeros(seg.nbytes + 8192, np.uint8)  # pageable, page-aligned view below
        a0 = (-buf.ctypes.data) % 4096
        arr = buf[a0:a0 + seg.nbytes]
        arr[:] = seg
        host_register(arr)
        try:
            st = self._d.transform_host(reverse, tid, arr, off, length, cap, flags)
        finally:
            host_unregister(arr)
        seg[:] = arr
        return st


@pytest.mark.parametrize("shards,pinned", [(2, False), (3, True), (4, False)])
def test_dispatch_gathers_interleaved_registered_bundles(oracle, shards, pinned):
    """A registered bundle over several shards: each shard's packets lie
    scattered over the caller's segment, and the GPU gathers them over PCIe
    and writes them back (srtp_pipeline_submit_gather, round 6) instead of a
    host copy through the pinned slots -- from the engine's pinned pool and
    from registered pageable memory, with a forged and a replayed packet and
    mixed lengths, bit for bit against the oracle; the dispatcher's host time
    spent copying packet bytes stays small."""
    _gpu()
    d = SRTPDispatcher([0] * shards, max_contexts=1 << 14, max_factories=16, max_transformers=16)
    try:
        twin = Twin(_InHostBuffer(d) if pinned else _InRegistered(d))
        (k, s), = synth.keys(93 + shards, 1)
        fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        b = synth.rtp_bundle(40000, 500, (60, 1300), seed=94 + shards)
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
        assert (st == N.STATUS_OK).all()
        prot = b.copy()
        prot.seg, prot.length = seg.copy(), ln.copy()
        prot.seg[int(prot.off[30000]) + 20] ^= 1          # a forgery
        idx = np.arange(40000)
        idx[100] = 99                                     # a replay
        r = synth.select(prot, idx)
        h0 = d.host_times()
        twin.run(rcv, True, r.seg, r.off, r.length, r.cap)
        h1 = d.host_times()
        # packing is now the per-packet arrays only: no 40-MB memcpy per direction
        assert (h1["pack_ms"] - h0["pack_ms"]) / max(h1["calls"] - h0["calls"], 1) < 20.0
    finally:
        d.close()
