"""Host-side SSRC sharding across GPUs, Python view of the
dispatcher's plan in ``libjitsi_amd/csrc/dispatch.cpp``.

SRTP contexts are independent per (transformer, SSRC) -- SRTPTransformer keeps
one context per SSRC and nothing else is shared except the read-only factory
keys (transform/srtp/SRTPTransformer.java:62,152-175).  So a bundle splits
into per-GPU sub-bundles by hashing the SSRC; each GPU owns its shard's
context state and no collective is needed on the data path.  Packets keep
their relative order inside a shard, which is all the per-context state
machine depends on.

``plan`` calls the product's own split (``srtp_dispatch_plan``, C ABI, runs
without a GPU): the shard of every packet and whether it could throw, which
decides the transformers whose contexts the dispatcher snapshots so that it
can roll back their packets after a throw on another shard
(SinglePacketTransformer's abort-on-throw, dispatch.cpp).  ``split`` /
``merge`` are the per-shard index lists and their inverse.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import _native as N


def shard_of_ssrc(ssrc: int, world: int) -> int:
    """srtp_shard_of: murmur3 fmix32(SSRC) mod world."""
    return int(N.lib().srtp_shard_of(int(ssrc) & 0xFFFFFFFF, int(world)))


def plan(world: int, seg: np.ndarray, off: np.ndarray, length: np.ndarray, cap: np.ndarray,
         kinds: Sequence[int], tids=0, flags=None, reverse: bool = False,
         abort_on_error: bool = True, tag_lens: Sequence[int] = (10,)):
    """(shard[n], may_throw[n], runs) of a bundle, as srtp_dispatch_transform_host
    splits it (runs = 2 when some packet could throw: contexts are snapshotted
    and a rollback re-run may follow).  ``tids`` is one transformer id or one
    per packet; ``kinds[t]`` is transformer t's kind; ``tag_lens`` the tag
    lengths of the policies in use."""
    n = len(off)
    seg = np.ascontiguousarray(seg, np.uint8)
    off = np.ascontiguousarray(off, np.uint32)
    length = np.ascontiguousarray(length, np.uint32)
    cap = np.ascontiguousarray(cap, np.uint32)
    kinds_a = np.ascontiguousarray(kinds, np.int32)
    fl = None if flags is None else np.ascontiguousarray(flags, np.uint32)
    if np.isscalar(tids):
        tids_p, tid0 = None, int(tids)
    else:
        tids_a = np.ascontiguousarray(tids, np.int32)
        tids_p, tid0 = tids_a.ctypes.data, -1
    mask = 0
    for t in tag_lens:
        mask |= 1 << int(t)
    shard = np.zeros(n, np.int32)
    may_throw = np.zeros(n, np.int32)
    rc = N.lib().srtp_dispatch_plan(int(world), int(abort_on_error), int(reverse),
                                    kinds_a.ctypes.data, len(kinds_a), mask, tids_p, tid0,
                                    seg.ctypes.data, seg.nbytes, off.ctypes.data,
                                    length.ctypes.data, cap.ctypes.data,
                                    None if fl is None else fl.ctypes.data, n,
                                    shard.ctypes.data, may_throw.ctypes.data)
    N.check(rc, None, "srtp_dispatch_plan")
    return shard, may_throw, int(rc)


def split(shard: np.ndarray, world: int) -> List[np.ndarray]:
    """Packet indices per shard, each in original (array) order."""
    return [np.nonzero(shard == r)[0] for r in range(world)]


def merge(parts: List[np.ndarray], idx: List[np.ndarray], n: int) -> np.ndarray:
    """Scatter per-shard results (e.g. statuses) back into bundle order."""
    out = np.empty(n, dtype=parts[0].dtype if parts else np.int32)
    for p, i in zip(parts, idx):
        out[i] = p
    return out
