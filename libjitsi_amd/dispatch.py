"""Host-side SSRC sharding across GPUs.

SRTP contexts are independent per (transformer, SSRC) -- SRTPTransformer keeps
one context per SSRC and nothing else is shared except the read-only factory
keys (transform/srtp/SRTPTransformer.java:62,152-175).  So a bundle splits
into per-GPU sub-bundles by hashing the SSRC; each GPU owns its shard's
context state and no collective is needed on the data path.  Packets keep
their relative order inside a shard, which is all the per-context state
machine depends on.
"""
from __future__ import annotations

from typing import List

import numpy as np


def mix32(x: np.ndarray) -> np.ndarray:
    """murmur3 fmix32 finaliser (uint32 -> uint32)."""
    x = np.asarray(x, dtype=np.uint64) & 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & 0xFFFFFFFF
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & 0xFFFFFFFF
    x ^= x >> 16
    return x.astype(np.uint32)


def packet_ssrc(seg: np.ndarray, off: np.ndarray, rtcp: np.ndarray = None) -> np.ndarray:
    """RawPacket.getSSRC (bytes 8..11) or getRTCPSSRC (bytes 4..7) per packet."""
    o = off.astype(np.int64)
    base = o + 8 if rtcp is None else o + np.where(rtcp, 4, 8)
    b = [seg[base + k].astype(np.uint32) for k in range(4)]
    return (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3]


def shard_of(ssrc: np.ndarray, world: int) -> np.ndarray:
    return (mix32(ssrc) % np.uint32(world)).astype(np.int32)


def split(ssrc: np.ndarray, world: int) -> List[np.ndarray]:
    """Packet indices per shard, each in original (array) order."""
    sh = shard_of(ssrc, world)
    return [np.nonzero(sh == r)[0] for r in range(world)]


def merge(parts: List[np.ndarray], idx: List[np.ndarray], n: int) -> np.ndarray:
    """Scatter per-shard results (e.g. statuses) back into bundle order."""
    out = np.empty(n, dtype=parts[0].dtype if parts else np.int32)
    for p, i in zip(parts, idx):
        out[i] = p
    return out
