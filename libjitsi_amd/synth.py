"""Deterministic synthetic SRTP workloads.

Seeds are ``0x5EED0000 + config_no``.  Packets of one SSRC appear in sequence
order; SSRCs are interleaved round-robin in a bundle.  Header: V=2, PT 111
(audio) / 96 (video), seq, ts = seq * ts_step, SSRC; payload bytes random.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

SEED_BASE = 0x5EED0000


@dataclass
class Bundle:
    seg: np.ndarray        # uint8 packed segment
    off: np.ndarray        # uint32, 16-B aligned
    length: np.ndarray     # uint32
    cap: np.ndarray        # uint32
    flags: np.ndarray      # uint32
    ssrc: np.ndarray       # uint32 per packet
    seq: np.ndarray        # uint32 per packet
    meta: dict = field(default_factory=dict)

    @property
    def n(self):
        return len(self.off)

    def copy(self) -> "Bundle":
        return Bundle(self.seg.copy(), self.off.copy(), self.length.copy(), self.cap.copy(),
                      self.flags.copy(), self.ssrc.copy(), self.seq.copy(), dict(self.meta))

    def packet(self, i: int) -> bytes:
        return self.seg[self.off[i]:self.off[i] + self.length[i]].tobytes()


def distinct_u32(rng: np.random.Generator, n: int) -> np.ndarray:
    out = np.unique(rng.integers(1, 2**32, size=int(n * 1.1) + 16, dtype=np.uint64).astype(np.uint32))
    while len(out) < n:
        out = np.unique(np.concatenate([out, rng.integers(1, 2**32, size=n, dtype=np.uint64)
                                        .astype(np.uint32)]))
    return rng.permutation(out)[:n]


def keys(seed: int, n: int = 1):
    """n (master key 16 B, master salt 14 B) pairs."""
    rng = np.random.default_rng(seed ^ 0xC0FFEE)
    return [(rng.integers(0, 256, 16, dtype=np.uint8).tobytes(),
             rng.integers(0, 256, 14, dtype=np.uint8).tobytes()) for _ in range(n)]


def layout(length: np.ndarray, room: int = 16):
    cap = ((length.astype(np.int64) + room + 15) // 16 * 16).astype(np.uint32)
    off = np.zeros(len(length), np.uint64)
    if len(length) > 1:
        off[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    total = int(off[-1] + cap[-1]) if len(length) else 16
    assert total < 2**32, "bundle larger than 4 GiB"
    return off.astype(np.uint32), cap, total


def rtp_bundle(n_packets: int, n_ssrc: int, pkt_len, seed: int, pt: int = 96,
               ts_step: int = 3000, seq0=None, ssrcs=None, ext_frac: float = 0.0) -> Bundle:
    """RTP packets: packet i belongs to SSRC i % n_ssrc, seq = seq0 + i // n_ssrc.
    pkt_len is an int or a (lo, hi) inclusive range.  ext_frac of the packets
    carry a one-element RFC 5285 header extension (X bit, 8 extra bytes)."""
    rng = np.random.default_rng(seed)
    if ssrcs is None:
        ssrcs = distinct_u32(rng, n_ssrc)
    ssrcs = np.asarray(ssrcs, np.uint32)
    if seq0 is None:
        seq0 = rng.integers(0, 65536, n_ssrc, dtype=np.uint32)
    seq0 = np.asarray(seq0, np.uint32)
    idx = np.arange(n_packets, dtype=np.int64)
    s = idx % n_ssrc
    seq = ((seq0[s].astype(np.int64) + idx // n_ssrc) & 0xFFFF).astype(np.uint32)
    if isinstance(pkt_len, tuple):
        length = rng.integers(pkt_len[0], pkt_len[1] + 1, n_packets, dtype=np.int64).astype(np.uint32)
    else:
        length = np.full(n_packets, pkt_len, np.uint32)
    off, cap, total = layout(length)
    seg = rng.integers(0, 256, total, dtype=np.uint8)
    o = off.astype(np.int64)
    has_ext = rng.random(n_packets) < ext_frac if ext_frac > 0 else np.zeros(n_packets, bool)
    has_ext &= length >= 24
    seg[o] = np.where(has_ext, 0x90, 0x80).astype(np.uint8)
    seg[o + 1] = pt & 0x7F
    seg[o + 2] = (seq >> 8).astype(np.uint8)
    seg[o + 3] = (seq & 0xFF).astype(np.uint8)
    ts = (seq.astype(np.uint64) * ts_step) & 0xFFFFFFFF
    for k in range(4):
        seg[o + 4 + k] = ((ts >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
        seg[o + 8 + k] = ((ssrcs[s] >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
    e = o[has_ext]
    seg[e + 12] = 0xBE
    seg[e + 13] = 0xDE
    seg[e + 14] = 0
    seg[e + 15] = 1  # one 32-bit word of extension data
    return Bundle(seg, off, length, cap, np.zeros(n_packets, np.uint32), ssrcs[s].copy(), seq,
                  {"ssrcs": ssrcs, "seq0": seq0, "seed": seed})


def rtp_bundle_skewed(n_packets: int, n_ssrc: int, pkt_len, seed: int, zipf_s: float = 1.1,
                      pt: int = 96, ts_step: int = 3000) -> Bundle:
    """RTP packets whose SSRCs follow a Zipf(zipf_s) popularity over n_ssrc
    streams (rank r has weight 1 / r^s), in random interleaving; each SSRC's
    packets carry consecutive sequence numbers in bundle order.  meta["counts"]
    holds each packet's SSRC's packet count in the bundle (the per-bundle
    sequence advance)."""
    rng = np.random.default_rng(seed)
    ssrcs = distinct_u32(rng, n_ssrc)
    w = 1.0 / np.arange(1, n_ssrc + 1, dtype=np.float64) ** zipf_s
    s = rng.choice(n_ssrc, size=n_packets, p=w / w.sum())
    seq0 = rng.integers(0, 65536, n_ssrc, dtype=np.uint32)
    order = np.argsort(s, kind="stable")
    rank = np.empty(n_packets, np.int64)
    counts = np.bincount(s, minlength=n_ssrc)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    rank[order] = np.arange(n_packets) - np.repeat(starts, counts)
    seq = ((seq0[s].astype(np.int64) + rank) & 0xFFFF).astype(np.uint32)
    length = (np.full(n_packets, pkt_len, np.uint32) if not isinstance(pkt_len, tuple) else
              rng.integers(pkt_len[0], pkt_len[1] + 1, n_packets, dtype=np.int64).astype(np.uint32))
    off, cap, total = layout(length)
    seg = rng.integers(0, 256, total, dtype=np.uint8)
    o = off.astype(np.int64)
    seg[o] = 0x80
    seg[o + 1] = pt & 0x7F
    seg[o + 2] = (seq >> 8).astype(np.uint8)
    seg[o + 3] = (seq & 0xFF).astype(np.uint8)
    ts = (seq.astype(np.uint64) * ts_step) & 0xFFFFFFFF
    for k in range(4):
        seg[o + 4 + k] = ((ts >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
        seg[o + 8 + k] = ((ssrcs[s] >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
    return Bundle(seg, off, length, cap, np.zeros(n_packets, np.uint32), ssrcs[s].copy(), seq,
                  {"ssrcs": ssrcs, "seq0": seq0, "seed": seed, "counts": counts[s].astype(np.int64),
                   "zipf_s": zipf_s})


def rtcp_bundle(n_packets: int, n_ssrc: int, len_range=(28, 200), seed: int = 0,
                ssrcs=None) -> Bundle:
    """RTCP SR/RR-shaped packets (V=2, PT 200/201, length field), random body."""
    rng = np.random.default_rng(seed)
    if ssrcs is None:
        ssrcs = distinct_u32(rng, n_ssrc)
    ssrcs = np.asarray(ssrcs, np.uint32)
    idx = np.arange(n_packets)
    s = idx % n_ssrc
    length = (rng.integers(len_range[0], len_range[1] + 1, n_packets) // 4 * 4).astype(np.uint32)
    length = np.maximum(length, 12).astype(np.uint32)
    off, cap, total = layout(length)
    seg = rng.integers(0, 256, total, dtype=np.uint8)
    o = off.astype(np.int64)
    seg[o] = 0x80
    seg[o + 1] = np.where(rng.random(n_packets) < 0.5, 200, 201).astype(np.uint8)
    words = (length // 4 - 1).astype(np.uint32)
    seg[o + 2] = (words >> 8).astype(np.uint8)
    seg[o + 3] = (words & 0xFF).astype(np.uint8)
    for k in range(4):
        seg[o + 4 + k] = ((ssrcs[s] >> (24 - 8 * k)) & 0xFF).astype(np.uint8)
    return Bundle(seg, off, length, cap, np.zeros(n_packets, np.uint32), ssrcs[s].copy(),
                  np.zeros(n_packets, np.uint32), {"ssrcs": ssrcs, "seed": seed})


def concat(bundles) -> Bundle:
    """Concatenate bundles into one segment (offsets rebased)."""
    segs, offs, base = [], [], 0
    for b in bundles:
        segs.append(b.seg)
        offs.append(b.off.astype(np.uint64) + base)
        base += len(b.seg)
    return Bundle(np.concatenate(segs), np.concatenate(offs).astype(np.uint32),
                  np.concatenate([b.length for b in bundles]),
                  np.concatenate([b.cap for b in bundles]),
                  np.concatenate([b.flags for b in bundles]),
                  np.concatenate([b.ssrc for b in bundles]),
                  np.concatenate([b.seq for b in bundles]), {})


def realign(b: Bundle, align: int) -> Bundle:
    """The same packets with every region starting on an `align`-byte boundary
    (caps unchanged; the gap after each region is zero)."""
    if align <= 16:
        return b
    stride = ((b.cap.astype(np.int64) + align - 1) // align) * align
    off = np.zeros(b.n, np.int64)
    if b.n > 1:
        off[1:] = np.cumsum(stride[:-1])
    seg = np.zeros(int(off[-1] + stride[-1]) if b.n else 16, np.uint8)
    src = b.off.astype(np.int64)
    if b.n and np.all(b.cap == b.cap[0]):  # vectorised for uniform caps
        c = int(b.cap[0])
        idx = src[:, None] + np.arange(c)[None, :]
        seg[(off[:, None] + np.arange(c)[None, :]).ravel()] = b.seg[idx.ravel()]
    else:
        for i in range(b.n):
            seg[off[i]:off[i] + b.cap[i]] = b.seg[src[i]:src[i] + b.cap[i]]
    return Bundle(seg, off.astype(np.uint32), b.length.copy(), b.cap.copy(), b.flags.copy(),
                  b.ssrc.copy(), b.seq.copy(), dict(b.meta))


def select(b: Bundle, order: np.ndarray) -> Bundle:
    """Re-pack packets of b in the given order (indices may repeat: duplicates)."""
    order = np.asarray(order, np.int64)
    length = b.length[order].copy()
    cap = b.cap[order].copy()
    off = np.zeros(len(order), np.uint64)
    if len(order) > 1:
        off[1:] = np.cumsum(cap[:-1].astype(np.uint64))
    total = int(off[-1] + cap[-1]) if len(order) else 16
    seg = np.zeros(total, np.uint8)
    for j, i in enumerate(order):
        seg[off[j]:off[j] + cap[j]] = b.seg[b.off[i]:b.off[i] + b.cap[i]]
    return Bundle(seg, off.astype(np.uint32), length, cap, b.flags[order].copy(),
                  b.ssrc[order].copy(), b.seq[order].copy(), dict(b.meta))
