"""GPU: seeded randomized parity of the engine against the CPU oracle.

Each round draws a bundle mixing RTP and RTCP packets of several
transformers (AES-CM _80/_32, AES-F8, NULL-cipher profiles), random sizes,
header extensions, DISCARD/SILENCE/SKIP flags and null elements; the
protected output is then faulted (bit flips, replays, reordering, stale
packets, truncations) and unprotected.  SDES-style factory swaps and
DTLS-style transformer replacements happen between rounds.  Every bundle must
agree with the oracle bit for bit (statuses, lengths, whole segment, context
state) -- Twin.run asserts it.
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O
from harness import Twin

pytestmark = pytest.mark.gpu

PROFILES = ["AES_CM_128_HMAC_SHA1_80", "AES_CM_128_HMAC_SHA1_32", "F8_128_HMAC_SHA1_80",
            "NULL_HMAC_SHA1_80"]


def make_pair(twin, kind, prof, key_seed):
    (k, s), = synth.keys(key_seed, 1)
    pols = profile_policies(prof)
    fs, fr = twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols)
    return {"kind": kind, "prof": prof, "s": twin.transformer(kind, fs),
            "r": twin.transformer(kind, fr)}


def fault(b, rng, per_pkt_ts):
    """Reorder, replay, drop stale copies in, flip bits, truncate some packets."""
    n = b.n
    order = list(range(n))
    for i in range(n):
        if rng.random() < 0.08:
            j = min(n - 1, i + int(rng.integers(1, 12)))
            order[i], order[j] = order[j], order[i]
    out = []
    for pos, i in enumerate(order):
        out.append(i)
        r = rng.random()
        if r < 0.03:
            out.append(i)
        elif r < 0.04 and pos > 80:
            out.append(order[pos - int(rng.integers(66, 80))])
    fb = synth.select(b, np.array(out))
    ts = [per_pkt_ts[i] for i in out]
    for i in range(fb.n):
        L = int(fb.length[i])
        r = rng.random()
        if r < 0.03 and L > 0:
            fb.seg[fb.off[i] + int(rng.integers(0, L))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif r < 0.04:
            fb.length[i] = np.uint32(max(0, L - int(rng.integers(1, 30))))
    return fb, ts


@pytest.mark.parametrize("seed,abort,check_replay",
                         [(1, True, True), (2, True, True), (3, True, True), (4, False, True),
                          (5, True, False)])
def test_randomized_mixed_bundles(engine_factory, oracle, seed, abort, check_replay):
    eng = engine_factory(max_contexts=1 << 14, max_factories=256, max_transformers=256,
                         max_batch=1 << 14, abort_on_error=abort, check_replay=check_replay)
    twin = Twin(eng, check_replay=check_replay)
    rng = np.random.default_rng(9000 + seed)
    pairs = [make_pair(twin, kind, prof, 900 + 10 * seed + j)
             for j, (kind, prof) in enumerate((k, p) for p in PROFILES for k in (0, 1))]
    seq_base = int(rng.integers(0, 65536))
    seen = set()
    for rnd in range(5):
        if rnd == 2:  # SDES-style: new factories swapped into two transformers
            for pr in pairs[:2]:
                (k, s), = synth.keys(950 + seed, 1)
                pols = profile_policies(pr["prof"])
                pr["s"].set_factory(twin.factory(True, k, s, *pols), True)
                pr["r"].set_factory(twin.factory(False, k, s, *pols), False)
        if rnd == 3:  # DTLS-style: a brand-new transformer pair
            pairs[4] = make_pair(twin, pairs[4]["kind"], pairs[4]["prof"], 970 + seed)
        parts, ts_s, ts_r = [], [], []
        for j, pr in enumerate(pairs):
            n_j = int(rng.integers(20, 200))
            if pr["kind"] == 0:
                bj = synth.rtp_bundle(n_j, 5, (12, 1400), seed=1000 * seed + 10 * rnd + j,
                                      ext_frac=0.2, ssrcs=np.arange(5, dtype=np.uint32) + 40 * j,
                                      seq0=np.full(5, (seq_base + 40 * rnd) & 0xFFFF, np.uint32))
            else:
                bj = synth.rtcp_bundle(n_j, 3, (12, 300), seed=2000 * seed + 10 * rnd + j,
                                       ssrcs=np.arange(3, dtype=np.uint32) + 40 * j)
            parts.append(bj)
            ts_s += [pr["s"]] * bj.n
            ts_r += [pr["r"]] * bj.n
        b = synth.concat(parts)
        perm = rng.permutation(b.n)
        b = synth.select(b, perm)
        ts_s = [ts_s[i] for i in perm]
        ts_r = [ts_r[i] for i in perm]
        flags = np.zeros(b.n, np.uint32)
        flags[rng.random(b.n) < 0.02] = N.PKT_FLAG_SKIP
        for i in np.nonzero(rng.random(b.n) < 0.01)[0]:
            ts_s[i] = None  # null elements of the RawPacket[] array
        seg, ln, st = twin.run(ts_s, False, b.seg, b.off, b.length, b.cap, flags=flags,
                               abort_on_error=abort)
        pb = b.copy()
        pb.seg, pb.length = seg, ln
        fb, ts_f = fault(pb, rng, ts_r)
        fl = np.zeros(fb.n, np.uint32)
        fl[rng.random(fb.n) < 0.05] = N.PKT_FLAG_SILENCE
        fl[rng.random(fb.n) < 0.03] = N.PKT_FLAG_DISCARD
        _, _, st_r = twin.run(ts_f, True, fb.seg, fb.off, fb.length, fb.cap, flags=fl,
                              abort_on_error=abort)
        seen |= set(int(v) for v in st) | set(int(v) for v in st_r)
    O.set_check_replay(True)
    # the mix really exercised the drop paths, not only clean round trips (SRTCP
    # replay checks are not config-gated, so replays show up either way)
    assert {N.STATUS_OK, N.STATUS_DROP_AUTH, N.STATUS_DROP_REPLAY, N.STATUS_SKIPPED} <= seen, seen
