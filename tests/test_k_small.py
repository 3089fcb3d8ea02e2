"""GPU: k_small -- a bundle of up to 255 packets in one workgroup and one launch.

The per-packet callers' bundles (a lone synchronous call is a bundle of one)
are small; k_small runs the split path's phases for them behind barriers
instead of kernel boundaries: parse, an in-LDS rank sort, the tag check
(unprotect), the walk (wave 0: one tile; abort-on-throw's dry and limit passes
back to back), the keystream over every lane, and the MAC and trailer
(protect).  Every bundle here is compared with the oracle bit for bit
(statuses, lengths, the whole segment, context state), and the engine's
counters show which path ran it (srtp_stats.small_bundles).  The other GPU
parity tests take it too whenever their bundles are this small.
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

import test_gpu_parity as G
from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
P32 = profile_policies("AES_CM_128_HMAC_SHA1_32")
PNULL80 = profile_policies("NULL_HMAC_SHA1_80")


def small_count(eng):
    return eng.stats()["small_bundles"]


@pytest.fixture(params=[True, False], ids=["abort", "no_abort"])
def twin(request, engine_factory, oracle):
    e = engine_factory(abort_on_error=request.param, max_contexts=1 << 12, max_factories=64,
                       max_transformers=128)
    t = Twin(e)
    t.abort = request.param
    return t


def test_which_bundles_take_one_launch(engine_factory, oracle):
    """1 and 255 packets: k_small; 256: the multi-kernel chain; a key set
    outside the split path's rule (F8) or SRTP_DEBUG_NO_SMALL: the chain."""
    eng = engine_factory(max_contexts=1 << 12, max_factories=16, max_transformers=16)
    twin = Twin(eng)
    (k, s), = synth.keys(5000, 1)
    f = twin.factory(True, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    seq0 = np.array([100, 200, 300], np.uint32)
    for n, small in ((1, True), (255, True), (256, False), (7, True)):
        b = synth.rtp_bundle(n, 3, 200, seed=5000 + n, seq0=seq0)
        seq0 = seq0 + (n + 2) // 3 + 1
        c0 = small_count(eng)
        twin.run(t, False, b.seg, b.off, b.length, b.cap)
        assert small_count(eng) - c0 == (1 if small else 0), n
    eng.set_debug(N.DEBUG_NO_SMALL)
    b = synth.rtp_bundle(5, 3, 200, seed=5999, seq0=seq0)
    c0 = small_count(eng)
    twin.run(t, False, b.seg, b.off, b.length, b.cap)
    assert small_count(eng) == c0
    eng.set_debug(0)
    # an F8 key set in the engine: its bundles keep the chain
    ff = twin.factory(True, k, s, *G.PF8)
    tf = twin.transformer(O.KIND_RTP, ff)
    b = synth.rtp_bundle(4, 2, 200, seed=5998, ssrcs=[0x5000, 0x5001])
    c0 = small_count(eng)
    twin.run(tf, False, b.seg, b.off, b.length, b.cap)
    assert small_count(eng) == c0


@pytest.mark.parametrize("n", [1, 2, 31, 32, 63, 64, 65, 128, 200, 255])
def test_round_trips_with_faults(twin, n):
    """n mixed-size packets over several transformers and key sets (_80, _32),
    a few invalid or skipped, protect, then unprotect with tampering, a replay
    and reordering, then the same packets again (all replays)."""
    rng = np.random.default_rng(5100 + n)
    facs = []
    for j in range(3):
        (k, s), = synth.keys(5100 + 7 * n + j, 1)
        pols = P32 if j == 2 else P80
        facs.append((twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols)))
    snd = [twin.transformer(O.KIND_RTP, f[0]) for f in facs]
    rcv = [twin.transformer(O.KIND_RTP, f[1]) for f in facs]
    n_ssrc = max(1, min(12, n // 4))
    b = synth.rtp_bundle(n, n_ssrc, (40, 1400), seed=5200 + n, ext_frac=0.1,
                         ssrcs=[0x7000 + 64 * n + i for i in range(n_ssrc)])
    who = (np.arange(n) % n_ssrc) % 3
    flags = np.zeros(n, np.uint32)
    ln = b.length.copy()
    if n >= 32:
        ln[rng.choice(n, 1)] = 8                   # RawPacket.isInvalid
        flags[rng.choice(n, 1)] = N.PKT_FLAG_SKIP
    c0 = small_count(twin.engine)
    seg, ln2, st = twin.run([snd[w] for w in who], False, b.seg, b.off, ln, b.cap, flags,
                            abort_on_error=twin.abort)
    assert small_count(twin.engine) == c0 + 1
    seg = seg.copy()
    ok = np.nonzero(st == N.STATUS_OK)[0]
    order = np.arange(n)
    if len(ok) > 3:
        seg[int(b.off[ok[len(ok) // 2]]) + 13] ^= 2          # a forged header byte
        seg[int(b.off[ok[-1]]) + int(ln2[ok[-1]]) - 1] ^= 1  # a tag bit
        order = np.concatenate([order, [ok[0]]])             # an exact replay at the end
        if n > 8:
            order[[1, 5]] = order[[5, 1]]                    # reordered
    rseg, roff, rln, rcap = _gather(seg, b.off, ln2, b.cap, order)
    rwho = who[order]
    rflags = flags[order]
    twin.run([rcv[w] for w in rwho], True, rseg, roff, rln, rcap, rflags, abort_on_error=twin.abort)
    _, _, st3 = twin.run([rcv[w] for w in rwho], True, rseg, roff, rln, rcap, rflags,
                         abort_on_error=twin.abort)
    assert (st3 == N.STATUS_OK).sum() == 0
    # (255 packets plus the replay: 256, the chain's)
    assert small_count(twin.engine) == c0 + (3 if len(order) <= 255 else 1)
    for t in snd + rcv:
        t.close()


def _gather(seg, off, ln, cap, order):
    """The packets `order` (indices may repeat) packed into a new segment."""
    caps = cap[order].astype(np.int64)
    room = (caps + 15) // 16 * 16
    noff = np.concatenate([[0], np.cumsum(room[:-1])]).astype(np.uint32)
    out = np.zeros(int(room.sum()), np.uint8)
    for j, i in enumerate(order):
        out[int(noff[j]):int(noff[j]) + int(cap[i])] = seg[int(off[i]):int(off[i]) + int(cap[i])]
    return out, noff, ln[order].copy(), cap[order].copy()


@pytest.mark.parametrize("n,seq0", [(64, 65500), (255, 65400), (255, 100), (40, 65535)])
def test_one_stream_chains(twin, n, seq0):
    """One SSRC carrying the whole bundle (a medium chain of 32+ records:
    walk_long inside k_small's wave 0), across the sequence wrap (ROC + 1),
    then unprotected in two bundles with faults."""
    (k, s), = synth.keys(5300 + n, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(n, 1, (100, 1200), seed=5300 + n, seq0=np.array([seq0], np.uint32),
                         ssrcs=[0x9000 + seq0])
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap, abort_on_error=twin.abort)
    assert (st == N.STATUS_OK).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = G.inject_faults(pb, np.random.default_rng(5300 + n))
    h = fb.n // 2
    for idx in (np.arange(h), np.arange(h, fb.n)):
        sub = synth.select(fb, idx)
        twin.run(rcv, True, sub.seg, sub.off, sub.length, sub.cap, abort_on_error=twin.abort)


def test_srtp_and_srtcp_one_bundle(twin):
    """SRTP and SRTCP of _80, _32 and NULL-cipher key sets in one small
    bundle each way (the kinds' IVs, E bit and index words)."""
    facs = []
    for j, pols in enumerate((P80, P32, PNULL80)):
        (k, s), = synth.keys(5400 + j, 1)
        facs.append((twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols)))
    rtp = synth.rtp_bundle(90, 9, (60, 1000), seed=5401, ssrcs=[0xA000 + i for i in range(9)])
    rtcp = synth.rtcp_bundle(30, 6, seed=5402)
    both = synth.concat([rtp, rtcp])
    n, seg, off, ln, cap = both.n, both.seg, both.off, both.length, both.cap
    ts = [twin.transformer(O.KIND_RTP, f[0]) for f in facs] + [twin.transformer(O.KIND_RTCP, f[0]) for f in facs]
    tr = [twin.transformer(O.KIND_RTP, f[1]) for f in facs] + [twin.transformer(O.KIND_RTCP, f[1]) for f in facs]
    who = np.concatenate([np.arange(rtp.n) % 3, 3 + np.arange(rtcp.n) % 3])
    c0 = small_count(twin.engine)
    seg2, ln2, st = twin.run([ts[w] for w in who], False, seg, off, ln, cap, abort_on_error=twin.abort)
    assert (st == N.STATUS_OK).all()
    seg2 = seg2.copy()
    seg2[int(off[n - 1]) + 9] ^= 1  # an SRTCP packet forged
    twin.run([tr[w] for w in who], True, seg2, off, ln2, cap, abort_on_error=twin.abort)
    assert small_count(twin.engine) == c0 + 2


def test_malformed_packets(twin):
    """The reference's drops and throws (Q15, Q17) in a small bundle: with
    abort-on-throw the dry walk and the limit walk run in k_small's wave 0."""
    (k, s), = synth.keys(5500, 1)
    f = twin.factory(True, k, s, *P80)
    fr = twin.factory(False, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    r = twin.transformer(O.KIND_RTP, fr)
    pk = G.malformed_bundle()
    caps = np.array([(c + 15) // 16 * 16 for _, c in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(caps[:-1])]).astype(np.uint32)
    seg = np.zeros(int(caps.sum()), np.uint8)
    ln = np.array([len(p) for p, _ in pk], np.uint32)
    for i, (p, _) in enumerate(pk):
        seg[off[i]:off[i] + len(p)] = np.frombuffer(p, np.uint8)
    c0 = small_count(twin.engine)
    for _ in range(2):
        seg2, ln2, _ = twin.run(t, False, seg, off, ln, caps, abort_on_error=twin.abort)
        twin.run(r, True, seg2, off, ln2, caps, abort_on_error=twin.abort)
    tc = twin.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(6, 2, len_range=(12, 24), seed=3)
    twin.run(tc, True, cb.seg, cb.off, cb.length, cb.cap, abort_on_error=twin.abort)
    assert small_count(twin.engine) == c0 + 5
