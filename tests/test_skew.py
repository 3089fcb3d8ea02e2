"""GPU: skewed bundles -- one SSRC, or a Zipf popularity over many -- where a
context's chain of packets in one bundle is far longer than k_walk's LDS
window and goes through the wave-parallel walk (srtp_kernels.hip walk_long).

The serial dependency being parallelised is SRTPCryptoContext's per-packet
state machine (guessIndex :457-475, checkReplay :279-323, update :719-744).
Every bundle is checked bit-exact against the oracle (statuses, lengths,
segment bytes, context state): long in-order runs, sequence wraps (ROC
changes inside the chain, with tag re-checks and re-decryption), and the
packets that break the speculation -- tampered tags, exact replays,
reordered and stale packets, capacity errors, malformed packets without
abort-on-throw, replay checking off -- plus a long SRTCP chain.
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
P32 = profile_policies("AES_CM_128_HMAC_SHA1_32")


def faults(b, rng, frac=0.002, ssrc_seq=True):
    """Tamper, replay, reorder and stale packets at `frac` each."""
    n = b.n
    order = np.arange(n)
    for i in rng.choice(n - 20, int(frac * n), replace=False):  # reorder within 8
        j = i + int(rng.integers(1, 8))
        order[i], order[j] = order[j], order[i]
    dup = rng.choice(n, int(frac * n), replace=False)           # exact replays, later
    order = np.insert(order, np.minimum(dup + 50, n), dup)
    fb = synth.select(b, order)
    o = fb.off.astype(np.int64)
    for i in rng.choice(fb.n, int(frac * fb.n), replace=False):  # tamper
        fb.seg[o[i] + int(rng.integers(12, max(13, fb.length[i] - 1)))] ^= 0x10
    return fb


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 15, max_factories=256, max_transformers=256,
                          max_batch=1 << 17)


def test_one_ssrc_65536_packets_with_wraps(engine):
    twin = Twin(engine)
    (k, s), = synth.keys(201, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(1 << 16, 1, (60, 400), seed=202, seq0=[60000])  # wraps at packet 5536
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    seg2, ln2, st2 = twin.run(rcv, True, seg, b.off, ln, b.cap)
    assert (st2 == 0).all() and np.array_equal(ln2, b.length)
    assert engine.context_state(rcv.e, int(b.ssrc[0]))["roc"] == 1
    # the next bundle of the same stream, now with faults on the wire
    b2 = synth.rtp_bundle(40000, 1, (60, 400), seed=203, ssrcs=b.meta["ssrcs"],
                          seq0=[(60000 + (1 << 16)) & 0xFFFF])
    p2, pl2, ps2 = twin.run(snd, False, b2.seg, b2.off, b2.length, b2.cap)
    assert (ps2 == 0).all()
    pb = b2.copy()
    pb.seg, pb.length = p2, pl2
    fb = faults(pb, np.random.default_rng(204))
    _, _, st3 = twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap)
    assert (st3 == N.STATUS_DROP_AUTH).any() and (st3 == N.STATUS_DROP_REPLAY).any()
    assert (st3 == 0).sum() > 0.98 * b2.n


def test_zipf_mix_over_10k_ssrcs(engine):
    twin = Twin(engine)
    (k, s), = synth.keys(205, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle_skewed(1 << 17, 10000, (100, 1300), seed=206, zipf_s=1.1)
    counts = np.bincount(np.unique(b.ssrc, return_inverse=True)[1])
    assert counts.max() > 10000  # the top SSRC's chain is ~40x the LDS window
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap, check_state=False)
    assert (st == 0).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = faults(pb, np.random.default_rng(207), frac=0.001)
    _, _, st2 = twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, check_state=False)
    # state of the heaviest streams and a sample of the rest
    top = np.unique(b.ssrc)[np.argsort(-counts)[:20]]
    rng = np.random.default_rng(208)
    for ssrc in list(top) + list(rng.choice(np.unique(b.ssrc), 200, replace=False)):
        for t in (snd, rcv):
            so, se = t.o.state(int(ssrc)), engine.context_state(t.e, int(ssrc))
            assert (so is None) == (se is None)
            if so is not None:
                for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
                    assert int(so[key]) == int(se[key]), (hex(int(ssrc)), key, so, se)


def test_long_chain_breakers(engine_factory, oracle):
    """Capacity errors (protect), malformed packets without abort-on-throw,
    replay checking off, and a first packet (seqNumSet) inside long chains."""
    for check_replay in (True, False):
        eng = engine_factory(abort_on_error=False, check_replay=check_replay,
                             max_contexts=1024, max_factories=64, max_transformers=64)
        twin = Twin(eng, check_replay=check_replay)
        try:
            (k, s), = synth.keys(209, 1)
            fs, fr = twin.factory(True, k, s, *P32), twin.factory(False, k, s, *P32)
            snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
            b = synth.rtp_bundle(6000, 2, (60, 300), seed=210, seq0=[65000, 100])
            cap = b.cap.copy()
            cap[1000:1010] = ((b.length[1000:1010] + 15) // 16 * 16).astype(np.uint32)
            cap[1000:1010] = np.minimum(cap[1000:1010], b.length[1000:1010] + 2)  # no room for the tag
            o = b.off.astype(np.int64)
            b.seg[o[3000:3006]] = 0x8F  # CC=15: the cipher throws (no abort)
            b.length[3000:3006] = 60
            seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, cap, abort_on_error=False)
            assert (st == N.STATUS_ERR_CAPACITY).any() and (st == N.STATUS_ERR_MALFORMED).any()
            pb = b.copy()
            pb.seg, pb.length = seg, ln
            fb = faults(pb, np.random.default_rng(211), frac=0.01)
            twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, abort_on_error=False)
        finally:
            O.set_check_replay(True)


def test_long_srtcp_chain(engine):
    twin = Twin(engine)
    (k, s), = synth.keys(212, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    cs, cr = twin.transformer(O.KIND_RTCP, fs), twin.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(3000, 1, seed=213)
    seg, ln, st = twin.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    rb = synth.select(pc, np.r_[0:3000, 100:130, 2990:3000])
    twin.run(cr, True, rb.seg, rb.off, rb.length, rb.cap)


def test_multi_wrap_chain_with_loss(engine):
    """One SSRC wrapping twice within one bundle, received with 45% loss and
    light reordering.  k_unprotect guesses the ROC of a packet deep in a long
    chain from its rank in the chain; with this much loss the guess drifts
    more than half a wrap behind the true index for the later packets, so the
    walk overturns those guesses and re-checks their tags -- slower, and
    still bit-exact."""
    twin = Twin(engine)
    (k, s), = synth.keys(214, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(1 << 17, 1, (60, 200), seed=215, seq0=[40000])  # wraps at 25536, 91072
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    rng = np.random.default_rng(216)
    keep = np.sort(rng.choice(b.n, int(0.55 * b.n), replace=False))
    fb = faults(synth.select(pb, keep), rng, frac=0.001)
    _, _, st2 = twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap)
    assert (st2 == 0).sum() > 0.99 * keep.size
    assert engine.context_state(rcv.e, int(b.ssrc[0]))["roc"] == 2


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_chains_around_tile_size(engine, seed):
    """Chains of 250..520 packets (around the walk's 256-record tile), so that
    long chains start, end and break at every position of a tile, next to
    short ones: the chain pass (per-tile speculation with look-back) against
    the oracle in both directions, with first packets of new streams (no
    seqNumSet yet), replays / tampering / reordering, a receiver that misses
    every 97th packet, and a second bundle continuing the same streams."""
    rng = np.random.default_rng(300 + seed)
    lens = [int(x) for x in rng.integers(250, 521, 14)] + [int(x) for x in rng.integers(1, 40, 30)]
    chains_roundtrip(engine, rng, 310 + seed, lens, 0.003)


@pytest.mark.parametrize("seed", [0, 1])
def test_medium_chains(engine, seed):
    """Chains of 24..260 packets: around the first pass's one-lane / whole-wave
    threshold (32) and up to the chain pass's (256), several starting in one
    tile, with the same first packets, faults and lost packets as above."""
    rng = np.random.default_rng(400 + seed)
    lens = ([int(x) for x in rng.integers(24, 40, 24)] + [int(x) for x in rng.integers(40, 261, 30)] +
            [int(x) for x in rng.integers(1, 24, 30)])
    chains_roundtrip(engine, rng, 410 + seed, lens, 0.01)
    # each new stream's first packet (no seqNumSet) is walked one at a time
    assert engine.stats()["long_walked"] > 0


def chains_roundtrip(engine, rng, key_seed, lens, frac, stalls_expected=False):
    twin = Twin(engine)
    (k, s), = synth.keys(key_seed, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    ssrcs = rng.choice(1 << 30, len(lens), replace=False).astype(np.uint32) + 1000
    for rnd in range(2):
        parts = []
        for i, L in enumerate(lens):
            seq0 = np.array([int(rng.integers(0, 65536)) if rnd == 0 else 0], np.uint32)
            parts.append(synth.rtp_bundle(L, 1, (40, 300), seed=int(rng.integers(1 << 30)),
                                          ssrcs=ssrcs[i:i + 1], seq0=seq0))
        if rnd == 1:  # continue each stream where the first bundle left it
            for i, pb in enumerate(parts):
                st = twin.engine.context_state(snd.e, int(ssrcs[i]))
                q = (int(st["s_l"]) + 1 + np.arange(pb.n)) & 0xFFFF
                for j in range(pb.n):
                    pb.seg[pb.off[j] + 2] = q[j] >> 8
                    pb.seg[pb.off[j] + 3] = q[j] & 0xFF
        b = synth.concat(parts)
        perm = rng.permutation(b.n)  # interleave streams, each in its own order
        owner = np.concatenate([np.full(p.n, i) for i, p in enumerate(parts)])[perm]
        base = np.cumsum([0] + [p.n for p in parts])
        order = np.empty(b.n, int)
        for i in range(len(parts)):
            order[owner == i] = base[i] + np.arange(parts[i].n)
        b = synth.select(b, order)
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
        assert (st == 0).all()
        pb = b.copy()
        pb.seg, pb.length = seg, ln
        keep = np.ones(pb.n, bool)
        keep[::97] = False
        fb = faults(synth.select(pb, np.nonzero(keep)[0]), rng, frac=frac)
        twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap)
    if not stalls_expected:
        assert engine.stats()["chain_stalls"] == 0


def test_forced_chain_stall_stays_exact(engine_factory, oracle):
    """A chain-pass tile that gives up its look-back (a tile preempted for
    seconds) leaves its part of the chain to the fix-up run by the last tile
    to finish, which walks it from the exact state the tile before published.
    The test hook makes every third tile give up at once; every bundle must
    still match the oracle bit for bit, and the stall counter must show that
    the fix-up ran.  Chains: one SSRC over many tiles with wraps, Zipf heads,
    and chains around the tile size with faults."""
    eng = engine_factory(max_contexts=1 << 15, max_factories=64, max_transformers=64,
                         max_batch=1 << 17)
    eng.set_debug(N.DEBUG_FORCE_CHAIN_STALL)
    twin = Twin(eng)
    (k, s), = synth.keys(501, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(1 << 15, 1, (60, 300), seed=502, seq0=[50000])  # 128 tiles, one wrap
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = faults(pb, np.random.default_rng(503), frac=0.002)
    _, _, st2 = twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap)
    assert (st2 == 0).sum() > 0.99 * b.n
    assert not (st2 == N.STATUS_ERR_INTERNAL).any()
    zb = synth.rtp_bundle_skewed(1 << 16, 2000, (100, 600), seed=504, zipf_s=1.1)
    zseg, zln, zst = twin.run(snd, False, zb.seg, zb.off, zb.length, zb.cap, check_state=False)
    pz = zb.copy()
    pz.seg, pz.length = zseg, zln
    twin.run(rcv, True, pz.seg, pz.off, pz.length, pz.cap, check_state=False)
    for ssrc in np.unique(zb.ssrc)[:300]:
        for t in (snd, rcv):
            so, se = t.o.state(int(ssrc)), eng.context_state(t.e, int(ssrc))
            assert (so is None) == (se is None)
            if so is not None:
                for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
                    assert int(so[key]) == int(se[key]), (hex(int(ssrc)), key, so, se)
    rng = np.random.default_rng(505)
    lens = [int(x) for x in rng.integers(250, 900, 10)] + [int(x) for x in rng.integers(1, 40, 20)]
    chains_roundtrip(eng, rng, 506, lens, 0.003, stalls_expected=True)
    assert eng.stats()["chain_stalls"] > 0
    assert eng.stats()["status"]["ERR_INTERNAL"] == 0
