"""GPU parity: the MI355X engine against the CPU oracle on identical inputs.

Bit-exact on everything observable: per-packet status, length, every byte of
the packed segment (ciphertext, tags, SRTCP E|index words, untouched bytes)
and the per-SSRC context state (ROC, s_l, replay window, SRTCP indices).
Scenarios follow BASELINE.json's configs at sizes the oracle finishes in
seconds, plus the edge cases of SURVEY.md 8a (Q1-Q17).
"""
import numpy as np
import pytest

from libjitsi_amd import SRTPPolicy, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu

P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
P32 = profile_policies("AES_CM_128_HMAC_SHA1_32")
PNULL80 = profile_policies("NULL_HMAC_SHA1_80")
PNULL32 = profile_policies("NULL_HMAC_SHA1_32")
PF8 = profile_policies("F8_128_HMAC_SHA1_80")
LIBSRTP_KEY = bytes.fromhex("E1F97A0D3E018BE0D64FA32C06DE4139")
LIBSRTP_SALT = bytes.fromhex("0EC675AD498AFEEBB6960B3AABE6")


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 16, max_factories=1 << 10, max_transformers=1 << 12)


@pytest.fixture
def twin(engine):
    return Twin(engine)


def one_packet(pkt: bytes, cap=None):
    cap = cap or ((len(pkt) + 16 + 15) // 16 * 16)
    seg = np.zeros(cap, np.uint8)
    seg[:len(pkt)] = np.frombuffer(pkt, np.uint8)
    return seg, np.array([0], np.uint32), np.array([len(pkt)], np.uint32), np.array([cap], np.uint32)


def test_libsrtp_vectors_on_gpu(twin):
    """Published libsrtp srtp_driver vectors (RFC 3711 B.3 master key)."""
    f = twin.factory(True, LIBSRTP_KEY, LIBSRTP_SALT, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    seg, off, ln, cap = one_packet(bytes.fromhex("800f1234decafbadcafebabe") + b"\xab" * 16)
    seg_e, len_e, st = twin.run(t, False, seg, off, ln, cap)
    assert st[0] == 0 and len_e[0] == 38
    assert seg_e[:38].tobytes().hex() == (
        "800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402b78d6acc99ea179b8dbb")
    tc = twin.transformer(O.KIND_RTCP, f)
    rtcp = bytes.fromhex("81c8000bcafebabe") + b"\xab" * 16
    seg = np.zeros(128, np.uint8)
    seg[:24] = np.frombuffer(rtcp, np.uint8)
    seg[64:88] = np.frombuffer(rtcp, np.uint8)
    seg_e, len_e, st = twin.run(tc, False, seg, np.array([0, 64], np.uint32),
                                np.array([24, 24], np.uint32), np.array([64, 64], np.uint32))
    assert seg_e[64:64 + 38].tobytes().hex() == (
        "81c8000bcafebabe7128035be487b9bdbef89041f977a5a880000001993e08cd54d6c1230798")


def round_trip(twin, pols, b, bundle_sizes, key_seed):
    (k, s), = synth.keys(key_seed, 1)
    fs = twin.factory(True, k, s, *pols)
    fr = twin.factory(False, k, s, *pols)
    snd = twin.transformer(O.KIND_RTP, fs)
    rcv = twin.transformer(O.KIND_RTP, fr)  # Q1: separate receiver transformer
    start = 0
    for nb in bundle_sizes:
        sub = synth.select(b, np.arange(start, min(start + nb, b.n)))
        start += nb
        seg, ln, st = twin.run(snd, False, sub.seg, sub.off, sub.length, sub.cap)
        assert (st == 0).all()
        seg2, ln2, st2 = twin.run(rcv, True, seg, sub.off, ln, sub.cap)
        assert (st2 == 0).all()
        np.testing.assert_array_equal(ln2, sub.length)
        for i in range(0, sub.n, max(1, sub.n // 17)):
            assert sub.packet(i) == seg2[sub.off[i]:sub.off[i] + ln2[i]].tobytes()
        if start >= b.n:
            break


def test_config1_single_ssrc_160B_with_wrap(twin):
    """C1: one SSRC, 160-B Opus packets, protect -> separate receiver -> unprotect,
    across a sequence-number wrap (ROC 0 -> 1)."""
    b = synth.rtp_bundle(3000, 1, 160, seed=synth.SEED_BASE + 1, pt=111, ts_step=960,
                         seq0=[65536 - 1200])
    round_trip(twin, P80, b, [1, 7, 100, 1000, 1892], key_seed=1)


def test_config2_video_1200B(twin):
    """C2: many SSRCs, 1200-B video packets, batched protect (+ unprotect)."""
    b = synth.rtp_bundle(8192, 500, 1200, seed=synth.SEED_BASE + 2)
    round_trip(twin, P80, b, [4096, 4096], key_seed=2)


@pytest.mark.parametrize("pols", [P32, PNULL80, PNULL32, PF8], ids=["_32", "NULL_80", "NULL_32", "F8_80"])
def test_profiles_round_trip(twin, pols):
    b = synth.rtp_bundle(3000, 37, (60, 1400), seed=synth.SEED_BASE + 4, ext_frac=0.1)
    round_trip(twin, pols, b, [1000, 2000], key_seed=4)


def protect_with_oracle(pols, b, key_seed, sender_tid=None):
    (k, s), = synth.keys(key_seed, 1)
    f = O.Factory(True, k, s, *[O.Policy(p.encType, p.encKeyLength, p.authType, p.authKeyLength,
                                         p.authTagLength, p.saltKeyLength) for p in pols])
    t = O.Transformer(O.KIND_RTP, f, f)
    seg, ln = b.seg.copy(), b.length.copy()
    st = O.process(t, False, seg, b.off, ln, b.cap)
    assert (st == 0).all()
    out = b.copy()
    out.seg, out.length = seg, ln
    return out, (k, s)


def inject_faults(b, rng, tag_len=10):
    """C3 fault mix on protected packets: 1% tamper (header/payload/tag bit
    flips), 1% exact replays, 0.5% stale replays (> 64 back), 5% reordered
    within 16."""
    n = b.n
    order = list(range(n))
    # reorder: swap with a neighbour up to 16 ahead
    for i in range(n):
        if rng.random() < 0.05:
            j = min(n - 1, i + int(rng.integers(1, 17)))
            order[i], order[j] = order[j], order[i]
    out = []
    for pos, i in enumerate(order):
        out.append(i)
        r = rng.random()
        if r < 0.01:
            out.append(i)  # exact replay
        elif r < 0.015 and pos > 200:
            out.append(order[pos - int(rng.integers(130, 200))])  # stale
    fb = synth.select(b, np.array(out))
    tampered = rng.random(fb.n) < 0.01
    for i in np.nonzero(tampered)[0]:
        L = int(fb.length[i])
        where = rng.integers(0, 3)
        if where == 0:
            pos = int(rng.integers(0, 12))
        elif where == 1:
            pos = int(rng.integers(12, L - tag_len))
        else:
            pos = int(rng.integers(L - tag_len, L))
        fb.seg[fb.off[i] + pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    return fb


def test_config3_mixed_sizes_unprotect_with_faults(twin):
    """C3: 60-1400 B, unprotect only, tamper/replay/stale/reorder, 5% of SSRCs
    starting near seq 65535, 10% with a header extension."""
    rng = np.random.default_rng(synth.SEED_BASE + 3)
    n_ssrc = 60
    seq0 = rng.integers(0, 65536, n_ssrc).astype(np.uint32)
    seq0[rng.random(n_ssrc) < 0.05] = 65530
    seq0[:3] = [65520, 65530, 65535]
    b = synth.rtp_bundle(6000, n_ssrc, (60, 1400), seed=synth.SEED_BASE + 3, seq0=seq0,
                         ext_frac=0.1)
    pb, (k, s) = protect_with_oracle(P80, b, key_seed=3)
    fb = inject_faults(pb, rng)
    fr = twin.factory(False, k, s, *P80)
    rcv = twin.transformer(O.KIND_RTP, fr)
    sizes = [1, 500, 2500, fb.n]
    start = 0
    seen = {}
    for nb in sizes:
        idx = np.arange(start, min(start + nb, fb.n))
        if len(idx) == 0:
            break
        start += len(idx)
        sub = synth.select(fb, idx)
        _, _, st = twin.run(rcv, True, sub.seg, sub.off, sub.length, sub.cap)
        for v in st:
            seen[int(v)] = seen.get(int(v), 0) + 1
    assert seen.get(N.STATUS_DROP_AUTH, 0) > 0 and seen.get(N.STATUS_DROP_REPLAY, 0) > 0
    assert seen.get(N.STATUS_OK, 0) > 0.9 * fb.n


def test_discard_silence_flags_skip_decrypt(twin):
    b = synth.rtp_bundle(400, 4, 300, seed=11)
    pb, (k, s) = protect_with_oracle(P80, b, key_seed=11)
    fr = twin.factory(False, k, s, *P80)
    rcv = twin.transformer(O.KIND_RTP, fr)
    flags = np.zeros(pb.n, np.uint32)
    flags[::7] = N.PKT_FLAG_SILENCE
    flags[3::11] = N.PKT_FLAG_DISCARD
    flags[5::13] = N.PKT_FLAG_SKIP
    twin.run(rcv, True, pb.seg, pb.off, pb.length, pb.cap, flags=flags)


def test_config4_srtp_srtcp_mixed_rekey(twin):
    """C4: 90% SRTP + 10% SRTCP in one bundle, _80/_32/NULL profiles, rekey
    mid-stream SDES-style (set_factory keeps contexts, Q16) and DTLS-style
    (new transformers, all state fresh)."""
    rng = np.random.default_rng(synth.SEED_BASE + 4)
    keys = synth.keys(4, 6)
    pairs = []
    for (k, s), pols in zip(keys[:3], [P80, P32, PNULL80]):
        fs = twin.factory(True, k, s, *pols)
        fr = twin.factory(False, k, s, *pols)
        pairs.append(dict(rtp_s=twin.transformer(O.KIND_RTP, fs),
                          rtcp_s=twin.transformer(O.KIND_RTCP, fs),
                          rtp_r=twin.transformer(O.KIND_RTP, fr),
                          rtcp_r=twin.transformer(O.KIND_RTCP, fr), pols=pols))

    def bundle(step):
        parts, ts_s, ts_r = [], [], []
        for j, pr in enumerate(pairs):
            rb = synth.rtp_bundle(270, 9, (60, 1200), seed=1000 * step + j,
                                  ssrcs=np.arange(9, dtype=np.uint32) + 100 * j + 1,
                                  seq0=np.full(9, (step * 30 + 65500) & 0xFFFF, np.uint32))
            cb = synth.rtcp_bundle(30, 3, seed=2000 * step + j,
                                   ssrcs=np.arange(3, dtype=np.uint32) + 100 * j + 1)
            parts += [rb, cb]
            ts_s += [pr["rtp_s"]] * rb.n + [pr["rtcp_s"]] * cb.n
            ts_r += [pr["rtp_r"]] * rb.n + [pr["rtcp_r"]] * cb.n
        b = synth.concat(parts)
        perm = rng.permutation(b.n)
        return synth.select(b, perm), [ts_s[i] for i in perm], [ts_r[i] for i in perm]

    for step in range(4):
        if step == 2:  # SDES-style rekey: new factories swapped in, contexts kept
            for j, pr in enumerate(pairs):
                k, s = keys[3 + j]
                nfs = twin.factory(True, k, s, *pr["pols"])
                nfr = twin.factory(False, k, s, *pr["pols"])
                pr["rtp_s"].set_factory(nfs, True)
                pr["rtcp_s"].set_factory(nfs, True)
                pr["rtp_r"].set_factory(nfr, False)
                pr["rtcp_r"].set_factory(nfr, False)
        if step == 3:  # DTLS-style: brand-new transformers for pair 0
            k, s = keys[5]
            pols = pairs[0]["pols"]
            fs, fr = twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols)
            pairs[0].update(rtp_s=twin.transformer(O.KIND_RTP, fs),
                            rtcp_s=twin.transformer(O.KIND_RTCP, fs),
                            rtp_r=twin.transformer(O.KIND_RTP, fr),
                            rtcp_r=twin.transformer(O.KIND_RTCP, fr))
        b, ts_s, ts_r = bundle(step)
        seg, ln, st = twin.run(ts_s, False, b.seg, b.off, b.length, b.cap)
        seg2, ln2, st2 = twin.run(ts_r, True, seg, b.off, ln, b.cap)


def test_aes_f8_srtp_srtcp(twin):
    """SDES F8_128_HMAC_SHA1_80 (SRTPCipherF8): C3 faults on F8 SRTP, DISCARD /
    SILENCE flags, F8 SRTCP with replays, and one bundle mixing F8 and AES-CM
    transformers (the CM packets take the fused kernels, the F8 ones k_f8)."""
    rng = np.random.default_rng(synth.SEED_BASE + 8)
    (k, s), (k2, s2) = synth.keys(8, 2)
    fs, fr = twin.factory(True, k, s, *PF8), twin.factory(False, k, s, *PF8)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    seq0 = np.full(40, 65500, np.uint32)
    b = synth.rtp_bundle(3000, 40, (12, 1400), seed=81, ext_frac=0.1, seq0=seq0)
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = inject_faults(pb, rng)
    flags = np.zeros(fb.n, np.uint32)
    flags[::9] = N.PKT_FLAG_SILENCE
    flags[4::13] = N.PKT_FLAG_DISCARD
    _, _, st = twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, flags=flags)
    assert (st == N.STATUS_OK).sum() > 0.9 * fb.n and (st == N.STATUS_DROP_AUTH).any()
    cs, cr = twin.transformer(O.KIND_RTCP, fs), twin.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(300, 7, (12, 200), seed=82)
    seg, ln, st = twin.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    rb = synth.select(pc, np.r_[0:300, 5:40])  # + replays
    twin.run(cr, True, rb.seg, rb.off, rb.length, rb.cap)
    # mixed F8 + AES-CM bundle
    gs = twin.factory(True, k2, s2, *P80)
    t80 = twin.transformer(O.KIND_RTP, gs)
    b1 = synth.rtp_bundle(500, 9, (60, 1400), seed=83, ssrcs=np.arange(9, dtype=np.uint32) + 7)
    b2 = synth.rtp_bundle(500, 9, (60, 1400), seed=84, ssrcs=np.arange(9, dtype=np.uint32) + 7)
    mb = synth.concat([b1, b2])
    perm = rng.permutation(mb.n)
    ts = [snd] * b1.n + [t80] * b2.n
    mb = synth.select(mb, perm)
    twin.run([ts[i] for i in perm], False, mb.seg, mb.off, mb.length, mb.cap)


def test_replay_window_quirks_q6_q7_q13(twin):
    """Hand-built sequences that exercise the Java shift-width quirks:
    delta == 64 (long >> distance & 63), 1 << -delta with distance 31 (int,
    sign-extended), SRTCP reversed delta / backwards receivedIndex."""
    (k, s), = synth.keys(99, 1)
    fs = twin.factory(True, k, s, *P80)
    fr = twin.factory(False, k, s, *P80)
    snd = twin.transformer(O.KIND_RTP, fs)
    rcv = twin.transformer(O.KIND_RTP, fr)
    seqs = [1000, 1100, 1036, 1099, 1036, 1069, 1068, 1100 - 64, 1100 - 31, 1100 - 32, 1100 - 65,
            1200, 1137, 1136, 2000, 1990, 1969, 1968, 1937, 1936]
    b = synth.rtp_bundle(len(seqs), 1, 100, seed=5)
    for i, q in enumerate(seqs):  # rewrite seq fields
        b.seg[b.off[i] + 2] = q >> 8
        b.seg[b.off[i] + 3] = q & 0xFF
    twin_check_replay_sequences(twin, snd, rcv, b)
    # the same sequence one packet per bundle (state carried between bundles)
    snd1 = twin.transformer(O.KIND_RTP, twin.factory(True, k, s, *P80))
    rcv1 = twin.transformer(O.KIND_RTP, twin.factory(False, k, s, *P80))
    for i in range(b.n):
        sub = synth.select(b, np.array([i]))
        seg, ln, st = twin.run(snd1, False, sub.seg, sub.off, sub.length, sub.cap)
        twin.run(rcv1, True, seg, sub.off, ln, sub.cap)
    # SRTCP: protect 200 packets, deliver out of order / replayed
    cs = twin.transformer(O.KIND_RTCP, fs)
    cr = twin.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(200, 1, seed=6)
    seg, ln, st = twin.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    order = [0, 1, 5, 3, 3, 40, 39, 2, 100, 36, 37, 99, 150, 149, 86, 85, 60, 150, 199, 120, 130]
    sub = synth.select(pc, np.array(order))
    twin.run(cr, True, sub.seg, sub.off, sub.length, sub.cap)


def twin_check_replay_sequences(twin, snd, rcv, b):
    # the sender drops its own duplicates / stale packets too (Q3)
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st != 0).any()
    twin.run(rcv, True, seg, b.off, ln, b.cap)


def test_roc_guess_overturned_by_walk(twin):
    """Bundles whose in-bundle updates move s_l across the 2^15 guess
    thresholds: the ROC the verify/speculative-decrypt pass guessed from the
    bundle-start state (-1 for seq 60000, 0 for seq 10) differs from the walk's
    (0, 1), forcing the midstate re-check and the fix-up re-decryption."""
    (k, s), = synth.keys(31, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    for seqs in ([100], [30000, 60000, 10, 20, 40000, 70, 33000], [65000, 1000, 34000]):
        b = synth.rtp_bundle(len(seqs), 1, 333, seed=len(seqs))
        set_seqs(b, seqs)
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
        seg2, ln2, st2 = twin.run(rcv, True, seg, b.off, ln, b.cap)
        assert (st2 == st).all()


def test_recheck_state_at_the_seq_range_edges(twin):
    """k_unprotect skips the walk's re-check state for a context whose s_l
    and in-bundle SEQs lie within 32768 of each other (no ROC change can
    happen in the bundle).  Bundles right at that edge -- spans of 32766 to
    32769 above and below s_l, and wraps through 65535 -- must still come out
    as the oracle's, tag checks under a changed ROC included."""
    (k, s), = synth.keys(33, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    for span in (32766, 32767, 32768, 32769):
        for first, seqs in ((100, lambda x: [100 + x, 150, 100 + x - 1, 101]),
                            (40000, lambda x: [40000 - x, 40100, 40000 - x + 1]),
                            (65000, lambda x: [65535, 0, 1, (65000 + x) & 0xFFFF, 65001])):
            snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
            for q in ([first], seqs(span)):
                # one SSRC over both bundles: the second continues the context
                b = synth.rtp_bundle(len(q), 1, 200, seed=span + len(q), ssrcs=[0x5EC0 + span])
                set_seqs(b, q)
                seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
                twin.run(rcv, True, seg, b.off, ln, b.cap)


def test_recheck_state_at_the_far_threshold(twin, engine):
    """k_unprotect saves the walk's re-check state (midstate, ROC block) only
    for contexts with a packet 16384 or more (linear SEQ distance) from the
    bundle-start s_l (k_parse's far stamp).  Bundles at exactly
    16383 / 16384, s_l near 0 and near 65535 (circularly close, linearly far),
    a ROC rollover inside one bundle, and a far packet whose ROC the walk
    guesses differently from the verify pass (the re-check really runs:
    srtp_stats.roc_rechecks) -- every one as the oracle's."""
    (k, s), = synth.keys(35, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    cases = [
        (100, [100 + 16383, 101, 102], False),           # within 16383: quiet, no state saved
        (100, [100 + 16384, 101], False),                 # exactly 16384: far
        (16383, [0, 16383 + 16383, 16384], False),        # 0 lies 16383 below s_l: quiet
        (65530, [65535, 0, 1, 2, 65534], False),          # rollover in the bundle (0 is 65530 away)
        (65530, [65530 - 16383, 65531], False),           # backward, within the threshold
        (2, [20000, 40000, 40001], True),                 # 40000: verify guesses ROC - 1, the walk ROC
        (65000, [65000 + 300, 200, 32500, 32501], True),  # wrap, then packets the verify pass guesses apart
    ]
    for first, seqs, recheck in cases:
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        pre = [max(first - 2, 0), first] if first > 2 else [first]
        for q in (pre, seqs):
            b = synth.rtp_bundle(len(q), 1, 300, seed=first + len(q), ssrcs=[0xFA00 + first])
            set_seqs(b, q)
            before = engine.stats()["roc_rechecks"]
            seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
            twin.run(rcv, True, seg, b.off, ln, b.cap)
            if q is seqs and recheck:
                assert engine.stats()["roc_rechecks"] > before, (first, seqs)


def set_seqs(b, seqs):
    for i, q in enumerate(seqs):
        b.seg[b.off[i] + 2] = q >> 8
        b.seg[b.off[i] + 3] = q & 0xFF


def test_check_replay_disabled(engine_factory, oracle):
    eng = engine_factory(check_replay=False, max_contexts=1024, max_factories=64,
                         max_transformers=64)
    twin = Twin(eng, check_replay=False)
    try:
        (k, s), = synth.keys(7, 1)
        f = twin.factory(True, k, s, *P80)
        t = twin.transformer(O.KIND_RTP, f)
        b = synth.rtp_bundle(50, 2, 100, seed=8)
        sub = synth.select(b, np.array(list(range(50)) + list(range(10))))
        seg, ln, st = twin.run(t, False, sub.seg, sub.off, sub.length, sub.cap)
        assert (st == 0).all()
    finally:
        O.set_check_replay(True)


def malformed_bundle():
    """Packets on which the reference drops, or throws (Q15, Q17)."""
    rng = np.random.default_rng(42)
    pk = []

    def rtp(seq, ssrc, L, b0=0x80, ext=None, cap_extra=16):
        p = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        p[0] = b0
        p[1] = 96
        p[2:4] = seq.to_bytes(2, "big")
        p[8:12] = ssrc.to_bytes(4, "big")
        if ext is not None:
            cc = b0 & 0x0F
            p[12 + 4 * cc + 2:12 + 4 * cc + 4] = ext.to_bytes(2, "big")
        pk.append((bytes(p), L + cap_extra))

    rtp(1, 7, 100)
    rtp(2, 7, 100, b0=0x40)           # version 1: dropped on unprotect
    rtp(3, 7, 10)                     # too short: invalid
    rtp(4, 7, 100, b0=0x90, ext=0xFFFF)  # negative extension length (signed high byte)
    rtp(5, 7, 60, b0=0x8F)            # CC=15: header 72 > 60 -> negative payload
    rtp(6, 8, 64, b0=0x8F)            # CC=15, payload -8: throws (arraycopy -8)
    rtp(7, 8, 100, b0=0x90, ext=0x0400)  # ext length 4096 words: header > length
    rtp(8, 9, 100)
    rtp(9, 9, 100, b0=0x90, ext=3)
    return pk


@pytest.mark.parametrize("abort", [True, False])
def test_malformed_and_abort_semantics(engine_factory, oracle, abort):
    eng = engine_factory(abort_on_error=abort, max_contexts=1024, max_factories=64,
                         max_transformers=64)
    twin = Twin(eng)
    (k, s), = synth.keys(12, 1)
    f = twin.factory(True, k, s, *P80)
    fr = twin.factory(False, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    r = twin.transformer(O.KIND_RTP, fr)
    pk = malformed_bundle()
    caps = np.array([(c + 15) // 16 * 16 for _, c in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(caps[:-1])]).astype(np.uint32)
    seg = np.zeros(int(caps.sum()), np.uint8)
    ln = np.array([len(p) for p, _ in pk], np.uint32)
    for i, (p, _) in enumerate(pk):
        seg[off[i]:off[i] + len(p)] = np.frombuffer(p, np.uint8)
    for rep in range(2):
        seg2, ln2, st = twin.run(t, False, seg, off, ln, caps, abort_on_error=abort)
        seg3, ln3, st3 = twin.run(r, True, seg2, off, ln2, caps, abort_on_error=abort)
    # SRTCP short packets: index offset negative -> throw
    tc = twin.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(6, 2, len_range=(12, 24), seed=3)
    twin.run(tc, True, cb.seg, cb.off, cb.length, cb.cap, abort_on_error=abort)


def test_capacity_and_skip(twin):
    (k, s), = synth.keys(13, 1)
    f = twin.factory(True, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    b = synth.rtp_bundle(64, 4, 200, seed=13)
    cap = b.cap.copy()
    cap[::5] = 204  # no room for the 10-byte tag
    flags = np.zeros(b.n, np.uint32)
    flags[2::9] = N.PKT_FLAG_SKIP
    twin.run(t, False, b.seg, b.off, b.length, cap, flags=flags)


def test_factory_close_no_new_contexts(twin):
    (k, s), = synth.keys(14, 1)
    f = twin.factory(True, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f)
    b = synth.rtp_bundle(40, 4, 100, seed=14)
    twin.run(t, False, b.seg, b.off, b.length, b.cap)
    f.close()
    b2 = synth.rtp_bundle(40, 8, 100, seed=15, ssrcs=np.concatenate(
        [b.meta["ssrcs"], np.arange(4, dtype=np.uint32) + 77]))
    twin.run(t, False, b2.seg, b2.off, b2.length, b2.cap)
    t.close()
    twin.run(t, False, b2.seg, b2.off, b2.length, b2.cap)


def test_many_transformers_one_bundle(twin):
    """A bundle spanning 50 transformers (the aggregator case)."""
    rng = np.random.default_rng(21)
    ts, parts = [], []
    for j in range(50):
        (k, s), = synth.keys(100 + j, 1)
        f = twin.factory(True, k, s, *(P80 if j % 3 else P32))
        t = twin.transformer(O.KIND_RTP, f)
        bj = synth.rtp_bundle(int(rng.integers(1, 40)), int(rng.integers(1, 4)), (60, 1400),
                              seed=300 + j)
        parts.append(bj)
        ts += [t] * bj.n
    b = synth.concat(parts)
    perm = rng.permutation(b.n)
    sb = synth.select(b, perm)
    twin.run([ts[i] for i in perm], False, sb.seg, sb.off, sb.length, sb.cap)


def reseq(b, step):
    o = b.off.astype(np.int64)
    q = ((b.seg[o + 2].astype(np.int64) << 8) | b.seg[o + 3]) + step
    b.seg[o + 2] = ((q >> 8) & 0xFF).astype(np.uint8)
    b.seg[o + 3] = (q & 0xFF).astype(np.uint8)


def test_bench_loop_multi_step(twin):
    """bench.py's step at reduced size: protect -> unprotect -> advance every
    packet's seq by the packets per SSRC, repeated; includes SSRCs that wrap."""
    n, nssrc = 6000, 700
    rng = np.random.default_rng(77)
    seq0 = rng.integers(0, 65536, nssrc).astype(np.uint32)
    seq0[:20] = 65536 - rng.integers(1, 60, 20)
    b = synth.rtp_bundle(n, nssrc, 1200, seed=synth.SEED_BASE + 2, seq0=seq0)
    (k, s), = synth.keys(2, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    step = -(-n // nssrc)
    cur = b.copy()
    for it in range(6):
        seg, ln, st = twin.run(snd, False, cur.seg, cur.off, cur.length, cur.cap,
                               check_state=(it % 2 == 0))
        assert (st == 0).all(), np.bincount(st)
        seg2, ln2, st2 = twin.run(rcv, True, seg, cur.off, ln, cur.cap, check_state=(it % 2 == 0))
        assert (st2 == 0).all(), np.bincount(st2)
        cur.seg, cur.length = seg2, ln2
        reseq(cur, step)


def test_config5_125k_streams_with_faults(engine_factory, oracle):
    """C5 at one GPU's share of 10^6 streams (125k SSRCs): three protect
    bundles spanning all streams (5% starting near the seq wrap), then
    unprotect of the faulted stream (C3 mix) in two bundles -- bit-exact
    against the oracle at the table occupancy and sort width of that scale;
    the context state of 2000 sampled streams is compared at the end."""
    eng = engine_factory(max_contexts=1 << 18, max_factories=8, max_transformers=8,
                         max_batch=1 << 17)
    twin = Twin(eng)
    rng = np.random.default_rng(synth.SEED_BASE + 5)
    n_ssrc = 125000
    seq0 = rng.integers(0, 65536, n_ssrc).astype(np.uint32)
    seq0[rng.random(n_ssrc) < 0.05] = 65535
    b = synth.rtp_bundle(3 << 16, n_ssrc, 1200, seed=synth.SEED_BASE + 5, seq0=seq0)
    (k, s), = synth.keys(5, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    parts = []
    for j in range(3):
        sub = synth.select(b, np.arange(j << 16, (j + 1) << 16))
        seg, ln, st = twin.run(snd, False, sub.seg, sub.off, sub.length, sub.cap, check_state=False)
        assert (st == 0).all()
        sub.seg, sub.length = seg, ln
        parts.append(sub)
    fb = inject_faults(synth.concat(parts), rng)
    half = fb.n // 2
    for idx in (np.arange(0, half), np.arange(half, fb.n)):
        sub = synth.select(fb, idx)
        twin.run(rcv, True, sub.seg, sub.off, sub.length, sub.cap, check_state=False)
    ssrcs = b.meta["ssrcs"]
    for ssrc in rng.choice(ssrcs, 2000, replace=False):
        for t in (snd, rcv):
            so, se = t.o.state(int(ssrc)), eng.context_state(t.e, int(ssrc))
            assert (so is None) == (se is None)
            if so is not None:
                for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
                    assert int(so[key]) == int(se[key]), (ssrc, key)


def test_full_size_round_trip_properties(engine_factory):
    """BASELINE config 2 at full bundle size (2^18 x 1200 B, 10k SSRCs) on the
    device path: protect then unprotect restores every byte, all tags verify,
    lengths cycle 1200 -> 1210 -> 1200, and a second protect of the same
    bundle is rejected as replays (sender consistency check, Q3)."""
    import torch
    from libjitsi_amd import SRTPContextFactory, SRTPTransformer
    eng = engine_factory(max_contexts=1 << 16, max_factories=64, max_transformers=64)
    b = synth.rtp_bundle(1 << 18, 10000, 1200, seed=synth.SEED_BASE + 2)
    (k, s), = synth.keys(2, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *P80, engine=eng))
    dev = torch.device("cuda")
    seg = torch.from_numpy(b.seg).to(dev)
    off = torch.from_numpy(b.off.view(np.int32)).to(dev)
    ln = torch.from_numpy(b.length.view(np.int32)).to(dev)
    cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
    st = torch.empty(b.n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    eng.transform_device(False, snd.tid, seg, off, ln, cap, st, stream=stream)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert int((ln != 1210).sum()) == 0
    enc = seg.cpu().numpy()
    o = b.off.astype(np.int64)
    assert not np.array_equal(enc[o[0] + 12:o[0] + 1200], b.seg[o[0] + 12:o[0] + 1200])
    # the whole protected segment and every length against the oracle (fresh
    # oracle sender, same keys, the same 2^18-packet bundle)
    from harness import opol
    of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
    ot = O.Transformer(O.KIND_RTP, of, of)
    seg_o, len_o = b.seg.copy(), b.length.copy()
    st_o = O.process(ot, False, seg_o, b.off, len_o, b.cap)
    assert (st_o == 0).all() and np.array_equal(len_o, ln.cpu().numpy().view(np.uint32))
    if not np.array_equal(enc, seg_o):
        diff = np.nonzero(enc != seg_o)[0]
        raise AssertionError(f"{len(diff)} segment bytes differ from the oracle, first at {diff[:5]}")
    eng.transform_device(True, rcv.tid, seg, off, ln, cap, st, stream=stream)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert int((ln != 1200).sum()) == 0
    dec = seg.cpu().numpy()
    keep = np.ones(len(b.seg), bool)  # bytes past the shrunk length keep the old tag
    for j in range(10):
        keep[o + 1200 + j] = False
    assert np.array_equal(dec[keep], b.seg[keep])
    seg2 = torch.from_numpy(b.seg).to(dev)
    ln2 = torch.from_numpy(b.length.view(np.int32)).to(dev)
    eng.transform_device(False, snd.tid, seg2, off, ln2, cap, st, stream=stream)
    torch.cuda.synchronize()
    assert int((st == N.STATUS_DROP_REPLAY).sum()) == b.n
