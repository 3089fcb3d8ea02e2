"""CPU: the C oracle against the independent pure-Python restatement
(oracle/pyref.py: own FIPS-197 AES, hashlib HMAC) on small bundles that hit the
state machine's edge cases -- replays, reordering, ROC wraps, tampering,
malformed headers, abort-on-throw, SRTCP quirks, rekeys."""
import numpy as np
import pytest

from libjitsi_amd import synth
from oracle import pyref as R


def pols(tag_rtp=10, tag_rtcp=10, enc=1):
    return (enc, 16 if enc else 0, 1, 20, tag_rtp, 14 if enc else 0), \
           (enc, 16 if enc else 0, 1, 20, tag_rtcp, 14 if enc else 0)


class Pair:
    """Same factories/transformers in both restatements."""

    def __init__(self, oracle):
        self.O = oracle

    def factory(self, sender, k, s, p_rtp, p_rtcp):
        return (self.O.Factory(sender, k, s, self.O.Policy(*p_rtp), self.O.Policy(*p_rtcp)),
                R.Factory(sender, k, s, p_rtp, p_rtcp))

    def transformer(self, kind, f, r=None):
        r = r or f
        return self.O.Transformer(kind, f[0], r[0]), R.Transformer(kind, f[1], r[1])

    def run(self, ts, reverse, b, flags=None, abort=True):
        seg_o, len_o = b.seg.copy(), b.length.copy()
        seg_p, len_p = b.seg.copy(), b.length.copy()
        if isinstance(ts, tuple):
            st_o = self.O.process(ts[0], reverse, seg_o, b.off, len_o, b.cap, flags, abort)
            st_p = R.process(ts[1], reverse, seg_p, b.off, len_p, b.cap, flags, abort)
        else:
            st_o = self.O.process([t[0] for t in ts], reverse, seg_o, b.off, len_o, b.cap, flags,
                                  abort)
            st_p = R.process([t[1] for t in ts], reverse, seg_p, b.off, len_p, b.cap, flags, abort)
        assert list(st_o) == list(st_p)
        assert np.array_equal(len_o, len_p)
        assert np.array_equal(seg_o, seg_p)
        out = b.copy()
        out.seg, out.length = seg_o, len_o
        return out, np.asarray(st_o)


def set_seq(b, seqs):
    for i, q in enumerate(seqs):
        b.seg[b.off[i] + 2] = (q >> 8) & 0xFF
        b.seg[b.off[i] + 3] = q & 0xFF


@pytest.mark.parametrize("check", [True, False])
def test_replay_reorder_wrap(oracle, check):
    oracle.set_check_replay(check)
    R.CHECK_REPLAY[0] = check
    try:
        P = Pair(oracle)
        rng = np.random.default_rng(1)
        (k, s), = synth.keys(1, 1)
        fs, fr = P.factory(True, k, s, *pols()), P.factory(False, k, s, *pols())
        snd, rcv = P.transformer(0, fs), P.transformer(0, fr)
        base = 65536 - 40
        seqs = [(base + i) & 0xFFFF for i in range(120)]
        for _ in range(30):  # reorder / duplicate / stale / far jumps
            i = int(rng.integers(0, len(seqs)))
            seqs.insert(i, int(rng.choice([seqs[max(0, i - 3)], seqs[max(0, i - 70)],
                                            (seqs[i] + 40000) & 0xFFFF, seqs[i]])))
        b = synth.rtp_bundle(len(seqs), 1, 80, seed=2)
        set_seq(b, seqs)
        pb, st = P.run(snd, False, b)
        # receiver sees the sender's output, with some tags flipped
        for i in range(0, pb.n, 9):
            pb.seg[pb.off[i] + 20] ^= 1
        P.run(rcv, True, pb)
    finally:
        oracle.set_check_replay(True)
        R.CHECK_REPLAY[0] = True


def test_profiles_and_rekey(oracle):
    P = Pair(oracle)
    rng = np.random.default_rng(3)
    keys = synth.keys(3, 4)
    prof = [pols(), pols(4, 10), pols(10, 10, enc=0), pols(0, 0)]
    fs = [P.factory(True, k, s, *p) for (k, s), p in zip(keys, prof)]
    fr = [P.factory(False, k, s, *p) for (k, s), p in zip(keys, prof)]
    ts = [P.transformer(j % 2, fs[j]) for j in range(4)]
    tr = [P.transformer(j % 2, fr[j]) for j in range(4)]
    for step in range(3):
        parts, who = [], []
        for j in range(4):
            if j % 2 == 0:
                bj = synth.rtp_bundle(30, 3, (12, 300), seed=10 * step + j, ext_frac=0.3,
                                      ssrcs=np.arange(3, dtype=np.uint32) + 1,
                                      seq0=np.full(3, (65520 + 30 * step) & 0xFFFF, np.uint32))
            else:
                bj = synth.rtcp_bundle(30, 3, (12, 120), seed=10 * step + j,
                                       ssrcs=np.arange(3, dtype=np.uint32) + 1)
            parts.append(bj)
            who += [j] * bj.n
        b = synth.concat(parts)
        perm = rng.permutation(b.n)
        b = synth.select(b, perm)
        who = [who[i] for i in perm]
        pb, _ = P.run([ts[j] for j in who], False, b)
        P.run([tr[j] for j in who], True, pb)
        if step == 1:  # SDES-style rekey of transformer 0 / DTLS-style for 2
            (k, s), = synth.keys(50, 1)
            nf = P.factory(True, k, s, *prof[0])
            ts[0][0].set_factory(nf[0], True)
            ts[0][1].set_factory(nf[1], True)
            ts[2] = P.transformer(0, P.factory(True, *synth.keys(51, 1)[0], *prof[2]))


@pytest.mark.parametrize("abort", [True, False])
def test_malformed(oracle, abort):
    P = Pair(oracle)
    rng = np.random.default_rng(4)
    (k, s), = synth.keys(4, 1)
    f, fr = P.factory(True, k, s, *pols()), P.factory(False, k, s, *pols())
    t, r = P.transformer(0, f), P.transformer(0, fr)
    tc = P.transformer(1, fr)
    for rep in range(4):
        b = synth.rtp_bundle(60, 5, (8, 120), seed=40 + rep)
        for i in range(b.n):  # random first bytes: CC, X, version
            b.seg[b.off[i]] = int(rng.integers(0, 256))
            if rng.random() < 0.3:
                b.seg[b.off[i] + 14] = int(rng.integers(0, 256))
        b.cap[::7] = np.minimum(b.cap[::7], b.length[::7] + 4)
        pb, _ = P.run(t, False, b, abort=abort)
        P.run(r, True, pb, abort=abort)
        cb = synth.rtcp_bundle(20, 3, (12, 40), seed=60 + rep)
        P.run(tc, True, cb, abort=abort)


def test_aes_f8_profiles(oracle):
    """AES-F8 (SDES F8_128_HMAC_SHA1_80, SRTPCipherF8) for SRTP and SRTCP:
    protect, tampering, replays, a ROC wrap, extension headers, and the SRTCP
    quirk of ciphering only [8, 8 + length - 4 - tag)."""
    P = Pair(oracle)
    (k, s), = synth.keys(7, 1)
    for tags in ((10, 10), (4, 4), (4, 10)):
        f, fr = P.factory(True, k, s, *pols(*tags, enc=2)), P.factory(False, k, s, *pols(*tags, enc=2))
        t, r = P.transformer(0, f), P.transformer(0, fr)
        tc, rc = P.transformer(1, f), P.transformer(1, fr)
        for rep in range(3):
            b = synth.rtp_bundle(40, 3, (12, 300), seed=70 + rep, ext_frac=0.3,
                                 ssrcs=np.arange(3, dtype=np.uint32) + 9,
                                 seq0=np.full(3, (65525 + 40 * rep) & 0xFFFF, np.uint32))
            pb, st = P.run(t, False, b)
            assert (st == 0).all()
            pb.seg[pb.off[5] + 13] ^= 4  # tamper
            ub, st = P.run(r, True, synth.concat([pb, synth.select(pb, np.arange(3))]))  # + replays
            assert st[5] == 2 and (st[40:] == 1).all()
            for i in range(40):  # accepted packets come back as the original RTP
                if i != 5:
                    o = b.off[i]
                    assert st[i] == 0 and ub.length[i] == b.length[i]
                    assert np.array_equal(ub.seg[o:o + b.length[i]], b.seg[o:o + b.length[i]])
            cb = synth.rtcp_bundle(20, 3, (12, 120), seed=80 + rep,
                                   ssrcs=np.arange(3, dtype=np.uint32) + 9)
            pcb, st = P.run(tc, False, cb)
            assert (st == 0).all()
            ucb, st = P.run(rc, True, pcb)
            assert (st == 0).all()
            for i in range(cb.n):
                o = cb.off[i]
                assert np.array_equal(ucb.seg[o:o + cb.length[i]], cb.seg[o:o + cb.length[i]])


def test_f8_policy_bounds(oracle):
    """SRTCP F8 ciphers [8, 8 + length - 4 - tag): outside the packet without an
    HMAC trailer of >= 4 tag bytes, so such SRTCP policies are refused (the
    SRTP side of the same factory may use any tag length)."""
    (k, s), = synth.keys(9, 1)
    with pytest.raises(ValueError):
        oracle.Factory(True, k, s, oracle.Policy(2, 16, 1, 20, 10, 14), oracle.Policy(2, 16, 0, 0, 0, 14))
    with pytest.raises(ValueError):
        oracle.Factory(True, k, s, oracle.Policy(2, 16, 1, 20, 10, 14), oracle.Policy(2, 16, 1, 20, 2, 14))
    oracle.Factory(True, k, s, oracle.Policy(2, 16, 0, 0, 0, 14), oracle.Policy(2, 16, 1, 20, 4, 14))
