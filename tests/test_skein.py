"""Skein-MAC policies (ZRTP "SK32" / "SK64"): SRTPPolicy.SKEIN_AUTHENTICATION,
BaseSRTPCryptoContext.java:244-248, keyed in SRTPCryptoContext.java:421-428 and
SRTCPCryptoContext.java:185-192 with ParametersForSkein(authKey, Skein512,
tagLength * 8); ZRTPTransformEngine.java:867-909 builds the policies (32-byte
auth key, one policy for SRTP and SRTCP).

In the reference the MAC is bccontrib's SkeinMac. That jar is absent here, so
Skein-512 is restated three times -- the oracle's (oracle/skein.c), an
independent one in oracle/pyref.py, and the engine's host code
(host_crypto.cpp, srtp_skein512_mac, which also keys the GPU path) -- and
pinned by the published known answers of "The Skein Hash Function Family"
version 1.3: Skein-512-512 of the messages FF, FF FE .. C0 (64 bytes) and
FF FE .. 80 (128 bytes).  The keyed form (key UBI, then config, message,
output) is the same UBI with other type codes; the three restatements agree on
it for every key, message and output length tried.  The GPU path (k_skein, the
walk's re-check) is checked against the oracle on whole bundles.
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from libjitsi_amd.srtp import SRTPPolicy, derive_session_keys_auth, skein512_mac
from oracle import oracle as O
from oracle import pyref as R

from harness import Twin
from test_gpu_parity import inject_faults

SKEIN_512_512_KAT = {
    1: "71B7BCE6FE6452227B9CED6014249E5BF9A9754C3AD618CCC4E0AAE16B316CC8"
       "CA698D864307ED3E80B6EF1570812AC5272DC409B5A012DF2A579102F340617A",
    64: "45863BA3BE0C4DFC27E75D358496F4AC9A736A505D9313B42B2F5EADA79FC17F"
        "63861E947AFB1D056AA199575AD3F8C9A3CC1780B5E5FA4CAE050E989876625B",
    128: "91CCA510C263C4DDD010530A33073309628631F308747E1BCBAA90E451CAB92E"
         "5188087AF4188773A332303E6667A7A210856F742139000071F48E8BA2A5ADB7",
}

# the paper's precomputed IVs (the chaining value after the config UBI)
SKEIN_512_IV = {
    512: [0x4903ADFF749C51CE, 0x0D95DE399746DF03, 0x8FD1934127C79BCE, 0x9A255629FF352CB1,
          0x5DB62599DF6CA7B0, 0xEABE394CA9D5C3F4, 0x991112C71A75B523, 0xAE18A40B660FCC33],
    256: [0xCCD044A12FDB3E13, 0xE83590301A79A9EB, 0x55AEA0614F816E6F, 0x2A2767A4AE9B94DB,
          0xEC06025E74DD7683, 0xE7A436CDC4746251, 0xC36FBAF9393AD185, 0x3EEDBA1833EDFC13],
}

SKEIN_PROFILES = ["AES_CM_128_SKEIN_32", "AES_CM_128_SKEIN_64", "AES_256_CM_SKEIN_64",
                  "TWOFISH_CM_128_SKEIN_32", "TWOFISH_CM_256_SKEIN_64"]


@pytest.mark.parametrize("n", sorted(SKEIN_512_512_KAT))
def test_skein512_kat(n, oracle):
    msg = bytes(0xFF - i for i in range(n))
    want = SKEIN_512_512_KAT[n]
    assert O.skein512(msg).hex().upper() == want
    assert R.skein512_mac(b"", msg, 512).hex().upper() == want
    assert skein512_mac(b"", msg).hex().upper() == want


@pytest.mark.parametrize("bits", sorted(SKEIN_512_IV))
def test_skein512_iv(bits, oracle):
    assert O.skein512_iv(bits) == SKEIN_512_IV[bits]


def test_skein_mac_restatements_agree(oracle):
    rng = np.random.default_rng(11)
    for key_len, msg_len, bits in [(32, 0, 32), (32, 1, 32), (32, 63, 64), (32, 64, 32), (32, 65, 64),
                                   (32, 1214, 32), (17, 200, 64), (64, 130, 512), (1, 5, 8),
                                   (32, 4, 96)]:
        key, msg = rng.bytes(key_len), rng.bytes(msg_len)
        c = O.skein512(msg, bits, key)
        assert R.skein512_mac(key, msg, bits) == c
        assert skein512_mac(key, msg, bits) == c


def test_skein_kdf_auth_key_32(oracle):
    rng = np.random.default_rng(12)
    for klen, twofish in ((16, False), (32, False), (16, True)):
        mk, ms = rng.bytes(klen), rng.bytes(14)
        enc_type = N.TWOFISH_ENCRYPTION if twofish else N.AESCM_ENCRYPTION
        for rtcp in (False, True):
            got = derive_session_keys_auth(enc_type, mk, ms, rtcp, 32)
            assert got == O.derive_keys_auth(mk, ms, rtcp, 32, twofish)
            assert len(got[1]) == 32
            # the first 20 bytes are the HMAC policies' auth key (same PRF stream)
            assert got[1][:20] == (O.derive_keys_twofish(mk, ms, rtcp) if twofish
                                   else O.derive_keys(mk, ms, rtcp))[1]


def test_skein_policies_shape():
    for name in SKEIN_PROFILES:
        rtp, rtcp = profile_policies(name)
        for p in (rtp, rtcp):
            assert p.authType == SRTPPolicy.SKEIN_AUTHENTICATION and p.authKeyLength == 32
            assert p.authTagLength in (4, 8)


def test_skein_state_machine_crosscheck(oracle):
    """C oracle against the pure-Python restatement on AES-128-CM + Skein
    bundles: replays, a sequence wrap, tampered tags, SRTCP."""
    rng = np.random.default_rng(13)
    for name in ("AES_CM_128_SKEIN_32", "AES_CM_128_SKEIN_64"):
        rtp, rtcp = profile_policies(name)
        tp = (rtp.encType, rtp.encKeyLength, rtp.authType, rtp.authKeyLength, rtp.authTagLength,
              rtp.saltKeyLength)
        k, s = rng.bytes(16), rng.bytes(14)
        ofs = O.Factory(True, k, s, O.Policy(*tp), O.Policy(*tp))
        ofr = O.Factory(False, k, s, O.Policy(*tp), O.Policy(*tp))
        pfs, pfr = R.Factory(True, k, s, tp, tp), R.Factory(False, k, s, tp, tp)
        for kind in (O.KIND_RTP, O.KIND_RTCP):
            osn, orc = O.Transformer(kind, ofs, ofs), O.Transformer(kind, ofr, ofr)
            psn, prc = R.Transformer(kind, pfs, pfs), R.Transformer(kind, pfr, pfr)
            if kind == O.KIND_RTP:
                b = synth.rtp_bundle(120, 2, (12, 300), seed=14, seq0=np.full(2, 65500, np.uint32))
            else:
                b = synth.rtcp_bundle(60, 2, (12, 200), seed=15)
            sa, la = b.seg.copy(), b.length.copy()
            sb, lb = b.seg.copy(), b.length.copy()
            st_o = O.process(osn, False, sa, b.off, la, b.cap)
            st_p = R.process(psn, False, sb, b.off, lb, b.cap)
            assert list(st_o) == list(st_p) and np.array_equal(la, lb) and np.array_equal(sa, sb)
            assert (np.asarray(st_o) == 0).all()
            pb = b.copy()
            pb.seg, pb.length = sa, la
            rb = synth.select(pb, np.r_[0:pb.n, 0:10])  # + replays
            for i in range(0, rb.n, 7):  # tamper with some tags
                rb.seg[rb.off[i] + rb.length[i] - 1] ^= 0x40
            sa, la = rb.seg.copy(), rb.length.copy()
            sb, lb = rb.seg.copy(), rb.length.copy()
            st_o = O.process(orc, True, sa, rb.off, la, rb.cap)
            st_p = R.process(prc, True, sb, rb.off, lb, rb.cap)
            assert list(st_o) == list(st_p) and np.array_equal(la, lb) and np.array_equal(sa, sb)
            st_o = np.asarray(st_o)
            assert (st_o == O.DROP_AUTH).sum() > 0 and (st_o == 0).sum() > 0.7 * rb.n


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 14, max_factories=128, max_transformers=256)


def _flags(n):
    flags = np.zeros(n, np.uint32)
    flags[::9] = N.PKT_FLAG_SILENCE
    flags[4::13] = N.PKT_FLAG_DISCARD
    return flags


@pytest.mark.gpu
@pytest.mark.parametrize("name", SKEIN_PROFILES)
def test_skein_srtp_srtcp(engine, name):
    """Protect and unprotect through k_ext + k_skein (and the walk's Skein
    re-check for the ROCs the wrap overturns), bit-exact against the oracle:
    statuses, lengths, the whole segment and the context states."""
    pols = profile_policies(name)
    tag = pols[0].authTagLength
    klen = pols[0].encKeyLength
    tw = Twin(engine)
    rng = np.random.default_rng(len(name) + klen)
    k, s = rng.bytes(klen), rng.bytes(14)
    fs, fr = tw.factory(True, k, s, *pols), tw.factory(False, k, s, *pols)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(1500, 20, (12, 1400), seed=400 + klen, ext_frac=0.1,
                         seq0=np.full(20, 65500, np.uint32))
    seg, ln, st = tw.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).sum() > 0.99 * b.n
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = inject_faults(pb, rng, tag_len=tag)
    _, _, st = tw.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, flags=_flags(fb.n))
    assert (st == N.STATUS_OK).sum() > 0.9 * fb.n
    assert (st == N.STATUS_DROP_AUTH).sum() > 0
    cs, cr = tw.transformer(O.KIND_RTCP, fs), tw.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(200, 5, (12, 200), seed=401 + klen)
    seg, ln, st = tw.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    rb = synth.select(pc, np.r_[0:200, 3:20])  # + replays
    for i in range(1, 200, 11):
        rb.seg[rb.off[i] + rb.length[i] - 2] ^= 0x01
    _, _, st = tw.run(cr, True, rb.seg, rb.off, rb.length, rb.cap)
    assert (st[200:] == N.STATUS_DROP_REPLAY).all()
    assert (st[:200] == N.STATUS_DROP_AUTH).sum() == len(range(1, 200, 11))


@pytest.mark.gpu
def test_skein_null_cipher_and_roc_overturn(engine):
    """NULL cipher + Skein (the MAC only), and receiver bundles whose sequence
    numbers straddle the 2^15 guess thresholds so that the walk's ROC differs
    from k_unprotect's guess and the Skein tag is re-checked in the walk."""
    tw = Twin(engine)
    rng = np.random.default_rng(410)
    pol = SRTPPolicy(SRTPPolicy.NULL_ENCRYPTION, 0, SRTPPolicy.SKEIN_AUTHENTICATION, 32, 8, 0)
    k, s = rng.bytes(16), rng.bytes(14)
    fs, fr = tw.factory(True, k, s, pol, pol), tw.factory(False, k, s, pol, pol)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    cs, cr = tw.transformer(O.KIND_RTCP, fs), tw.transformer(O.KIND_RTCP, fr)
    b = synth.rtp_bundle(300, 3, (12, 700), seed=411)
    seg, ln, st = tw.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    _, _, st = tw.run(rcv, True, pb.seg, pb.off, pb.length, pb.cap)
    assert (st == 0).all()
    cb = synth.rtcp_bundle(50, 2, (12, 200), seed=412)
    seg, ln, st = tw.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    _, _, st = tw.run(cr, True, pc.seg, pc.off, pc.length, pc.cap)
    # the NULL cipher's SRTCP trailer carries index 0 (transformPacket :391-427,
    # SURVEY Q12): after each SSRC's first packet the receiver sees replays
    assert (st[:2] == 0).all() and (st[2:] == N.STATUS_DROP_REPLAY).all()
    # ROC overturned in-bundle (AES-CM + Skein-32)
    pols = profile_policies("AES_CM_128_SKEIN_32")
    fs, fr = tw.factory(True, k, s, *pols), tw.factory(False, k, s, *pols)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    for seqs in ([100], [30000, 60000, 10, 20, 40000, 70, 33000], [65000, 1000, 34000]):
        b = synth.rtp_bundle(len(seqs), 1, 333, seed=len(seqs))
        for i, q in enumerate(seqs):
            b.seg[b.off[i] + 2] = q >> 8
            b.seg[b.off[i] + 3] = q & 0xFF
        seg, ln, st = tw.run(snd, False, b.seg, b.off, b.length, b.cap)
        _, _, st2 = tw.run(rcv, True, seg, b.off, ln, b.cap)
        assert (st2 == st).all()


@pytest.mark.gpu
def test_skein_mixed_with_hmac_bundle(engine):
    """Skein and HMAC-SHA1 transformers interleaved in one bundle."""
    tw = Twin(engine)
    rng = np.random.default_rng(420)
    specs = [("AES_CM_128_SKEIN_32", 16), ("AES_CM_128_HMAC_SHA1_80", 16),
             ("AES_256_CM_SKEIN_64", 32), ("F8_128_HMAC_SHA1_80", 16), ("TWOFISH_CM_128_SKEIN_32", 16)]
    snds, rcvs, bundles = [], [], []
    for i, (name, klen) in enumerate(specs):
        pols = profile_policies(name)
        k, s = rng.bytes(klen), rng.bytes(14)
        snds.append(tw.transformer(O.KIND_RTP, tw.factory(True, k, s, *pols)))
        rcvs.append(tw.transformer(O.KIND_RTP, tw.factory(False, k, s, *pols)))
        bundles.append(synth.rtp_bundle(300, 4, (60, 1200), seed=421 + i))
    mb = synth.concat(bundles)
    owner = np.concatenate([np.full(b.n, i) for i, b in enumerate(bundles)])
    which = rng.permutation(owner)
    perm = np.empty(mb.n, int)
    base = np.cumsum([0] + [b.n for b in bundles])
    for i in range(len(bundles)):
        perm[which == i] = base[i] + np.arange(bundles[i].n)
    mb = synth.select(mb, perm)
    ow = owner[perm]
    seg, ln, st = tw.run([snds[i] for i in ow], False, mb.seg, mb.off, mb.length, mb.cap)
    assert (st == 0).all()
    pm = mb.copy()
    pm.seg, pm.length = seg, ln
    _, ln2, st2 = tw.run([rcvs[i] for i in ow], True, pm.seg, pm.off, pm.length, pm.cap)
    assert (st2 == 0).all() and np.array_equal(ln2, mb.length)
