"""AES-256-CM (RFC 6188): SRTPCryptoContext with encKeyLength 32.

The reference reaches it through ZRTP's AES3 cipher (ZRTPTransformEngine.java
:873-900) and lists the AES_256_CM_HMAC_SHA1_80/_32 SDES suites
(SDesControlImpl.java:71-72). BaseSRTPCryptoContext (:187-215) keys
BouncyCastle's AES engine with the 32-byte master key, so deriveSrtpKeys
(:393-447) runs the AES-256 PRF and produces a 32-byte session key.
SRTPCipherCTR (:68-121) then runs 14-round AES over the same counter blocks.

* CPU: the RFC 6188 7.2 AES_256_CM_PRF known-answer vectors, checked against
  the engine's host KDF and against the oracle (OpenSSL AES-256).
* GPU (k_ext): SRTP and SRTCP protect/unprotect with the C3 fault mix, DISCARD /
  SILENCE flags, the _32 suite, and a bundle mixing AES-256 and AES-128
  transformers. Every bundle is bit-exact against the oracle.
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from libjitsi_amd.srtp import derive_session_keys
from oracle import oracle as O

from harness import Twin
from test_gpu_parity import inject_faults

P256_80 = profile_policies("AES_256_CM_HMAC_SHA1_80")
P256_32 = profile_policies("AES_256_CM_HMAC_SHA1_32")
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")

# RFC 6188 7.2 (AES_256_CM_PRF test vectors), index 0
RFC6188_MK = bytes.fromhex("f0f04914b513f2763a1b1fa130f10e2998f6f6e43e4309d1e622a0e332b9f1b6")
RFC6188_MS = bytes.fromhex("3b04803de51ee7c96423ab5b78d2")
RFC6188_ENC = bytes.fromhex("5ba1064e30ec51613cad926c5a28ef731ec7fb397f70a960653caf06554cd8c4")
RFC6188_AUTH = bytes.fromhex("fd9c32d39ed5fbb5a9dc96b30818454d1313dc05")
RFC6188_SALT = bytes.fromhex("fa31791685ca444a9e07c6c64e93")


def keys256(seed, n=1):
    rng = np.random.default_rng(seed ^ 0x256)
    return [(rng.bytes(32), rng.bytes(14)) for _ in range(n)]


def test_rfc6188_prf_vectors(oracle):
    for kdf in (derive_session_keys, O.derive_keys):
        enc, auth, salt = kdf(RFC6188_MK, RFC6188_MS)
        assert enc == RFC6188_ENC and auth == RFC6188_AUTH and salt == RFC6188_SALT
    # SRTCP labels 3..5 agree between the engine and the oracle
    assert derive_session_keys(RFC6188_MK, RFC6188_MS, True) == O.derive_keys(RFC6188_MK, RFC6188_MS, True)


def test_policy_table():
    p, q = P256_80
    assert (p.encKeyLength, p.saltKeyLength, p.authTagLength, q.authTagLength) == (32, 14, 10, 10)
    assert P256_32[0].authTagLength == 4 and P256_32[1].authTagLength == 10


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 15, max_factories=256, max_transformers=512)


@pytest.mark.gpu
@pytest.mark.parametrize("pols,tag", [(P256_80, 10), (P256_32, 4)])
def test_aes256_srtp_srtcp(engine, pols, tag):
    tw = Twin(engine)
    rng = np.random.default_rng(256 + tag)
    (k, s), = keys256(11 + tag)
    fs, fr = tw.factory(True, k, s, *pols), tw.factory(False, k, s, *pols)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(3000, 40, (12, 1400), seed=257 + tag, ext_frac=0.1,
                         seq0=np.full(40, 65500, np.uint32))
    seg, ln, st = tw.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).sum() > 0.99 * b.n
    pb = b.copy()
    pb.seg, pb.length = seg, ln
    fb = inject_faults(pb, rng, tag_len=tag)
    flags = np.zeros(fb.n, np.uint32)
    flags[::9] = N.PKT_FLAG_SILENCE
    flags[4::13] = N.PKT_FLAG_DISCARD
    _, _, st = tw.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, flags=flags)
    assert (st == N.STATUS_OK).sum() > 0.9 * fb.n and (st == N.STATUS_DROP_AUTH).any()
    cs, cr = tw.transformer(O.KIND_RTCP, fs), tw.transformer(O.KIND_RTCP, fr)
    cb = synth.rtcp_bundle(300, 7, (12, 200), seed=258 + tag)
    seg, ln, st = tw.run(cs, False, cb.seg, cb.off, cb.length, cb.cap)
    pc = cb.copy()
    pc.seg, pc.length = seg, ln
    rb = synth.select(pc, np.r_[0:300, 5:40])  # + replays
    _, _, st = tw.run(cr, True, rb.seg, rb.off, rb.length, rb.cap)
    assert (st[:300] == 0).sum() > 0.95 * 300 and (st[300:] == N.STATUS_DROP_REPLAY).all()


@pytest.mark.gpu
def test_mixed_aes256_aes128_bundle(engine):
    """One bundle, both key lengths: the AES-128 packets take the fused
    kernels (and speculative decryption), the AES-256 ones k_ext."""
    tw = Twin(engine)
    rng = np.random.default_rng(259)
    (k, s), = keys256(12)
    (k2, s2), = synth.keys(13, 1)
    a_s, a_r = tw.factory(True, k, s, *P256_80), tw.factory(False, k, s, *P256_80)
    b_s, b_r = tw.factory(True, k2, s2, *P80), tw.factory(False, k2, s2, *P80)
    ta, ra = tw.transformer(O.KIND_RTP, a_s), tw.transformer(O.KIND_RTP, a_r)
    tb, rb_ = tw.transformer(O.KIND_RTP, b_s), tw.transformer(O.KIND_RTP, b_r)
    b1 = synth.rtp_bundle(600, 9, (60, 1400), seed=260)
    b2 = synth.rtp_bundle(600, 9, (60, 1400), seed=261)
    mb = synth.concat([b1, b2])
    # interleave the two bundles, each stream keeping its order
    which = rng.permutation(np.r_[np.zeros(b1.n, int), np.ones(b2.n, int)])
    perm = np.empty(mb.n, int)
    perm[which == 0] = np.arange(b1.n)
    perm[which == 1] = b1.n + np.arange(b2.n)
    ts = [ta] * b1.n + [tb] * b2.n
    rs = [ra] * b1.n + [rb_] * b2.n
    mb = synth.select(mb, perm)
    seg, ln, st = tw.run([ts[i] for i in perm], False, mb.seg, mb.off, mb.length, mb.cap)
    assert (st == 0).all()
    pm = mb.copy()
    pm.seg, pm.length = seg, ln
    _, ln2, st2 = tw.run([rs[i] for i in perm], True, pm.seg, pm.off, pm.length, pm.cap)
    assert (st2 == 0).all() and np.array_equal(ln2, mb.length)


@pytest.mark.gpu
def test_short_master_key_refused(engine):
    from libjitsi_amd import SRTPContextFactory
    (k, s), = synth.keys(14, 1)  # 16-byte key for a 32-byte policy
    with pytest.raises(N.SrtpError):
        SRTPContextFactory(True, k, s, *P256_80, engine=engine)
