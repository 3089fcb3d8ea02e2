"""GPU parity for every HMAC-SHA1 tag length the engine accepts (1..12 bytes;
SRTPPolicy.authTagLength, BaseSRTPCryptoContext.java:269-278 truncates the
digest to it), SRTP and SRTCP in one bundle, packet lengths 60-1400 B so the
trailer starts at every alignment: k_protect writes the E|index word and the
tag with word stores when they start 4-byte aligned and byte stores otherwise;
k_unprotect compares the received tag from its 16-B piece(s), one or two.
Protect, tamper with some tags, then unprotect -- oracle and
engine on identical bytes, statuses, lengths, segment and context state
bit-exact.  Bundles of 9000 packets run the fused kernels; bundles of 700 the
small-bundle path (k_ctr_small + the MAC-only kernels)."""
import numpy as np
import pytest

from libjitsi_amd import SRTPPolicy, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu

P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 14, max_factories=256, max_transformers=512)


def with_tag(p: SRTPPolicy, T: int) -> SRTPPolicy:
    return SRTPPolicy(p.encType, p.encKeyLength, p.authType, p.authKeyLength, T, p.saltKeyLength)


@pytest.mark.parametrize("n_rtp", [9000, 700], ids=["fused", "small"])
@pytest.mark.parametrize("T", list(range(1, 13)))
def test_every_tag_length_round_trip_with_tampering(engine, T, n_rtp):
    twin = Twin(engine)
    pols = [with_tag(p, T) for p in P80]
    (k, s), = synth.keys(700 + T, 1)
    fs, fr = twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols)
    rtp_s, rtp_r = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    rtcp_s, rtcp_r = twin.transformer(O.KIND_RTCP, fs), twin.transformer(O.KIND_RTCP, fr)
    rb = synth.rtp_bundle(n_rtp, 40, (60, 1400), seed=8000 + T, ext_frac=0.1)
    cb = synth.rtcp_bundle(max(40, n_rtp // 20), 5, seed=9000 + T)
    b = synth.concat([rb, cb])  # each stream in order (the sender's replay check too)
    rng = np.random.default_rng(T * 31 + n_rtp)
    is_rtp = np.arange(b.n) < rb.n
    ts_s = [rtp_s if r else rtcp_s for r in is_rtp]
    ts_r = [rtp_r if r else rtcp_r for r in is_rtp]
    # the trailer starts at every offset mod 16
    assert len({int(x) % 16 for x in b.length[is_rtp]}) == 16
    seg, ln, st = twin.run(ts_s, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    # tamper: one bit of the tag (always detected: every tag byte is compared;
    # a flipped E|index bit would pass a 1-byte tag one time in 256)
    seg = seg.copy()
    bad = np.nonzero(rng.random(b.n) < 0.03)[0]
    for i in bad:
        L = int(ln[i])
        pos = int(rng.integers(L - T, L))
        seg[b.off[i] + pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
    seg2, ln2, st2 = twin.run(ts_r, True, seg, b.off, ln, b.cap)
    good = np.setdiff1d(np.arange(b.n), bad)
    assert (st2[good] == 0).all()
    assert (st2[bad] != 0).all()
    assert (st2[bad] == N.STATUS_DROP_AUTH).sum() > 0
    np.testing.assert_array_equal(ln2[good], b.length[good])
