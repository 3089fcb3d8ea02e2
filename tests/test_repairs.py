"""GPU: k_unprotect_fix's repairs at every density, and the crypto kernels'
lane order on mixed-size bundles, against the oracle.

k_unprotect decrypts speculatively; a packet the walk then rejects (a replay,
a forged tag) must get its ciphertext back, and one whose ROC guess was
overturned its keystream redone (SRTPCryptoContext.reverseTransformPacket
:572-705: replay check, then auth, then decryption).  k_unprotect_fix lists a
workgroup's repairs and spreads their 64-B chunks over its lanes (up to four
per lane; a workgroup with more walks one packet per lane).  These bundles
drive the three regimes: a few repairs per workgroup, a few hundred (several
chunk jobs per lane), and every packet (more jobs than lanes).  Every bundle
is compared with the oracle bit for bit: statuses, lengths, whole segment,
context state (tests/harness.py).
"""
import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


@pytest.fixture(scope="module")
def engine(engine_factory, oracle):
    return engine_factory(max_contexts=1 << 14, max_factories=64, max_transformers=64,
                          max_batch=1 << 15)


def _pair(twin, seed):
    (k, s), = synth.keys(seed, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    return twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)


@pytest.mark.parametrize("frac", [0.02, 0.15, 1.0], ids=["few", "hundreds", "all"])
def test_replays_and_forgeries_restored(engine, frac):
    """Bundle 1 accepted; bundle 2 replays a fraction of bundle 1 (whole
    1200-B packets, many chunks each) mixed with forged tags and fresh
    packets: every replay and forgery comes back as ciphertext, unchanged."""
    twin = Twin(engine)
    snd, rcv = _pair(twin, 301 + int(100 * frac))
    n = 8192
    b = synth.rtp_bundle(2 * n, 500, 1200, seed=302)
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    b.seg, b.length = seg, ln
    first = synth.select(b, np.arange(n))
    fresh = synth.select(b, np.arange(n, 2 * n))
    _, _, st1 = twin.run(rcv, True, first.seg, first.off, first.length, first.cap)
    assert (st1 == 0).all()
    rng = np.random.default_rng(303)
    k = int(frac * n)
    # bundle 2: k replays of bundle 1, the rest fresh packets, 1 % of them forged
    order = np.concatenate([np.arange(k), n + np.arange(n - k)])
    both = synth.concat([first, fresh])
    b2 = synth.select(both, order[rng.permutation(len(order))] if frac < 1.0 else order)
    forged = rng.choice(b2.n, max(1, b2.n // 100), replace=False)
    o = b2.off.astype(np.int64)
    b2.seg[o[forged] + 600] ^= 0x01
    _, _, st2 = twin.run(rcv, True, b2.seg, b2.off, b2.length, b2.cap)
    assert (st2 == N.STATUS_DROP_REPLAY).sum() >= k - len(forged)
    assert (st2 == N.STATUS_DROP_AUTH).sum() > 0 or frac == 1.0


def test_mixed_sizes_lane_order(engine):
    """Packets of 24 length classes (40 B - 4 KB) in one bundle over many
    streams, protect and unprotect, with a few forgeries: the crypto kernels
    take lanes in length-class order, and every packet still matches."""
    twin = Twin(engine)
    snd, rcv = _pair(twin, 311)
    b = synth.rtp_bundle(20000, 3000, (40, 4000), seed=312)
    seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
    assert (st == 0).all()
    rng = np.random.default_rng(313)
    o = b.off.astype(np.int64)
    bad = rng.choice(b.n, 200, replace=False)
    seg = seg.copy()
    seg[o[bad] + 20] ^= 0x80
    _, _, st2 = twin.run(rcv, True, seg, b.off, ln, b.cap)
    assert (st2 == N.STATUS_DROP_AUTH).sum() == 200
