"""GPU: the small-bundle paths against the oracle (round 4).

Bundles of up to one sort tile (2048 records) are sorted by one workgroup in
LDS (k_sort_tile) instead of the multi-pass sort, and the crypto kernels
spread a small bundle's waves over every CU in workgroups of 4-16 waves
(aes_block) instead of 16.  Both change how the work is laid out, never the
results: every bundle here is compared with the oracle bit for bit (statuses,
lengths, the whole segment, context state), at sizes around each boundary
(1, one wave, one tile, one tile + 1, the 4-wave / 8-wave workgroup switch),
with every sort-key width the engine uses (one 8-bit pass, two, and the wide
two-pass sort), mixed packet lengths (the length-class lane order), invalid
and skipped packets (records that are sorted but not walked), faults and
several transformers per bundle.
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

# max_contexts -> context table 2 * next_pow2 slots -> sort key ctx_bits + 1:
# 8 bits (one pass), 14 bits (two 8-bit passes), 18 bits (an 8-bit pass and a
# 10-bit one), 20 bits (wide: two 10-bit passes)
TABLES = {"key8": 64, "key14": 1 << 12, "key18": 1 << 16, "key20": 1 << 18}


@pytest.fixture(scope="module", params=list(TABLES), ids=list(TABLES))
def twin(request, engine_factory, oracle):
    e = engine_factory(max_contexts=TABLES[request.param], max_factories=64, max_transformers=64)
    return Twin(e)


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 2047, 2048, 2049, 5000])
def test_bundle_sizes_round_trip(twin, n):
    """Protect and unprotect (with faults) of n mixed-size packets over two
    transformers per direction, a few packets invalid (length < 12) or
    skipped."""
    rng = np.random.default_rng(1000 + n)
    (k, s), = synth.keys(900 + n, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd = [twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fs)]
    rcv = [twin.transformer(O.KIND_RTP, fr), twin.transformer(O.KIND_RTP, fr)]
    n_ssrc = max(1, min(16, n // 3))  # 2 x 16 contexts: the key8 table holds 64
    b = synth.rtp_bundle(n, n_ssrc, (40, 1400), seed=1100 + n, ext_frac=0.1)
    who = (np.arange(n) % n_ssrc) % 2  # each SSRC through one of the two transformers
    flags = np.zeros(n, np.uint32)
    ln = b.length.copy()
    if n >= 64:
        ln[rng.choice(n, 2, replace=False)] = 8  # RawPacket.isInvalid
        flags[rng.choice(n, 2, replace=False)] = N.PKT_FLAG_SKIP
    seg, ln2, st = twin.run([snd[w] for w in who], False, b.seg, b.off, ln, b.cap, flags)
    assert (st == N.STATUS_OK).sum() >= n - 4
    seg = seg.copy()
    o = b.off.astype(np.int64)
    ok = np.nonzero(st == N.STATUS_OK)[0]
    if len(ok) > 4:  # a forged packet and a tag bit flipped
        seg[o[ok[len(ok) // 2]] + 14] ^= 1
        i = ok[-1]
        seg[o[i] + int(ln2[i]) - 1] ^= 0x40
    twin.run([rcv[w] for w in who], True, seg, b.off, ln2, b.cap, flags)
    # the same packets again: every one a replay now
    _, _, st3 = twin.run([rcv[w] for w in who], True, seg, b.off, ln2, b.cap, flags)
    assert (st3 == N.STATUS_OK).sum() == 0
    for t in snd + rcv:  # the contexts become tombstones for the next size
        t.close()
    fs.close()
    fr.close()


def test_many_key_sets_one_small_bundle(engine_factory, oracle):
    """A bundle like the per-packet path's: one packet per transformer, each
    transformer its own factory (key set), _80 and _32, SRTP and SRTCP --
    every wave mixes key sets (the per-lane key schedule) -- then faults."""
    twin = Twin(engine_factory(max_contexts=1 << 12, max_factories=64, max_transformers=128))
    T = 24
    facs = []
    for j in range(T):
        (k, s), = synth.keys(2000 + j, 1)
        pols = P80 if j % 3 else P32
        facs.append((twin.factory(True, k, s, *pols), twin.factory(False, k, s, *pols), pols))
    snd = [twin.transformer(O.KIND_RTP, f[0]) for f in facs]
    rcv = [twin.transformer(O.KIND_RTP, f[1]) for f in facs]
    b = synth.rtp_bundle(300, 100, (60, 1300), seed=2100)
    who = np.arange(300) % T
    seg, ln, st = twin.run([snd[w] for w in who], False, b.seg, b.off, b.length, b.cap)
    assert (st == N.STATUS_OK).all()
    seg = seg.copy()
    seg[int(b.off[17]) + 30] ^= 4
    twin.run([rcv[w] for w in who], True, seg, b.off, ln, b.cap)
    # SRTCP of the same factories
    csnd = [twin.transformer(O.KIND_RTCP, f[0]) for f in facs]
    crcv = [twin.transformer(O.KIND_RTCP, f[1]) for f in facs]
    cb = synth.rtcp_bundle(120, 30, seed=2101)
    cwho = np.arange(120) % T
    cseg, cln, cst = twin.run([csnd[w] for w in cwho], False, cb.seg, cb.off, cb.length, cb.cap)
    assert (cst == N.STATUS_OK).all()
    twin.run([crcv[w] for w in cwho], True, cseg, cb.off, cln, cb.cap)


def test_spread_workgroup_boundaries(engine_factory, oracle):
    """Bundle sizes where the crypto kernels' workgroup changes: up to 4
    waves per CU (4-wave workgroups), 5-8 (8-wave), and a full 16; the
    protect and unprotect of each against the oracle, C3 faults on the way
    back."""
    e = engine_factory(max_contexts=1 << 15, max_factories=16, max_transformers=16)
    twin = Twin(e)
    (k, s), = synth.keys(3000, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    for n in (16384 + 64, 65536 + 64, 140000):
        rng = np.random.default_rng(n)
        b = synth.rtp_bundle(n, 2000, (60, 300), seed=3100 + n)
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap, check_state=False)
        assert (st == N.STATUS_OK).all()
        pb = b.copy()
        pb.seg, pb.length = seg, ln
        fb = G.inject_faults(pb, rng)
        twin.run(rcv, True, fb.seg, fb.off, fb.length, fb.cap, check_state=False)


def test_maximum_size_packets(engine_factory, oracle):
    """Packets up to the 64-KB region limit, RTP and RTCP, in a small bundle
    (k_ctr_small's lanes loop over thousands of counter blocks per packet; the
    MAC-only kernels hash a thousand blocks) and in a large one (the fused
    kernels' counter precompute runs out past block 256 and the generic loop
    finishes), each against the oracle with a forged packet on the way back."""
    e = engine_factory(max_contexts=1 << 12, max_factories=16, max_transformers=16)
    twin = Twin(e)
    (k, s), = synth.keys(4000, 1)
    fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
    snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
    csnd, crcv = twin.transformer(O.KIND_RTCP, fs), twin.transformer(O.KIND_RTCP, fr)
    for n, lens in ((6, (40000, 65000)), (9000, (3000, 9000))):
        b = synth.rtp_bundle(n, 3, lens, seed=4100 + n)
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap, check_state=n < 100)
        assert (st == N.STATUS_OK).all()
        seg = seg.copy()
        seg[int(b.off[n - 1]) + 1000] ^= 2
        _, _, st2 = twin.run(rcv, True, seg, b.off, ln, b.cap, check_state=n < 100)
        assert (st2 == N.STATUS_DROP_AUTH).sum() == 1
    cb = synth.rtcp_bundle(5, 2, len_range=(30000, 60000), seed=4200)
    cseg, cln, cst = twin.run(csnd, False, cb.seg, cb.off, cb.length, cb.cap)
    assert (cst == N.STATUS_OK).all()
    twin.run(crcv, True, cseg, cb.off, cln, cb.cap)
