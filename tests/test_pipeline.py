"""GPU: the pinned-host bundle pipeline (srtp_pipeline_*, SURVEY.md 8d
end-to-end path / 8f.2 bundle former) against the CPU oracle.

Bundles are packed straight into the pipeline's pinned slots, several are in
flight at once (H2D of one overlapping the kernels of another), and each
slot's results must equal the oracle's for the same bundles processed in
submission order: statuses, lengths and every segment byte.
"""
import numpy as np
import pytest

from libjitsi_amd import SRTPPipeline, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu

P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


def pack_into(slot, b, tids=None, flags=None):
    """Pack bundle b into a pinned slot; returns the segment bytes used."""
    nb = len(b.seg)
    slot["seg"][:nb] = b.seg
    slot["off"][:b.n] = b.off
    slot["len"][:b.n] = b.length
    slot["cap"][:b.n] = b.cap
    if tids is not None:
        slot["tids"][:b.n] = tids
    if flags is not None:
        slot["flags"][:b.n] = flags
    return nb


def oracle_run(t, reverse, b, tids_o=None, flags=None):
    seg, ln = b.seg.copy(), b.length.copy()
    st = O.process(tids_o if tids_o is not None else t, reverse, seg, b.off, ln, b.cap, flags)
    return seg, ln, np.asarray(st, np.int32)


@pytest.mark.parametrize("depth", [1, 3])
def test_pipeline_round_trips_match_oracle(engine_factory, oracle, depth):
    eng = engine_factory(max_contexts=1 << 14, max_factories=64, max_transformers=64,
                         max_batch=1 << 12)
    tw = Twin(eng)
    (k, s), = synth.keys(61, 1)
    fs, fr = tw.factory(True, k, s, *P80), tw.factory(False, k, s, *P80)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    bundles = [synth.rtp_bundle(1500, 40, (60, 1400), seed=600 + i, ext_frac=0.1,
                                ssrcs=np.arange(40, dtype=np.uint32) + 1,
                                seq0=np.full(40, (65500 + 38 * i) & 0xFFFF, np.uint32))
               for i in range(7)]
    max_seg = max(len(b.seg) for b in bundles)
    pl = SRTPPipeline(eng, max_packets=1500, max_seg_bytes=max_seg, depth=depth)
    # protect: submit round-robin over the slots, compare each when it completes
    expect, pending = [], {}
    for i, b in enumerate(bundles):
        expect.append(oracle_run(snd.o, False, b))
        j = i % depth
        if j in pending:
            check_slot(pl, j, *pending.pop(j))
        nb = pack_into(pl.slot(j), b)
        pl.submit(j, False, b.n, nb, tid=snd.tid)
        pending[j] = (expect[i], b)
    for j, args in list(pending.items()):
        check_slot(pl, j, *args)
    # unprotect the protected bundles, with DISCARD/SILENCE flags on some
    pending = {}
    for i, b in enumerate(bundles):
        pb = b.copy()
        pb.seg, pb.length = expect[i][0], expect[i][1]
        flags = np.zeros(pb.n, np.uint32)
        flags[i::17] = N.PKT_FLAG_SILENCE
        exp = oracle_run(rcv.o, True, pb, flags=flags)
        j = i % depth
        if j in pending:
            check_slot(pl, j, *pending.pop(j))
        nb = pack_into(pl.slot(j), pb, tids=np.full(pb.n, rcv.tid, np.int32), flags=flags)
        pl.submit(j, True, pb.n, nb, tid=None, use_flags=True)
        pending[j] = (exp, pb)
    for j, args in list(pending.items()):
        check_slot(pl, j, *args)
    pl.close()


def check_slot(pl, j, exp, b):
    pl.wait(j)
    sl = pl.slot(j)
    seg, ln, st = exp
    np.testing.assert_array_equal(sl["status"][:b.n], st)
    np.testing.assert_array_equal(sl["len"][:b.n], ln)
    np.testing.assert_array_equal(sl["seg"][:len(seg)], seg)


def test_pipeline_rejects_bad_regions(engine_factory):
    eng = engine_factory(max_contexts=1024, max_factories=8, max_transformers=8, max_batch=64)
    tw = Twin(eng)
    (k, s), = synth.keys(62, 1)
    t = tw.transformer(O.KIND_RTP, tw.factory(True, k, s, *P80))
    pl = SRTPPipeline(eng, max_packets=16, max_seg_bytes=4096, depth=2)
    b = synth.rtp_bundle(4, 1, 100, seed=1)
    nb = pack_into(pl.slot(0), b)
    pl.slot(0)["off"][1] = 8  # not 16-B aligned
    with pytest.raises(N.SrtpError):
        pl.submit(0, False, b.n, nb, tid=t.tid)
    pl.slot(0)["off"][1] = 4096  # outside the segment
    with pytest.raises(N.SrtpError):
        pl.submit(0, False, b.n, nb, tid=t.tid)
    with pytest.raises(N.SrtpError):  # more packets than the slot holds
        pl.submit(0, False, 17, nb, tid=t.tid)
    pl.close()


@pytest.mark.parametrize("n,lens", [(1, (1200, 1200)), (7, (60, 400)), (40, (100, 1400)),
                                    (60, (1100, 1200)), (255, (60, 200))])
def test_pipeline_small_bundles_one_launch(engine_factory, oracle, n, lens):
    """Bundles k_small takes through the pipeline: those of <= 64 KB in direct
    mode (the kernel reads the slot's packed block from pinned host memory and
    writes lengths, statuses and packets back: no copies), larger ones with
    the copies (60 x ~1.2 KB); protect, then unprotect with a forged packet
    and a replay, in flight over three slots; every slot against the oracle."""
    eng = engine_factory(max_contexts=1 << 12, max_factories=16, max_transformers=16, max_batch=1 << 10)
    tw = Twin(eng)
    (k, s), = synth.keys(70 + n, 1)
    fs, fr = tw.factory(True, k, s, *P80), tw.factory(False, k, s, *P80)
    snd, rcv = tw.transformer(O.KIND_RTP, fs), tw.transformer(O.KIND_RTP, fr)
    n_ssrc = max(1, min(8, n // 3))
    bundles = [synth.rtp_bundle(n, n_ssrc, lens, seed=7000 + 10 * n + i, ext_frac=0.1,
                                ssrcs=np.arange(n_ssrc, dtype=np.uint32) + 0x3000 + n)
               for i in range(4)]
    # consecutive bundles continue each stream's sequence
    for i, b in enumerate(bundles):
        per = (n + n_ssrc - 1) // n_ssrc
        for p in range(n):
            q = (1000 + i * per + p // n_ssrc) & 0xFFFF
            b.seg[b.off[p] + 2] = q >> 8
            b.seg[b.off[p] + 3] = q & 0xFF
    max_seg = max(len(b.seg) for b in bundles) + 4096
    pl = SRTPPipeline(eng, max_packets=max(n, 4) + 1, max_seg_bytes=max_seg, depth=3)
    c0 = eng.stats()["small_bundles"]
    expect, pending = [], {}
    for i, b in enumerate(bundles):
        expect.append(oracle_run(snd.o, False, b))
        j = i % 3
        if j in pending:
            check_slot(pl, j, *pending.pop(j))
        nb = pack_into(pl.slot(j), b)
        pl.submit(j, False, b.n, nb, tid=snd.tid)
        pending[j] = (expect[i], b)
    for j, args in list(pending.items()):
        check_slot(pl, j, *args)
    pending = {}
    for i, b in enumerate(bundles):
        pb = b.copy()
        pb.seg, pb.length = expect[i][0].copy(), expect[i][1]
        order = np.arange(pb.n)
        if i == 1 and n > 1:
            pb.seg[int(pb.off[n // 2]) + 14] ^= 1   # a forged payload byte
        if i == 2 and n > 1:
            order = np.concatenate([order[:-1], [0]])  # packet 0 again instead of the last: a replay
        sub = synth.select(pb, order)
        exp = oracle_run(rcv.o, True, sub)
        j = i % 3
        if j in pending:
            check_slot(pl, j, *pending.pop(j))
        nb = pack_into(pl.slot(j), sub)
        pl.submit(j, True, sub.n, nb, tid=rcv.tid)
        pending[j] = (exp, sub)
    for j, args in list(pending.items()):
        check_slot(pl, j, *args)
    assert eng.stats()["small_bundles"] - c0 == 8  # every bundle in one launch
    pl.close()
