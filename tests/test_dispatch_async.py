"""GPU: asynchronous host bundles through the dispatcher
(srtp_dispatch_submit_host / srtp_dispatch_wait_host).

A connector's send thread keeps several bundles in flight
(RTPConnectorOutputStream.java:268-300 hands a packet on and returns to its
queue): the next bundle is packed and sent while the previous one's last
chunks come back.  Bundles over the same contexts must still be processed in
submission order on every shard, and a synchronous call in between is
ordered with them.  Each scenario submits a sequence of bundles (sharing
SSRCs, so every context's state carries from one bundle to the next), waits
for them in a scrambled order, and compares every status, length and byte,
and the final context states, with the oracle running the same bundles one
after another in submission order.
"""
import numpy as np
import pytest

from libjitsi_amd import SRTPDispatcher, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


def _gpus():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def _bundles(nb, n, nssrc, seed, lens=(60, 1400)):
    """nb bundles over the same SSRCs, each advancing every SSRC's sequence."""
    out = []
    base = synth.rtp_bundle(n, nssrc, lens, seed=seed)
    per = np.bincount(np.arange(n) % nssrc, minlength=nssrc)[np.arange(n) % nssrc]
    o = base.off.astype(np.int64)
    for k in range(nb):
        b = synth.rtp_bundle(n, nssrc, lens, seed=seed)
        q = ((b.seg[o + 2].astype(np.int64) << 8) | b.seg[o + 3]) + k * per
        b.seg[o + 2] = (q >> 8) & 0xFF
        b.seg[o + 3] = q & 0xFF
        out.append(b)
    return out


@pytest.fixture(params=[1, 3], ids=["G1", "G3"])
def dtwin(request, oracle):
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    d = SRTPDispatcher([0] * request.param, max_contexts=1 << 14, max_factories=64,
                       max_transformers=64)
    yield Twin(d)
    d.close()


def _check(twin, t, reverse, bundles, results):
    """Oracle over the bundles in submission order against the engine's results."""
    outs = []
    for b, (seg_e, len_e, st_e) in zip(bundles, results):
        seg_o, len_o = b.seg.copy(), b.length.copy()
        st_o = O.process(t.o, reverse, seg_o, b.off, len_o, b.cap)
        bad = np.nonzero(st_o != st_e)[0]
        assert len(bad) == 0, f"status mismatch at {bad[:8].tolist()}: {st_o[bad[:8]]} vs {st_e[bad[:8]]}"
        assert np.array_equal(len_o, len_e)
        assert np.array_equal(seg_o, seg_e), "segment bytes differ from the oracle"
        outs.append((seg_o, len_o, st_o))
    return outs


def test_async_bundles_in_order_waits_scrambled(dtwin):
    """Six protect bundles in flight over the same 300 SSRCs (two chunks
    each on one shard), waited for in the order 2, 0, 5, 1, 4, 3; then their
    unprotect, the same way, with a synchronous call between the submits."""
    d = dtwin.engine
    (k, s), = synth.keys(81, 1)
    fs, fr = dtwin.factory(True, k, s, *P80), dtwin.factory(False, k, s, *P80)
    snd, rcv = dtwin.transformer(O.KIND_RTP, fs), dtwin.transformer(O.KIND_RTP, fr)
    bs = _bundles(6, 40000, 300, seed=82, lens=(60, 1400))
    work = [(b.seg.copy(), b.length.copy()) for b in bs]
    tk = [d.submit_host(False, snd.tid, w[0], b.off, w[1], b.cap) for b, w in zip(bs, work)]
    st = {}
    for i in (2, 0, 5, 1, 4, 3):
        st[i] = tk[i].wait()
    prot = _check(dtwin, snd, False, bs, [(w[0], w[1], st[i]) for i, w in enumerate(work)])
    # unprotect: the protected bundles, a synchronous call after the third submit
    rb = []
    for seg_o, len_o, _ in prot:
        rb.append((seg_o.copy(), len_o.copy()))
    tk2 = []
    for i, ((seg_i, len_i), b) in enumerate(zip(rb, bs)):
        if i == 3:
            st3 = d.transform_host(True, rcv.tid, seg_i, b.off, len_i, b.cap)
            tk2.append(None)
            continue
        tk2.append(d.submit_host(True, rcv.tid, seg_i, b.off, len_i, b.cap))
    st2 = {3: st3}
    for i in (5, 1, 0, 2, 4):
        st2[i] = tk2[i].wait()
    for i, (b, (seg_o, len_o, _)) in enumerate(zip(bs, prot)):
        so, lo = seg_o.copy(), len_o.copy()
        st_o = O.process(rcv.o, True, so, b.off, lo, b.cap)
        assert np.array_equal(st_o, st2[i]), f"bundle {i}: statuses differ"
        assert np.array_equal(lo, rb[i][1]) and np.array_equal(so, rb[i][0]), f"bundle {i}: bytes differ"
    dtwin.check_states([snd] * bs[0].n, bs[-1].seg, bs[-1].off, bs[-1].length)
    dtwin.check_states([rcv] * bs[0].n, bs[-1].seg, bs[-1].off, bs[-1].length)


def test_async_throwing_bundle_and_ticket_errors(dtwin):
    """A bundle with a packet that throws (the rollback path, which runs
    inside its submit) between two asynchronous ones; an unknown ticket, a
    ticket waited twice."""
    d = dtwin.engine
    (k, s), = synth.keys(84, 1)
    fs = dtwin.factory(True, k, s, *P80)
    snd = dtwin.transformer(O.KIND_RTP, fs)
    bs = _bundles(3, 3000, 40, seed=85, lens=(40, 700))
    o = bs[1].off.astype(np.int64)
    for i in (100, 1500):  # CC=15 with X: the header length runs past the packet
        bs[1].seg[o[i]] = 0x9F
    work = [(b.seg.copy(), b.length.copy()) for b in bs]
    tk = [d.submit_host(False, snd.tid, w[0], b.off, w[1], b.cap) for b, w in zip(bs, work)]
    sts = [t.wait() for t in tk]
    assert (sts[1] == N.STATUS_ERR_MALFORMED).any() and (sts[1] == N.STATUS_NOT_PROCESSED).any()
    _check(dtwin, snd, False, bs, [(w[0], w[1], st) for w, st in zip(work, sts)])
    with pytest.raises(Exception):
        N.check(N.lib().srtp_dispatch_wait_host(d.h, tk[0].ticket), None, "wait", dispatch=d.h)
    with pytest.raises(Exception):
        N.check(N.lib().srtp_dispatch_wait_host(d.h, 987654321), None, "wait", dispatch=d.h)


def test_async_outstanding_limit_and_destroy(oracle):
    """At most 64 bundles outstanding (SRTP_EAGAIN beyond); a dispatcher
    destroyed with bundles never waited for completes them first."""
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    d = SRTPDispatcher([0, 0], max_contexts=4096, max_factories=8, max_transformers=8)
    twin = Twin(d)
    (k, s), = synth.keys(86, 1)
    fs = twin.factory(True, k, s, *P80)
    snd = twin.transformer(O.KIND_RTP, fs)
    bs = _bundles(65, 64, 8, seed=87, lens=(100, 300))
    work = [(b.seg.copy(), b.length.copy()) for b in bs]
    tk = [d.submit_host(False, snd.tid, w[0], b.off, w[1], b.cap) for b, w in zip(bs[:64], work[:64])]
    with pytest.raises(Exception):
        d.submit_host(False, snd.tid, work[64][0], bs[64].off, work[64][1], bs[64].cap)
    sts = [t.wait() for t in tk]
    _check(twin, snd, False, bs[:64], [(w[0], w[1], st) for w, st in zip(work[:64], sts)])
    # never waited for: destroy completes it into the caller's arrays
    w = (bs[64].seg.copy(), bs[64].length.copy())
    t = d.submit_host(False, snd.tid, w[0], bs[64].off, w[1], bs[64].cap)
    d.close()
    seg_o, len_o = bs[64].seg.copy(), bs[64].length.copy()
    st_o = O.process(snd.o, False, seg_o, bs[64].off, len_o, bs[64].cap)
    assert (st_o == 0).all() and np.array_equal(seg_o, w[0]) and np.array_equal(len_o, w[1])
    assert t.ticket > 0
