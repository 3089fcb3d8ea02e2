"""GPU: the bundle aggregator (srtp_aggregator_*) against the
oracle.

The reference transforms one packet per call: RTPConnectorInputStream.java
:425-452 and RTPConnectorOutputStream.java:268-300,652-830 pass 1-element
arrays through SinglePacketTransformer.java:121-216. Here several producer
threads submit packets of several transformers concurrently. The aggregator
bundles them, and its callbacks report each packet's outcome in completion
order. The oracle then runs every packet as its own 1-element array, in that
same order, and each status, length and byte must match. Each producer's
packets must complete in its submission order. A packet the cipher throws on
must not stop its transformer's later packets.
"""
import threading
import time

import numpy as np
import pytest

from libjitsi_amd import SRTPAggregator, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
P32 = profile_policies("AES_CM_128_HMAC_SHA1_32")


def oracle_one(t, reverse, data, flags=0):
    """One packet through the oracle as a 1-element array."""
    L = len(data)
    cap = L if reverse else L + 16
    seg = np.zeros(max((cap + 15) // 16 * 16, 16), np.uint8)
    seg[:L] = np.frombuffer(data, np.uint8)
    ln = np.array([L], np.uint32)
    st = O.process(t.o, reverse, seg, np.zeros(1, np.uint32), ln, np.array([cap], np.uint32),
                   np.array([flags], np.uint32), False)
    return int(st[0]), seg[:int(ln[0])].tobytes()


class Collector:
    def __init__(self):
        self.lock = threading.Lock()
        self.got = []

    def __call__(self, cookie, status, data):
        with self.lock:
            self.got.append((cookie, status, data))


def packets(b):
    o = b.off.astype(np.int64)
    return [b.seg[o[i]:o[i] + int(b.length[i])].tobytes() for i in range(b.n)]


def run_producers(agg, items, n_threads, reverse):
    """items: list of (transformer, data, flags); thread k submits items k, k+n, ..."""
    def work(k):
        for i in range(k, len(items), n_threads):
            t, data, fl = items[i]
            agg.submit(reverse, t.e, data, fl, cookie=i)
    th = [threading.Thread(target=work, args=(k,)) for k in range(n_threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    agg.flush()


def check_against_oracle(col, items, reverse, n_threads):
    got = list(col.got)
    cookies = [c for c, _, _ in got]
    assert sorted(cookies) == list(range(len(items)))
    pos = {c: i for i, c in enumerate(cookies)}
    for k in range(n_threads):  # each producer's packets complete in its order
        mine = [pos[i] for i in range(k, len(items), n_threads)]
        assert mine == sorted(mine)
    outs = {}
    for c, st, data in got:  # the oracle, one packet at a time, in completion order
        t, inp, fl = items[c]
        st_o, out_o = oracle_one(t, reverse, inp, fl)
        assert st == st_o, (c, N.STATUS_NAMES[st] if 0 <= st < 10 else st, N.STATUS_NAMES[st_o])
        assert data == out_o, (c, len(data), len(out_o))
        outs[c] = (st, data)
    return outs


def test_concurrent_producers_vs_oracle(engine_factory, oracle):
    E = engine_factory(abort_on_error=False, max_contexts=4096, max_factories=64,
                       max_transformers=64)
    tw = Twin(E)
    (k1, s1), (k2, s2) = synth.keys(71, 2)
    f1s, f1r = tw.factory(True, k1, s1, *P80), tw.factory(False, k1, s1, *P80)
    f2s, f2r = tw.factory(True, k2, s2, *P32), tw.factory(False, k2, s2, *P32)
    A, rA = tw.transformer(O.KIND_RTP, f1s), tw.transformer(O.KIND_RTP, f1r)
    B, rB = tw.transformer(O.KIND_RTP, f2s), tw.transformer(O.KIND_RTP, f2r)
    Cc, rC = tw.transformer(O.KIND_RTCP, f1s), tw.transformer(O.KIND_RTCP, f1r)
    ba = synth.rtp_bundle(300, 8, (40, 1300), seed=72, seq0=np.full(8, 65400, np.uint32))
    bb = synth.rtp_bundle(200, 3, (40, 600), seed=73)
    bc = synth.rtcp_bundle(60, 4, seed=74)
    pa, pb, pc = packets(ba), packets(bb), packets(bc)
    for i in (17, 150, 151):  # CC=15: the cipher throws (ERR_MALFORMED, this packet only)
        x = bytearray(pa[i][:60])
        x[0] = 0x8F
        pa[i] = bytes(x)
    fa = [0] * len(pa)
    fa[30] = N.PKT_FLAG_DISCARD
    items = []  # interleave the three streams
    ia = ib = ic = 0
    rng = np.random.default_rng(75)
    while ia < len(pa) or ib < len(pb) or ic < len(pc):
        r = rng.random()
        if r < 0.55 and ia < len(pa):
            items.append((A, pa[ia], fa[ia])); ia += 1
        elif r < 0.85 and ib < len(pb):
            items.append((B, pb[ib], 0)); ib += 1
        elif ic < len(pc):
            items.append((Cc, pc[ic], 0)); ic += 1
    col = Collector()
    agg = SRTPAggregator(E, col, max_packets=64, max_bytes=1 << 20, deadline_us=500, depth=4)
    try:
        run_producers(agg, items, 4, False)
        outs = check_against_oracle(col, items, False, 4)
        st = np.array([outs[i][0] for i in range(len(items))])
        # producers reorder a stream's packets slightly: the sender's own replay
        # check (SRTPCryptoContext.transformPacket) may drop a late one, as the oracle does
        assert (st == N.STATUS_ERR_MALFORMED).sum() == 3 and (st == 0).sum() > 0.9 * len(items)
        assert agg.stats()["bundles"] >= len(items) // 64

        # receive side: the protected packets, plus replays and a forged tag
        rmap = {id(A): rA, id(B): rB, id(Cc): rC}
        ritems = [(rmap[id(t)], outs[i][1], 0) for i, (t, _, _) in enumerate(items)
                  if outs[i][0] == 0]
        ritems += [ritems[5], ritems[40], ritems[41]]
        forged = bytearray(ritems[60][1])
        forged[-1] ^= 1
        ritems.append((ritems[60][0], bytes(forged), 0))
        col.got.clear()
        run_producers(agg, ritems, 3, True)
        routs = check_against_oracle(col, ritems, True, 3)
        rst = np.array([routs[i][0] for i in range(len(ritems))])
        assert (rst == 0).sum() > 0.9 * len(ritems)
        assert (rst[-4:] != 0).all()  # the three replays and the forged tag
    finally:
        agg.close()


def test_deadline_flush(engine_factory, oracle):
    E = engine_factory(abort_on_error=False, max_contexts=1024, max_factories=16,
                       max_transformers=16)
    tw = Twin(E)
    (k, s), = synth.keys(76, 1)
    A = tw.transformer(O.KIND_RTP, tw.factory(True, k, s, *P80))
    col = Collector()
    agg = SRTPAggregator(E, col, max_packets=1024, deadline_us=2000, depth=3)
    try:
        b = synth.rtp_bundle(5, 1, (100, 200), seed=77)
        for i, d in enumerate(packets(b)):
            agg.submit(False, A.e, d, cookie=i)
        t0 = time.time()
        while len(col.got) < 5 and time.time() - t0 < 5:
            time.sleep(0.005)
        assert len(col.got) == 5  # sealed by the deadline, no flush
        assert [c for c, _, _ in col.got] == list(range(5))
    finally:
        agg.close()


def test_backpressure_many_bundles(engine_factory, oracle):
    """More packets than the slots hold: producers block and resume."""
    E = engine_factory(abort_on_error=False, max_contexts=4096, max_factories=16,
                       max_transformers=16)
    tw = Twin(E)
    (k, s), = synth.keys(78, 1)
    A = tw.transformer(O.KIND_RTP, tw.factory(True, k, s, *P80))
    b = synth.rtp_bundle(3000, 50, (60, 300), seed=79)
    items = [(A, d, 0) for d in packets(b)]
    col = Collector()
    agg = SRTPAggregator(E, col, max_packets=32, max_bytes=1 << 16, deadline_us=200, depth=3)
    try:
        run_producers(agg, items, 6, False)
        check_against_oracle(col, items, False, 6)
        assert agg.stats()["completed"] == len(items)
    finally:
        agg.close()


def test_refuses_abort_on_error_engine(engine_factory):
    E = engine_factory(abort_on_error=True, max_contexts=1024, max_factories=16,
                       max_transformers=16)
    with pytest.raises(N.SrtpError):
        SRTPAggregator(E, lambda *a: None)
