"""CPU: host-side pieces of the asynchronous per-packet path.

srtp_packet_may_throw decides which arrays may skip their own bundle and share
the aggregator's (srtp_rawpacket_batch_set_aggregator): it must be exactly
srtp_dispatch_plan's per-packet may-throw mark (a superset of the reference's
throws: RawPacket.getHeaderLength, SRTPCipherCTR.process bounds,
RawPacket.getSRTCPIndex -- SRTPCryptoContext.java:482-525,
SRTCPCryptoContext.java:315-374), for RTP and RTCP, both directions, every flag.
"""
import ctypes as C

import numpy as np

from libjitsi_amd import _native as N


def test_packet_may_throw_matches_dispatch_plan():
    L = N.lib()
    rng = np.random.default_rng(11)
    n = 4000
    seg = np.zeros(n * 128, np.uint8)
    off = (np.arange(n) * 128).astype(np.uint32)
    ln = rng.integers(8, 112, n).astype(np.uint32)
    cap = np.minimum(ln + rng.integers(0, 17, n), 112).astype(np.uint32)
    fl = rng.choice([0, N.PKT_FLAG_DISCARD, N.PKT_FLAG_SILENCE], n).astype(np.uint32)
    for i in range(n):
        o = int(off[i])
        seg[o:o + 128] = rng.integers(0, 256, 128, dtype=np.uint8)
        b0 = 0x80 | int(rng.integers(0, 16))
        if rng.random() < 0.5:
            b0 |= 0x10  # an extension header: its signed length decides
        seg[o] = b0
    kinds = np.array([N.KIND_RTP, N.KIND_RTCP], np.int32)
    for tag_mask in (1 << 10, (1 << 10) | (1 << 4), 1 | (1 << 10), 0x1FFF):
        for reverse in (0, 1):
            for t in (0, 1):
                shard = np.zeros(n, np.int32)
                mt = np.zeros(n, np.int32)
                rc = L.srtp_dispatch_plan(1, 1, reverse, kinds.ctypes.data, 2, tag_mask, None, t,
                                          seg.ctypes.data, seg.nbytes, off.ctypes.data, ln.ctypes.data,
                                          cap.ctypes.data, fl.ctypes.data, n, shard.ctypes.data, mt.ctypes.data)
                assert rc in (1, 2)
                got = np.array([L.srtp_packet_may_throw(int(kinds[t]), reverse,
                                                        C.c_char_p(seg[int(off[i]):int(off[i]) + 128].tobytes()),
                                                        int(ln[i]), int(cap[i]), int(fl[i]), tag_mask)
                                for i in range(n)], np.int32)
                assert np.array_equal(got, mt), (tag_mask, reverse, t)
                if t == 0 or reverse:  # RTCP protect never throws
                    assert mt.any() and not mt.all()
