"""GPU: the RawPacket[] marshalling of the Java drop-in -- the C functions a
JNI shim calls (srtp_rawpacket_transform, libjitsi_amd/csrc/rawpacket.cpp),
driven through SRTPTransformer.transform / reverseTransform and
transform_bundle on one engine and on a 3-shard dispatcher -- against the
oracle on the same bytes and against the Java buffer rules:

* SinglePacketTransformer.java:121-216 -- array order, null elements skipped,
  each element replaced by the result or null, the same array returned, a
  throw rethrown after the earlier packets were transformed, later packets
  untouched;
* RawPacket.append (RawPacket.java:203-220) -- in place when the buffer has
  room after the payload, else a new buffer of exactly length + tag;
* RawPacket.grow (:885-893) -- SRTCP protect always gets a new buffer of
  length + 4 + tag (SRTCPCryptoContext.java:413);
* RawPacket.shrink (:1284-1292) -- unprotect shrinks in place, also for a
  packet whose tag check fails or that throws after the shrink.
"""
import copy

import numpy as np
import pytest

from libjitsi_amd import (RawPacket, SRTCPTransformer, SRTPContextFactory, SRTPTransformer,
                          SRTPTransformException, pack, profile_policies, synth, transform_bundle)
from libjitsi_amd.srtp import _rp_batch
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import opol

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
RNG = np.random.default_rng(5150)


@pytest.fixture(scope="module", params=["engine", "dispatch3"])
def eng(request, engine_factory, oracle):
    if request.param == "engine":
        yield engine_factory(max_contexts=4096, max_factories=256, max_transformers=256)
        return
    from libjitsi_amd import SRTPDispatcher
    d = SRTPDispatcher([0] * 3, max_contexts=4096, max_factories=256, max_transformers=256)
    yield d
    d.close()


def rtp(seq, ssrc, L, b0=0x80, room=0, offset=0, cc_ext=None):
    """A RawPacket whose buffer holds `offset` junk bytes, the packet, and
    `room` spare bytes after it."""
    p = bytearray(RNG.integers(0, 256, L, dtype=np.uint8).tobytes())
    p[0], p[1] = b0, 96
    p[2:4] = (seq & 0xFFFF).to_bytes(2, "big")
    p[8:12] = ssrc.to_bytes(4, "big")
    if cc_ext is not None:
        cc = b0 & 0x0F
        p[12 + 4 * cc + 2:12 + 4 * cc + 4] = cc_ext.to_bytes(2, "big")
    buf = bytes(RNG.integers(0, 256, offset, dtype=np.uint8)) + bytes(p) + bytes(room)
    return RawPacket(buf, offset, L)


def oracle_run(ot, pkts, reverse):
    seg, off, ln, cap, fl = pack(pkts, reverse=reverse)
    st = O.process(ot, reverse, seg, off, ln, cap, fl)
    return seg, off, ln, st


def snapshot(p):
    return None if p is None else (bytes(p.buffer), p.offset, p.length, id(p.buffer))


def test_protect_unprotect_rawpackets(eng):
    (k, s), = synth.keys(500, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *P80, engine=eng))
    of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
    ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
    ot, otr = O.Transformer(O.KIND_RTP, of, of), O.Transformer(O.KIND_RTP, ofr, ofr)
    pkts = []
    for i in range(60):
        room = 10 if i % 3 == 0 else (0 if i % 3 == 1 else 64)  # exact fit / realloc / spare
        pkts.append(rtp(100 + i // 4, 0x1000 + i % 4, int(RNG.integers(60, 1300)), room=room,
                        offset=int(RNG.integers(0, 40))))
    pkts[7] = None
    pkts[33] = None
    before = [snapshot(p) for p in pkts]
    bufs = [None if p is None else p.buffer for p in pkts]
    seg_o, off_o, ln_o, st_o = oracle_run(ot, pkts, False)
    arr = pkts
    out = snd.transform(arr)
    assert out is arr and arr[7] is None and arr[33] is None
    for i, p in enumerate(arr):
        if p is None:
            continue
        assert st_o[i] == 0
        L0 = before[i][2]
        assert p.length == L0 + 10 == ln_o[i]
        assert p.data() == seg_o[off_o[i]:off_o[i] + ln_o[i]].tobytes()
        spare = len(bufs[i]) - before[i][1] - L0
        if spare >= 10:  # append in place: same buffer object, same offset
            assert p.buffer is bufs[i] and p.offset == before[i][1]
        else:            # append reallocates: exact-size buffer at offset 0
            assert p.buffer is not bufs[i] and p.offset == 0 and len(p.buffer) == L0 + 10
    # unprotect: tamper a few, replay one; drops become None, the objects shrink
    prot = [None if p is None else RawPacket(bytes(p.buffer), p.offset, p.length) for p in arr]
    prot[10].buffer[prot[10].offset + 30] ^= 1
    prot[20].buffer[prot[20].offset + prot[20].length - 1] ^= 0x80  # tag byte
    prot.append(RawPacket(bytes(prot[5].buffer), prot[5].offset, prot[5].length))  # replay
    keep = list(prot)
    seg_r, off_r, ln_r, st_r = oracle_run(otr, copy.deepcopy(prot), True)
    out = rcv.reverseTransform(prot)
    assert out is prot
    for i, p in enumerate(out):
        if keep[i] is None:
            assert p is None
            continue
        obj = keep[i]
        assert obj.length == ln_r[i]
        assert obj.data() == seg_r[off_r[i]:off_r[i] + ln_r[i]].tobytes()
        if st_r[i] == N.STATUS_OK:
            assert p is obj
        else:
            assert p is None
    assert st_r[10] == st_r[20] == N.STATUS_DROP_AUTH and st_r[-1] == N.STATUS_DROP_REPLAY


def test_srtcp_grow_always_reallocates(eng):
    (k, s), = synth.keys(501, 1)
    t = SRTCPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng))
    of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
    ot = O.Transformer(O.KIND_RTCP, of, of)
    cb = synth.rtcp_bundle(12, 3, seed=502)
    pkts = [RawPacket(cb.seg[cb.off[i]:cb.off[i] + cb.length[i]].tobytes() + bytes(100), 0,
                      int(cb.length[i])) for i in range(cb.n)]
    bufs = [p.buffer for p in pkts]
    seg_o, off_o, ln_o, st_o = oracle_run(ot, pkts, False)
    t.transform(pkts)
    for i, p in enumerate(pkts):
        L0 = int(cb.length[i])
        assert p.buffer is not bufs[i] and p.offset == 0 and len(p.buffer) == L0 + 4 + 10
        assert p.length == L0 + 14 == ln_o[i]
        assert p.data() == seg_o[off_o[i]:off_o[i] + ln_o[i]].tobytes()


def _valid_srtp(k, s, seq, ssrc, hdr: bytes, body_len: int, buflen: int):
    """An SRTP packet with a correct _80 tag (ROC 0) over header + body; the
    RawPacket buffer is exactly `buflen` bytes."""
    enc, auth, salt = O.derive_keys(k, s, False)
    p = bytearray(hdr + bytes(RNG.integers(0, 256, body_len, dtype=np.uint8)))
    p[2:4] = seq.to_bytes(2, "big")
    p[8:12] = ssrc.to_bytes(4, "big")
    tag = O.hmac_sha1(auth, bytes(p) + (0).to_bytes(4, "big"))[:10]
    full = bytes(p) + tag
    assert buflen >= len(full)
    return RawPacket(full + bytes(buflen - len(full)), 0, len(full))


def test_throw_midway_aborts_rest_and_keeps_shrink(eng):
    """reverseTransform: packet 2 authenticates, is shrunk, then its header
    length (CC=15 + X, the extension length read past the buffer) throws in
    processPacketAESCM: packets 0-1 are transformed, packet 2 keeps the shrink
    and stays in the array, packets 3.. are untouched, the exception is raised,
    and the transformer counts it."""
    (k, s), = synth.keys(503, 1)
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *P80, engine=eng))
    ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
    otr = O.Transformer(O.KIND_RTP, ofr, ofr)
    hdr = bytes([0x80, 96]) + bytes(10)
    bad_hdr = bytes([0x9F, 96]) + bytes(10)
    pkts = [_valid_srtp(k, s, 10, 77, hdr, 100, 110 + 16),
            _valid_srtp(k, s, 11, 77, hdr, 50, 60 + 16),
            _valid_srtp(k, s, 12, 77, bad_hdr, 18, 40),  # 40-B buffer: getHeaderLength reads byte 74
            _valid_srtp(k, s, 13, 77, hdr, 80, 90 + 16),
            _valid_srtp(k, s, 14, 78, hdr, 80, 90 + 16)]
    before = [snapshot(p) for p in pkts]
    objs = list(pkts)
    seg_r, off_r, ln_r, st_r = oracle_run(otr, copy.deepcopy(pkts), True)
    assert st_r.tolist() == [0, 0, N.STATUS_ERR_MALFORMED, N.STATUS_NOT_PROCESSED,
                             N.STATUS_NOT_PROCESSED]
    with pytest.raises(SRTPTransformException):
        rcv.reverseTransform(pkts)
    assert [p is o for p, o in zip(pkts, objs)] == [True] * 5
    for i in (0, 1):
        assert pkts[i].length == ln_r[i] == before[i][2] - 10
        assert pkts[i].data() == seg_r[off_r[i]:off_r[i] + ln_r[i]].tobytes()
    assert pkts[2].length == before[2][2] - 10 == ln_r[2]  # shrunk before the throw
    for i in (3, 4):
        assert snapshot(pkts[i]) == before[i]
    assert rcv.exceptionsInReverseTransform == 1
    # the context of ssrc 77 saw packets 10, 11 (and 12's replay-window entry
    # is not set: the reference threw before update)
    st = eng.context_state(rcv, 77)
    assert st is not None and st["s_l"] == 11 and eng.context_state(rcv, 78) is None


def test_transform_bundle_many_transformers_and_predicate(eng):
    """transform_bundle over three transformers (one with a throwing packet)
    equals each transformer's own transform(); a predicate filters packets."""
    keys = synth.keys(504, 3)
    ts, ots = [], []
    for k, s in keys:
        ts.append(SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng)))
        of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
        ots.append(O.Transformer(O.KIND_RTP, of, of))
    pkts, owner = [], []
    for i in range(45):
        j = i % 3
        b0 = 0x8F if (j == 1 and i == 22) else 0x80  # transformer 1 throws at packet 22
        # (CC=15: a 72-B header on a 60-B packet, payload length -12: SRTPCipherCTR throws)
        pkts.append(rtp(500 + i, 0x2000 + j, 60 if b0 == 0x8F else int(RNG.integers(80, 400)),
                        b0=b0, room=16))
        owner.append(ts[j])
    ref = copy.deepcopy(pkts)
    before = [snapshot(p) for p in pkts]
    seg_o, off_o, ln_o, cap_o, fl_o = pack(ref)
    st_o = O.process([ots[ts.index(t)] for t in owner], False, seg_o, off_o, ln_o, cap_o, fl_o)
    with pytest.raises(SRTPTransformException):
        transform_bundle(owner, pkts, False)
    for i, p in enumerate(pkts):
        if st_o[i] == N.STATUS_NOT_PROCESSED:
            assert snapshot(p) == before[i]
        elif st_o[i] == 0:
            assert p.data() == seg_o[off_o[i]:off_o[i] + ln_o[i]].tobytes()
    assert (st_o == N.STATUS_NOT_PROCESSED).sum() == len([i for i in range(23, 45) if i % 3 == 1])
    # predicate: odd sequence numbers only; the others pass through untouched
    (k, s), = synth.keys(505, 1)
    t = SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng),
                        packetPredicate=lambda p: p.getSequenceNumber() % 2 == 1)
    pp = [rtp(900 + i, 0x3000, 200, room=16) for i in range(10)]
    raw = [snapshot(p) for p in pp]
    t.transform(pp)
    for i, p in enumerate(pp):
        if (900 + i) % 2 == 1:
            assert p.length == 210
        else:
            assert snapshot(p) == raw[i]


def test_c_marshalling_raw_abi(eng):
    """srtp_rawpacket_transform called directly (as the JNI shim does), with
    null elements, a predicate-skipped element, DISCARD / SILENCE flags, a
    packet past its buffer (RawPacket.isInvalid), and an element whose
    protect needs a new buffer: statuses, need_len, lengths and bytes against
    the oracle run of the same RawPacket[]."""
    import ctypes as C
    (k, s), = synth.keys(506, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=eng))
    of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
    ot = O.Transformer(O.KIND_RTP, of, of)
    pkts = [rtp(40 + i, 0x5000 + i % 3, int(RNG.integers(40, 500)), room=(0 if i % 4 == 0 else 20),
                offset=int(RNG.integers(0, 9))) for i in range(24)]
    pkts[3] = None
    pkts[9] = RawPacket(bytes(pkts[9].buffer), pkts[9].offset, len(pkts[9].buffer) + 5)  # invalid
    skip = np.zeros(len(pkts), np.uint32)
    skip[11] = N.PKT_FLAG_SKIP
    pkts[14].flags = N.PKT_FLAG_DISCARD
    ref = copy.deepcopy(pkts)
    seg_o, off_o, ln_o, cap_o, fl_o = pack([None if skip[i] else p for i, p in enumerate(ref)])
    st_o = O.process(ot, False, seg_o, off_o, ln_o, cap_o, fl_o)
    n = len(pkts)
    L = N.lib()
    bufs = (C.c_void_p * n)()
    views = []
    buf_len = np.zeros(n, np.uint32)
    offset = np.zeros(n, np.uint32)
    length = np.zeros(n, np.uint32)
    flags = skip.copy()
    for i, p in enumerate(pkts):
        if p is None:
            continue
        v = (C.c_char * len(p.buffer)).from_buffer(p.buffer)
        views.append(v)
        bufs[i] = C.addressof(v)
        buf_len[i], offset[i], length[i] = len(p.buffer), p.offset, p.length
        flags[i] |= p.flags
    status = np.zeros(n, np.int32)
    need = np.zeros(n, np.uint32)
    thrown = C.c_int32(7)
    before = [snapshot(p) for p in pkts]
    rc = L.srtp_rawpacket_transform(_rp_batch(eng), 0, None, snd.tid, bufs, buf_len.ctypes.data,
                                    offset.ctypes.data, length.ctypes.data, flags.ctypes.data,
                                    status.ctypes.data, need.ctypes.data, n, C.byref(thrown))
    del views
    assert rc == 0 and thrown.value == -1
    exp = st_o.copy()
    exp[3] = N.STATUS_SKIPPED
    assert status.tolist() == exp.tolist()
    assert status[9] == N.STATUS_DROP_INVALID and status[11] == N.STATUS_SKIPPED
    for i, p in enumerate(pkts):
        if p is None or status[i] == N.STATUS_SKIPPED:
            assert snapshot(p) == before[i]
            continue
        assert length[i] == ln_o[i]
        want = seg_o[off_o[i]:off_o[i] + ln_o[i]].tobytes()
        if need[i]:
            assert need[i] == ln_o[i] and length[i] > buf_len[i] - offset[i]
            data, dl = C.POINTER(C.c_uint8)(), C.c_uint32()
            assert L.srtp_rawpacket_result(_rp_batch(eng), i, C.byref(data), C.byref(dl)) == 0
            assert C.string_at(data, dl.value) == want
            assert bytes(p.buffer) == before[i][0]  # the caller moves it to a new buffer
        elif status[i] == 0:
            assert bytes(p.buffer[p.offset:p.offset + length[i]]) == want
    assert (need > 0).sum() >= 3
