"""The JNI shim (src/native/srtp_mi355x/SrtpMi355x.c), compiled unmodified
against a stub JNI header and driven through a toy JVM (tests/jni_stub/).

The image has no JDK, so the Java classes under src/org/ cannot be compiled
here; the C half of the drop-in can.  tests/jni_stub/libfakejni.so is the shim
plus fakejvm.c, which implements the JNI calls the shim makes over byte[] /
int[] / Object[] and RawPacket objects (RawPacket.java:53-73).  The CPU test
checks that every native method SrtpMi355x.java declares is exported; the GPU
tests call the exported JNI functions exactly as the Java classes do --
dispatcher, factories, transformers, transformOne (GpuTransformerBase's
per-packet path) and transformPackets (its array path) -- and compare every
RawPacket's bytes, length, buffer replacement and the nulled / thrown elements
with the oracle.  The toy JVM also checks that no array region is ever out of
range and that local frames balance.
"""
import ctypes as C
import os
import re
import threading

import numpy as np
import pytest

from libjitsi_amd import profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import opol

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "jni_stub", "libfakejni.so")
JAVA = os.path.join(ROOT, "src", "org", "jitsi", "impl", "neomedia", "transform", "srtp", "mi355x",
                    "SrtpMi355x.java")
PREFIX = "Java_org_jitsi_impl_neomedia_transform_srtp_mi355x_SrtpMi355x_"
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")

vp, i32, i64, u8 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint8


def java_natives():
    src = open(JAVA).read()
    return re.findall(r"static native \w+(?:\[\])? (\w+)\(", src)


def load():
    if not os.path.exists(LIB):
        pytest.skip("tests/jni_stub/libfakejni.so not built (__graft_entry__.build())")
    L = C.CDLL(LIB)
    J = lambda n: getattr(L, PREFIX + n)  # noqa: E731
    L.fj_env.restype = vp
    L.fj_rawpacket_class.restype = vp
    for f, a, r in [("fj_new_bytes", [C.c_char_p, i32], vp), ("fj_new_ints", [vp, i32], vp),
                    ("fj_new_objects", [i32], vp), ("fj_set_element", [vp, i32, vp], None),
                    ("fj_get_element", [vp, i32], vp), ("fj_new_packet", [vp, i32, i32, i32], vp),
                    ("fj_packet_buffer", [vp], vp), ("fj_packet_offset", [vp], i32),
                    ("fj_packet_length", [vp], i32), ("fj_bytes_len", [vp], i32),
                    ("fj_bytes_read", [vp, vp], None), ("fj_exceptions", [], C.c_int),
                    ("fj_frames", [], C.c_int), ("fj_reset", [], None), ("fj_ints_read", [vp, vp], None),
                    ("fj_fail_new_arrays", [C.c_int], None), ("fj_exception_pending", [], C.c_int)]:
        getattr(L, f).argtypes, getattr(L, f).restype = a, r
    sig = {"deviceCount": ([], i32), "dispatchCreate": ([vp, i32, i32], i64), "dispatchDestroy": ([i64], None),
           "factoryCreate": ([i64, u8, vp, vp, vp, vp], i32), "factoryClose": ([i64, i32], i32),
           "transformerCreate": ([i64, i32, i32, i32], i32), "transformerSetFactory": ([i64, i32, i32, u8], i32),
           "transformerClose": ([i64, i32], i32),
           "transformPackets": ([i64, i64, u8, i32, vp, vp], i32), "aggregatorCreate": ([i64, i32, i32, i32], i64),
           "aggregatorDestroy": ([i64], None), "transformOne": ([i64, u8, i32, vp], i32),
           "queueCreate": ([i64, i32], i64), "queueDestroy": ([i64], None),
           "queueSubmit": ([i64, u8, i32, vp, u8, i64], i32), "queueReap": ([i64, vp, vp, u8], i32)}
    for n, (a, r) in sig.items():
        J(n).argtypes, J(n).restype = [vp, vp] + a, r
    return L, J


def test_shim_exports_every_java_native():
    """Every `static native` method of SrtpMi355x.java has its JNI symbol."""
    L, J = load()
    names = java_natives()
    assert len(names) >= 14
    for n in names:
        J(n)  # raises AttributeError when missing
    # no GPU needed: without one the device count is 0, and Java refuses to start
    env, cls = L.fj_env(), L.fj_rawpacket_class()
    assert J("deviceCount")(env, cls) >= 0


class Jvm:
    """The Java side of the shim, as SrtpMi355x / GpuTransformerBase call it."""

    def __init__(self, n_shards=2):
        self.L, self.J = load()
        self.env, self.cls = self.L.fj_env(), self.L.fj_rawpacket_class()
        devs = np.zeros(n_shards, np.int32)
        self.d = self.J("dispatchCreate")(self.env, self.cls, self.L.fj_new_ints(devs.ctypes.data, n_shards),
                                          1, 1 << 14)
        assert self.d
        self.agg = self.J("aggregatorCreate")(self.env, self.cls, self.d, 0, 0, 0)  # the defaults
        assert self.agg

    def close(self):
        self.J("aggregatorDestroy")(self.env, self.cls, self.agg)
        self.J("dispatchDestroy")(self.env, self.cls, self.d)
        assert self.L.fj_exceptions() == 0, "the shim read or wrote an array region out of range"
        assert self.L.fj_frames() == 0, "unbalanced local frames"
        self.L.fj_reset()

    def ints(self, a):
        a = np.ascontiguousarray(a, np.int32)
        return self.L.fj_new_ints(a.ctypes.data, len(a))

    def factory(self, sender, key, salt, pol):
        p = self.ints([pol.encType, pol.encKeyLength, pol.authType, pol.authKeyLength, pol.authTagLength,
                       pol.saltKeyLength])
        f = self.J("factoryCreate")(self.env, self.cls, self.d, int(sender), self.L.fj_new_bytes(key, len(key)),
                                    self.L.fj_new_bytes(salt, len(salt)), p, p)
        assert f >= 0
        return f

    def transformer(self, kind, fwd, rev):
        t = self.J("transformerCreate")(self.env, self.cls, self.d, kind, fwd, rev)
        assert t >= 0
        return t

    def packet(self, data, offset=0, extra=0):
        buf = b"\xee" * offset + data + b"\x00" * extra
        return self.L.fj_new_packet(self.L.fj_new_bytes(buf, len(buf)), offset, len(data), 0)

    def packet_bytes(self, p):
        b = self.L.fj_packet_buffer(p)
        raw = (C.c_uint8 * self.L.fj_bytes_len(b))()
        self.L.fj_bytes_read(b, raw)
        o, n = self.L.fj_packet_offset(p), self.L.fj_packet_length(p)
        return bytes(raw[o:o + n]), b

    def one(self, reverse, tid, p):
        return self.J("transformOne")(self.env, self.cls, self.agg, int(reverse), tid, p)

    def array(self, reverse, tid, pkts, skip=None):
        arr = self.L.fj_new_objects(len(pkts))
        for i, p in enumerate(pkts):
            self.L.fj_set_element(arr, i, p)
        sk = self.ints(skip) if skip is not None else None
        r = self.J("transformPackets")(self.env, self.cls, self.d, self.agg, int(reverse), tid, arr, sk)
        return r, [self.L.fj_get_element(arr, i) for i in range(len(pkts))]


class PacketQueue:
    """GpuPacketQueue.java over the shim's queue entries: a ring of the
    RawPackets in flight by submission number, reaped in submission order."""

    def __init__(self, jvm, max_in_flight):
        self.jvm, self.J, self.env, self.cls = jvm, jvm.J, jvm.env, jvm.cls
        self.q = self.J("queueCreate")(self.env, self.cls, jvm.agg, max_in_flight)
        assert self.q
        self.n = max_in_flight
        self.ring = jvm.L.fj_new_objects(max_in_flight)
        self.status = jvm.ints(np.zeros(min(max_in_flight, 1024), np.int32))
        self.nst = min(max_in_flight, 1024)
        self.pkts = [None] * max_in_flight
        self.submitted = self.reaped = 0

    def submit(self, reverse, tid, p, skip=False):
        """False when the queue is full (GpuPacketQueue.submit)."""
        if self.submitted - self.reaped == self.n:
            return False
        i = self.submitted % self.n
        self.jvm.L.fj_set_element(self.ring, i, p)
        rc = self.J("queueSubmit")(self.env, self.cls, self.q, int(reverse), tid, p, int(skip), self.submitted)
        if rc == N.EAGAIN:
            return False
        assert rc == 0, rc
        self.pkts[i] = p
        self.submitted += 1
        return True

    def reap(self, wait=True):
        """[(packet, status)] in submission order (GpuPacketQueue.reap)."""
        if self.submitted == self.reaped:
            return []
        n = self.J("queueReap")(self.env, self.cls, self.q, self.ring, self.status, int(wait))
        assert n >= 0, n
        st = np.zeros(self.nst, np.int32)
        self.jvm.L.fj_ints_read(self.status, st.ctypes.data)
        out = []
        for k in range(n):
            i = self.reaped % self.n
            out.append((self.pkts[i], int(st[k])))
            self.pkts[i] = None
            self.reaped += 1
        return out

    def close(self):
        self.J("queueDestroy")(self.env, self.cls, self.q)


def oracle_one(ot, reverse, data, extra=0):
    L = len(data)
    avail = L + extra
    cap = min(max(avail, L + 16), 65535) if not reverse else avail
    seg = np.zeros(max((cap + 15) // 16 * 16, 16), np.uint8)
    seg[:L] = np.frombuffer(data, np.uint8)
    ln = np.array([L], np.uint32)
    st = O.process(ot, reverse, seg, np.zeros(1, np.uint32), ln, np.array([cap], np.uint32),
                   np.zeros(1, np.uint32), True)
    return int(st[0]), seg[:int(ln[0])].tobytes()


def rtp(ssrc, seq, n, rng, bad_ext=False):
    b = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    b[0], b[1] = 0x80, 96
    b[2:4] = (seq & 0xFFFF).to_bytes(2, "big")
    b[8:12] = ssrc.to_bytes(4, "big")
    if bad_ext:  # an extension length past the packet: the reference throws
        b[0] |= 0x10
        b[12:16] = b"\xbe\xde\x7f\xff"
    return bytes(b)


@pytest.mark.gpu
def test_jni_per_packet_and_array_paths_vs_oracle():
    jvm = Jvm(n_shards=2)
    try:
        (k, s), = synth.keys(31, 1)
        fs, fr = jvm.factory(True, k, s, P80[0]), jvm.factory(False, k, s, P80[0])
        ts, tr = jvm.transformer(0, fs, fs), jvm.transformer(0, fr, fr)
        ofs = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
        ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
        ots, otr = O.Transformer(O.KIND_RTP, ofs, ofs), O.Transformer(O.KIND_RTP, ofr, ofr)
        rng = np.random.default_rng(7)
        # per packet (transformOne): a new buffer where append reallocates, in
        # place where there is room (extra bytes behind the packet, an offset)
        prot = []
        for q in range(8):
            data = rtp(0x1234 + (q & 1), 500 + q, 200 + 40 * q, rng)
            extra, off = (16, 3) if q % 3 == 0 else (0, 0)
            p = jvm.packet(data, off, extra)
            b0 = jvm.L.fj_packet_buffer(p)
            st = jvm.one(False, ts, p)
            ost, ob = oracle_one(ots, False, data, extra)
            got, b = jvm.packet_bytes(p)
            assert st == ost == N.STATUS_OK and got == ob
            assert (b == b0) == (extra >= 10)  # the reference's append: in place only with room
            prot.append(got)
        # the array path (transformPackets): a replay, a forgery and a throw in
        # mid-array; later packets of the transformer are not processed
        bad = bytearray(prot[5])
        bad[-1] ^= 1
        inputs = [prot[0], prot[1], prot[0], bytes(bad), prot[2], rtp(0x1234, 9, 40, rng, bad_ext=True),
                  prot[3], prot[4]]
        pkts = [jvm.packet(x) for x in inputs]
        r, out = jvm.array(True, tr, pkts)
        seg = np.zeros(sum((len(x) + 15) // 16 * 16 for x in inputs), np.uint8)
        off = np.zeros(len(inputs), np.uint32)
        pos = 0
        for i, x in enumerate(inputs):
            off[i] = pos
            seg[pos:pos + len(x)] = np.frombuffer(x, np.uint8)
            pos += (len(x) + 15) // 16 * 16
        ln = np.array([len(x) for x in inputs], np.uint32)
        st_o = O.process(otr, True, seg, off, ln, ln.copy(), None, True)
        thrown = [i for i, s in enumerate(st_o) if s == N.STATUS_ERR_MALFORMED]
        assert r == (thrown[0] + 1 if thrown else 0)
        for i in range(len(inputs)):
            if st_o[i] in (N.STATUS_OK, N.STATUS_ERR_MALFORMED):
                assert out[i] == pkts[i]
                got, _ = jvm.packet_bytes(pkts[i])
                assert got == seg[off[i]:off[i] + ln[i]].tobytes(), i
            elif st_o[i] == N.STATUS_NOT_PROCESSED:
                assert out[i] == pkts[i]
                got, _ = jvm.packet_bytes(pkts[i])
                assert got == inputs[i]  # untouched
            else:
                assert out[i] is None, (i, N.STATUS_NAMES[st_o[i]])  # the reference returned null
    finally:
        jvm.close()


@pytest.mark.gpu
def test_jni_per_packet_from_many_threads_vs_oracle():
    """16 "JVM threads" call transformOne at once, each on its own SSRCs."""
    jvm = Jvm(n_shards=3)
    try:
        keys = synth.keys(41, 4)
        tids, otids = [], []
        for k, s in keys:
            f = jvm.factory(True, k, s, P80[0])
            tids.append(jvm.transformer(0, f, f))
            of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
            otids.append(O.Transformer(O.KIND_RTP, of, of))
        scripts = []
        for t in range(16):
            rng = np.random.default_rng(100 + t)
            scripts.append([(t % 4, rtp(0x9000 + t, 40 + q, int(rng.integers(60, 1300)), rng)) for q in range(20)])
        results = [None] * 16
        errs = []

        def work(t):
            try:
                out = []
                for ti, data in scripts[t]:
                    p = jvm.packet(data)
                    st = jvm.one(False, tids[ti], p)
                    out.append((st, jvm.packet_bytes(p)[0]))
                results[t] = out
            except Exception as ex:  # noqa: BLE001
                errs.append(ex)
        th = [threading.Thread(target=work, args=(t,)) for t in range(16)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs
        for t in range(16):
            for (ti, data), (st, got) in zip(scripts[t], results[t]):
                ost, ob = oracle_one(otids[ti], False, data)
                assert st == ost and got == ob
    finally:
        jvm.close()


def rtp_of(k, s, q, n, rng, bad_ext=False):
    return rtp(0x50000000 + 8 * k + s, 1000 + 97 * k + q, n, rng, bad_ext)


class FjJob(C.Structure):
    """struct fj_job (tests/jni_stub/fakejvm.c): one "JVM thread" driving GpuPacketQueue."""
    _fields_ = [("agg", C.c_int64), ("reverse", C.c_uint8), ("depth", C.c_int32), ("n", C.c_int32),
                ("tids", C.c_void_p), ("pkts", C.c_void_p), ("status", C.c_void_p),
                ("max_in_flight", C.c_int32), ("rc", C.c_int32)]


@pytest.mark.gpu
def test_jni_queue_64_threads_in_flight_vs_oracle():
    """GpuPacketQueue: 64 "JVM threads" (a connector send thread each; native
    threads of the stand-in JVM running GpuPacketQueue's loop over the shim's
    queueSubmit / queueReap, fakejvm.c fj_drive), 50 sender and 50 receiver
    transformers, each thread with a 64-packet queue and >= 32 packets in
    flight.  Protect with throws (an extension header past the packet) in
    mid-stream, then unprotect of the results with replays and forgeries;
    every RawPacket -- status, bytes, length, and the new buffer where
    RawPacket.append reallocates -- against the oracle replaying each thread's
    packets as 1-element arrays in its submission order (each thread owns its
    SSRCs, so that is each context's order)."""
    T, NT, PER, DEPTH = 64, 50, 96, 64
    jvm = Jvm(n_shards=2)
    try:
        jvm.L.fj_drive_queues.argtypes = [C.POINTER(FjJob), C.c_int]
        keys = synth.keys(77, NT)
        ts, tr, ots, otr = [], [], [], []
        for k, s in keys:
            fs, fr = jvm.factory(True, k, s, P80[0]), jvm.factory(False, k, s, P80[0])
            ts.append(jvm.transformer(0, fs, fs))
            tr.append(jvm.transformer(0, fr, fr))
            ofs = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
            ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
            ots.append(O.Transformer(O.KIND_RTP, ofs, ofs))
            otr.append(O.Transformer(O.KIND_RTP, ofr, ofr))
        # per thread: (transformer index, data, buffer extra, offset)
        scripts = []
        for k in range(T):
            rng = np.random.default_rng(500 + k)
            sc = []
            for q in range(PER):
                s = q % 3
                bad = q == 40 and k % 4 == 0
                data = rtp_of(k, s, q // 3, int(rng.integers(60, 1300)), rng, bad_ext=bad)
                extra, off = [(0, 0), (16, 5), (3, 0)][q % 3]
                sc.append(((3 * k + s) % NT, data, extra, off))
            scripts.append(sc)

        def run_all(reverse, all_items):
            """fj_drive on T native threads; per thread [(status, bytes, same buffer)]."""
            keep = []
            jobs = (FjJob * T)()
            for k in range(T):
                items = all_items[k]
                pk = [jvm.packet(d, off, extra) for _, d, extra, off in items]
                b0 = [jvm.L.fj_packet_buffer(p) for p in pk]
                tids = np.array([(tr if reverse else ts)[ti] for ti, _, _, _ in items], np.int32)
                parr = (C.c_void_p * len(pk))(*pk)
                st = np.full(len(pk), -100, np.int32)
                keep.append((pk, b0, tids, parr, st))
                jobs[k] = FjJob(jvm.agg, int(reverse), DEPTH, len(pk), tids.ctypes.data, C.cast(parr, C.c_void_p),
                                st.ctypes.data, 0, 0)
            assert jvm.L.fj_drive_queues(jobs, T) == 0
            out = []
            for k in range(T):
                assert jobs[k].rc == 0, (k, jobs[k].rc)
                pk, b0, _, _, st = keep[k]
                out.append([(int(x), jvm.packet_bytes(p)[0], jvm.L.fj_packet_buffer(p) == b)
                            for x, p, b in zip(st, pk, b0)])
            return out, sorted(jobs[k].max_in_flight for k in range(T))

        results, in_flight = run_all(False, scripts)
        print("max packets in flight per thread (protect):", in_flight)
        assert in_flight[0] >= 32
        seen = set()
        protected = []
        for k in range(T):
            pr = []
            for (ti, data, extra, off), (st, got, same_buf) in zip(scripts[k], results[k]):
                ost, ob = oracle_one(ots[ti], False, data, extra)
                assert st == ost and got == ob, (k, N.STATUS_NAMES[st], N.STATUS_NAMES[ost])
                if ost == N.STATUS_OK:
                    assert same_buf == (extra >= 10)  # append: in place only with room
                    pr.append((ti, got))
                seen.add(st)
            protected.append(pr)
        assert N.STATUS_ERR_MALFORMED in seen
        # unprotect: the thread's protected packets with a replay and a forgery
        un = []
        for k in range(T):
            items = [(ti, d, 0, 0) for ti, d in protected[k]]
            bad = bytearray(items[12][1])
            bad[-3] ^= 0x40
            items.insert(9, (items[12][0], bytes(bad), 0, 0))  # forgery of a packet yet to come
            items.insert(15, items[4])                           # exact replay
            un.append(items)
        results, in_flight = run_all(True, un)
        print("max packets in flight per thread (unprotect):", in_flight)
        assert in_flight[0] >= 32
        seen = set()
        for k in range(T):
            for (ti, data, extra, off), (st, got, _) in zip(un[k], results[k]):
                ost, ob = oracle_one(otr[ti], True, data, extra)
                assert st == ost and got == ob, (k, N.STATUS_NAMES[st], N.STATUS_NAMES[ost])
                seen.add(st)
        assert {N.STATUS_OK, N.STATUS_DROP_REPLAY, N.STATUS_DROP_AUTH} <= seen
    finally:
        jvm.close()


@pytest.mark.gpu
def test_jni_small_arrays_share_bundles_vs_oracle():
    """transformPackets of arrays that cannot throw (replays, forgeries, a
    predicate-skipped element and a packet longer than its buffer, but no
    malformed header) from 16 threads at once: they run through the thread's
    queue on the aggregator's lanes; every element against the oracle."""
    T, NT = 16, 8
    jvm = Jvm(n_shards=2)
    try:
        keys = synth.keys(88, NT)
        ts, tr, ots, otr = [], [], [], []
        for k, s in keys:
            fs, fr = jvm.factory(True, k, s, P80[0]), jvm.factory(False, k, s, P80[0])
            ts.append(jvm.transformer(0, fs, fs))
            tr.append(jvm.transformer(0, fr, fr))
            ofs = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
            ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
            ots.append(O.Transformer(O.KIND_RTP, ofs, ofs))
            otr.append(O.Transformer(O.KIND_RTP, ofr, ofr))
        res = [None] * T
        errs = []

        def work(k):
            try:
                rng = np.random.default_rng(900 + k)
                ti = k % NT
                out = []
                for rnd in range(6):
                    datas = [rtp_of(k, q % 2, 8 * rnd + q, int(rng.integers(60, 1300)), rng) for q in range(8)]
                    pk = [jvm.packet(d, 0, 16 if q % 2 else 0) for q, d in enumerate(datas)]
                    r, o = jvm.array(False, ts[ti], pk)
                    prot = [(r, [(x is not None, jvm.packet_bytes(p)[0]) for x, p in zip(o, pk)])]
                    got = [g for _, g in prot[0][1]]
                    ins = list(got)
                    ins[3] = ins[1]                      # replay
                    f = bytearray(ins[5])
                    f[20] ^= 1
                    ins[5] = bytes(f)                    # forgery
                    pk2 = [jvm.packet(d) for d in ins]
                    skip = np.zeros(8, np.int32)
                    skip[6] = 1                          # the packet predicate said no
                    long_p = jvm.L.fj_new_packet(jvm.L.fj_new_bytes(ins[7], len(ins[7])), 0, len(ins[7]) + 5, 0)
                    pk2[7] = long_p                      # length past its buffer: RawPacket.isInvalid
                    r2, o2 = jvm.array(True, tr[ti], pk2, skip)
                    out.append((datas, r, prot, ins, r2, [(x is not None, jvm.packet_bytes(p)[0]
                                                           if q != 7 else None) for q, (x, p) in enumerate(zip(o2, pk2))]))
                res[k] = out
            except Exception as ex:  # noqa: BLE001
                errs.append(ex)

        th = [threading.Thread(target=work, args=(k,)) for k in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errs, errs[:3]
        for k in range(T):
            ti = k % NT
            for datas, r, prot, ins, r2, un in res[k]:
                assert r == 0
                for q, (d, (kept, got)) in enumerate(zip(datas, prot[0][1])):
                    ost, ob = oracle_one(ots[ti], False, d, 16 if q % 2 else 0)
                    assert kept == (ost == N.STATUS_OK) and got == ob
                assert r2 == 0
                for q, (d, (kept, got)) in enumerate(zip(ins, un)):
                    if q == 6:
                        assert kept and got == d        # skipped: untouched
                        continue
                    if q == 7:
                        assert not kept                 # DROP_INVALID: null
                        continue
                    ost, ob = oracle_one(otr[ti], True, d)
                    assert kept == (ost == N.STATUS_OK) and got == ob, (q, N.STATUS_NAMES[ost])
    finally:
        jvm.close()


@pytest.mark.gpu
def test_jni_main_thread_array_then_close():
    """An array that cannot throw, sent on the thread that then closes the
    aggregator (the thread's queue on the aggregator made
    aggregatorDestroy wait forever): the queue lives for the call only."""
    jvm = Jvm(n_shards=2)
    closed = threading.Event()
    try:
        (k, s), = synth.keys(61, 1)
        f = jvm.factory(True, k, s, P80[0])
        t = jvm.transformer(0, f, f)
        of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
        ot = O.Transformer(O.KIND_RTP, of, of)
        rng = np.random.default_rng(61)
        datas = [rtp(0x6100, 10 + q, 300 + 50 * q, rng) for q in range(6)]
        pk = [jvm.packet(d, 0, 16) for d in datas]
        r, out = jvm.array(False, t, pk)
        assert r == 0
        for d, p in zip(datas, pk):
            ost, ob = oracle_one(ot, False, d, 16)
            assert ost == N.STATUS_OK and jvm.packet_bytes(p)[0] == ob
    finally:
        th = threading.Thread(target=lambda: (jvm.close(), closed.set()), daemon=True)
        th.start()
        th.join(60)
    assert closed.is_set(), "aggregatorDestroy did not return"


@pytest.mark.gpu
def test_jni_queue_reap_out_of_memory_keeps_order():
    """queueReap when the JVM cannot allocate a packet's new buffer (protect
    of packets whose buffers have no room for the tag: RawPacket.append
    reallocates): the reaped count still comes back, that packet's status is
    SRTP_STATUS_ERR_INTERNAL (handed on as null), the OutOfMemoryError is
    cleared, and the packets after it -- in this reap and the next -- are
    written back in submission order against the oracle."""
    jvm = Jvm(n_shards=1)
    try:
        (k, s), = synth.keys(62, 1)
        f = jvm.factory(True, k, s, P80[0])
        t = jvm.transformer(0, f, f)
        of = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
        ot = O.Transformer(O.KIND_RTP, of, of)
        rng = np.random.default_rng(62)
        q = PacketQueue(jvm, 16)
        datas = [rtp(0x6200, 20 + i, 200 + 30 * i, rng) for i in range(12)]
        pk = [jvm.packet(d) for d in datas]  # no room: each result needs a new buffer
        got = []
        for p in pk[:6]:
            assert q.submit(False, t, p)
        jvm.L.fj_fail_new_arrays(1)
        while len(got) < 6:
            got += q.reap(True)
        assert jvm.L.fj_exception_pending() == 0
        for p in pk[6:]:
            assert q.submit(False, t, p)
        while len(got) < 12:
            got += q.reap(True)
        q.close()
        sts = [st for _, st in got]
        assert [p for p, _ in got] == pk
        assert sts[0] == N.STATUS_ERR_INTERNAL and sts.count(N.STATUS_ERR_INTERNAL) == 1
        for i, (d, p) in enumerate(zip(datas, pk)):
            ost, ob = oracle_one(ot, False, d)
            if i == 0:
                continue  # its result could not be written back: the Java side drops it
            assert sts[i] == ost == N.STATUS_OK and jvm.packet_bytes(p)[0] == ob, i
    finally:
        jvm.L.fj_fail_new_arrays(0)
        jvm.close()


class FjLoop(C.Structure):
    """struct fj_loop (tests/jni_stub/fakejvm.c): one connector thread running
    GpuConnectorLoops.Send (reverse 0) or .Receive (reverse 1)."""
    _fields_ = [("agg", C.c_int64), ("reverse", C.c_uint8), ("tid", C.c_int32), ("n_in", C.c_int32),
                ("depth", C.c_int32), ("inp", C.c_void_p), ("bursts", C.c_void_p), ("n_bursts", C.c_int32),
                ("out", C.c_void_p), ("n_out", C.c_int32), ("n_dropped", C.c_int32),
                ("max_in_flight", C.c_int32), ("polls_empty", C.c_int32), ("rc", C.c_int32)]


@pytest.mark.gpu
def test_jni_connector_loops_vs_oracle():
    """GpuConnectorLoops.Send and .Receive (src/org/.../mi355x/GpuConnectorLoops.java)
    as 8 send threads and 8 receive threads of the stand-in JVM
    (fakejvm.c fj_loop_run): input in bursts of 1-40 datagrams, up to 256
    packets in flight per thread.  Each send thread's protected packets go out
    in the order they were queued, each as the oracle's; the receive threads
    get them with replays and forgeries mixed in and hand on, in arrival
    order, exactly the packets the oracle accepts, with its bytes."""
    T, PER = 8, 300
    jvm = Jvm(n_shards=2)
    L = jvm.L
    L.fj_run_loops.argtypes, L.fj_run_loops.restype = [C.c_void_p, C.c_int], C.c_int
    try:
        keys = synth.keys(70, T)
        snd, rcv, osnd, orcv = [], [], [], []
        for k, s in keys:
            fs, fr = jvm.factory(True, k, s, P80[0]), jvm.factory(False, k, s, P80[0])
            snd.append(jvm.transformer(0, fs, fs))
            rcv.append(jvm.transformer(0, fr, fr))
            ofs = O.Factory(True, k, s, opol(P80[0]), opol(P80[1]))
            ofr = O.Factory(False, k, s, opol(P80[0]), opol(P80[1]))
            osnd.append(O.Transformer(O.KIND_RTP, ofs, ofs))
            orcv.append(O.Transformer(O.KIND_RTP, ofr, ofr))

        def run(reverse, tids, inputs, seed):
            rng = np.random.default_rng(seed)
            keep, loops = [], (FjLoop * T)()
            for t in range(T):
                arr = (C.c_void_p * len(inputs[t]))(*[L.fj_new_bytes(d, len(d)) for d in inputs[t]])
                bl, left = [], len(inputs[t])
                while left:
                    bl.append(min(left, int(rng.integers(1, 41))))
                    left -= bl[-1]
                bursts = np.array(bl, np.int32)
                out = (C.c_void_p * len(inputs[t]))()
                keep += [arr, bursts, out]
                loops[t] = FjLoop(jvm.agg, int(reverse), tids[t], len(inputs[t]), 256, C.cast(arr, C.c_void_p),
                                  bursts.ctypes.data, len(bl), C.cast(out, C.c_void_p), 0, 0, 0, 0, 0)
            assert L.fj_run_loops(loops, T) == 0
            res = []
            for t in range(T):
                lp = loops[t]
                assert lp.rc == 0, (t, lp.rc)
                outs = C.cast(lp.out, C.POINTER(C.c_void_p))
                res.append(([jvm.packet_bytes(outs[i])[0] for i in range(lp.n_out)], lp))
            return res

        rng = np.random.default_rng(71)
        sent = [[rtp(0x7000 + 4 * t + (q % 3), 3000 + 11 * t + q, int(rng.integers(60, 1300)), rng)
                 for q in range(PER)] for t in range(T)]
        out_s = run(False, snd, sent, 72)
        for t in range(T):
            got, lp = out_s[t]
            assert lp.n_dropped == 0 and len(got) == PER
            assert lp.max_in_flight >= 32
            for d, g in zip(sent[t], got):
                ost, ob = oracle_one(osnd[t], False, d)
                assert ost == N.STATUS_OK and g == ob
        # the receivers: the wire order, with replays and forgeries
        wire = []
        for t in range(T):
            w = list(out_s[t][0])
            for q in range(0, PER, 37):
                w.insert(q + 5, w[q])                          # a replay
                f = bytearray(w[q + 2])
                f[-3] ^= 0x40
                w.insert(q + 9, bytes(f))                      # a forgery
            wire.append(w)
        out_r = run(True, rcv, wire, 73)
        for t in range(T):
            got, lp = out_r[t]
            want = []
            for d in wire[t]:
                ost, ob = oracle_one(orcv[t], True, d)
                if ost == N.STATUS_OK:
                    want.append(ob)
            assert lp.n_dropped == len(wire[t]) - len(want) > 0
            assert got == want
    finally:
        jvm.close()
