"""Host-side mirror of libjitsi's SRTP transformer API over the MI355X engine.

Same class and method names, argument meaning and error behaviour as the
reference (paths relative to src/org/jitsi/impl/neomedia/):

* ``SRTPPolicy``            transform/srtp/SRTPPolicy.java:24-120
* ``SRTPContextFactory``    transform/srtp/SRTPContextFactory.java:24-108
* ``RawPacket``             RawPacket.java (buffer/offset/length/flags + accessors)
* ``PacketTransformer``     transform/PacketTransformer.java:28-53
* ``SRTPTransformer``       transform/srtp/SRTPTransformer.java:53-219
* ``SRTCPTransformer``      transform/srtp/SRTCPTransformer.java:30-207

``transform(pkts)`` / ``reverseTransform(pkts)`` follow
SinglePacketTransformer.java:121-216: packets are processed in array order,
``None`` elements are skipped, each element is replaced by the transformed
packet or ``None`` (drop), and a packet on which the reference would throw
raises ``SRTPTransformException`` after the earlier packets were transformed
(the remaining elements of the array are left untouched).

All per-packet work runs on the GPU (libsrtp_mi355x.so); this module only
packs RawPackets into one bundle and unpacks the results.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N


class SRTPTransformException(RuntimeError):
    """What SinglePacketTransformer rethrows (RuntimeException)."""


class SRTPPolicy:
    NULL_ENCRYPTION = 0
    AESCM_ENCRYPTION = 1
    AESF8_ENCRYPTION = 2
    TWOFISH_ENCRYPTION = 3
    TWOFISHF8_ENCRYPTION = 4
    NULL_AUTHENTICATION = 0
    HMACSHA1_AUTHENTICATION = 1
    SKEIN_AUTHENTICATION = 2

    def __init__(self, encType: int, encKeyLength: int, authType: int, authKeyLength: int,
                 authTagLength: int, saltKeyLength: int):
        self.encType = encType
        self.encKeyLength = encKeyLength
        self.authType = authType
        self.authKeyLength = authKeyLength
        self.authTagLength = authTagLength
        self.saltKeyLength = saltKeyLength

    def getEncType(self): return self.encType
    def getEncKeyLength(self): return self.encKeyLength
    def getAuthType(self): return self.authType
    def getAuthKeyLength(self): return self.authKeyLength
    def getAuthTagLength(self): return self.authTagLength
    def getSaltKeyLength(self): return self.saltKeyLength

    def _c(self) -> N.Policy:
        return N.Policy(self.encType, self.encKeyLength, self.authType, self.authKeyLength,
                        self.authTagLength, self.saltKeyLength)

    def __repr__(self):
        return (f"SRTPPolicy(enc={self.encType}/{self.encKeyLength}, auth={self.authType}/"
                f"{self.authKeyLength}, tag={self.authTagLength}, salt={self.saltKeyLength})")


class SRTPPipeline:
    """Pinned-host bundle pipeline over one engine (srtp_pipeline_*, C ABI).

    ``depth`` slots of pinned host memory; a caller packs a bundle straight
    into a slot's arrays (``slot(i)``: numpy views ``seg``, ``off``, ``len``,
    ``cap``, ``flags``, ``tids``, ``status``), ``submit``s it (H2D on a copy
    stream, the engine's kernels, D2H on a second copy stream) and ``wait``s
    for the results in the same arrays.  Bundles run in submission order;
    while slot i's kernels run, slot j's copies proceed.  This is the bundle
    former the reference lacks (its I/O layer hands 1-element RawPacket[]
    arrays to PacketTransformer.transform, RTPConnectorOutputStream.java:268-300)."""

    def __init__(self, engine: "SRTPEngine", max_packets: int, max_seg_bytes: int, depth: int = 3):
        self.engine = engine
        h = C.c_void_p()
        N.check(N.lib().srtp_pipeline_create(engine.h, max_packets, max_seg_bytes, depth,
                                             C.byref(h)), engine.h, "srtp_pipeline_create")
        self.h = h
        self.depth = depth
        self._slots = []
        for i in range(depth):
            sl = N.PipelineSlot()
            N.check(N.lib().srtp_pipeline_slot_get(self.h, i, C.byref(sl)), engine.h, "slot_get")
            m = sl.max_packets

            def view(ptr, ct, count):
                return np.ctypeslib.as_array((ct * count).from_address(ptr))
            self._slots.append(dict(
                seg=view(sl.seg, C.c_uint8, sl.seg_cap), off=view(sl.off, C.c_uint32, m),
                len=view(sl.len, C.c_uint32, m), cap=view(sl.cap, C.c_uint32, m),
                flags=view(sl.flags, C.c_uint32, m), tids=view(sl.tids, C.c_int32, m),
                status=view(sl.status, C.c_int32, m)))

    def slot(self, i: int) -> dict:
        return self._slots[i]

    def submit(self, i: int, reverse: bool, n: int, seg_bytes: int, tid=None,
               use_flags: bool = False) -> None:
        """Enqueue slot i's first n packets; ``tid`` = one transformer id, or
        None to use the slot's per-packet ``tids``."""
        N.check(N.lib().srtp_pipeline_submit(self.h, i, int(reverse), int(tid is None),
                                             -1 if tid is None else int(tid), int(use_flags),
                                             n, seg_bytes), self.engine.h, "srtp_pipeline_submit")

    def wait(self, i: int) -> None:
        N.check(N.lib().srtp_pipeline_wait(self.h, i), self.engine.h, "srtp_pipeline_wait")

    def close(self) -> None:
        if self.h:
            self._slots = []
            N.lib().srtp_pipeline_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def profile_policies(profile: str):
    """(srtpPolicy, srtcpPolicy) of a DTLS-SRTP protection profile, as the table
    in transform/dtls/DtlsPacketTransformer.java:574-612 builds them (note the
    10-byte SRTCP tag of the _32 profiles), of the SDES F8 crypto suite
    (transform/sdes/SDesTransformEngine.java:129-176: AES-F8, 10-byte tags), or
    of the AES-256-CM suites (RFC 6188; SDesControlImpl.java:71-72 lists them,
    ZRTP's AES3 yields the same policy, ZRTPTransformEngine.java:873-900)."""
    P = SRTPPolicy
    table = {
        "AES_CM_128_HMAC_SHA1_80": (P.AESCM_ENCRYPTION, 16, 14, 10, 10),
        "AES_CM_128_HMAC_SHA1_32": (P.AESCM_ENCRYPTION, 16, 14, 4, 10),
        "NULL_HMAC_SHA1_80": (P.NULL_ENCRYPTION, 0, 0, 10, 10),
        "NULL_HMAC_SHA1_32": (P.NULL_ENCRYPTION, 0, 0, 4, 10),
        "F8_128_HMAC_SHA1_80": (P.AESF8_ENCRYPTION, 16, 14, 10, 10),
        # ZRTP "2FS" Twofish policies (ZRTPTransformEngine.java:864-900: Twofish
        # with HMAC-SHA1 "HS80"/"HS32"; key length 128 or 256 bits)
        "TWOFISH_CM_128_HMAC_SHA1_80": (P.TWOFISH_ENCRYPTION, 16, 14, 10, 10),
        "TWOFISH_CM_128_HMAC_SHA1_32": (P.TWOFISH_ENCRYPTION, 16, 14, 4, 10),
        "TWOFISH_CM_256_HMAC_SHA1_80": (P.TWOFISH_ENCRYPTION, 32, 14, 10, 10),
        "TWOFISH_F8_128_HMAC_SHA1_80": (P.TWOFISHF8_ENCRYPTION, 16, 14, 10, 10),
        "TWOFISH_F8_256_HMAC_SHA1_80": (P.TWOFISHF8_ENCRYPTION, 32, 14, 10, 10),
        # AES-256-CM (RFC 6188): SRTPCryptoContext with encKeyLength 32
        "AES_256_CM_HMAC_SHA1_80": (P.AESCM_ENCRYPTION, 32, 14, 10, 10),
        "AES_256_CM_HMAC_SHA1_32": (P.AESCM_ENCRYPTION, 32, 14, 4, 10),
    }
    # ZRTP "SK32" / "SK64" Skein-MAC policies (ZRTPTransformEngine.java:867-909:
    # SKEIN_AUTHENTICATION with a 32-byte auth key, tag of srtpAuthTagLen / 8
    # bytes, one policy for SRTP and SRTCP) over AES-CM ("AES1"/"AES3") or
    # Twofish ("2FS1"/"2FS3")
    skein = {
        "AES_CM_128_SKEIN_32": (P.AESCM_ENCRYPTION, 16, 4),
        "AES_CM_128_SKEIN_64": (P.AESCM_ENCRYPTION, 16, 8),
        "AES_256_CM_SKEIN_64": (P.AESCM_ENCRYPTION, 32, 8),
        "TWOFISH_CM_128_SKEIN_32": (P.TWOFISH_ENCRYPTION, 16, 4),
        "TWOFISH_CM_256_SKEIN_64": (P.TWOFISH_ENCRYPTION, 32, 8),
    }
    if profile in skein:
        enc, klen, tag = skein[profile]
        pol = P(enc, klen, P.SKEIN_AUTHENTICATION, 32, tag, 14)
        return pol, P(enc, klen, P.SKEIN_AUTHENTICATION, 32, tag, 14)
    enc, klen, slen, rtp_tag, rtcp_tag = table[profile]
    return (P(enc, klen, P.HMACSHA1_AUTHENTICATION, 20, rtp_tag, slen),
            P(enc, klen, P.HMACSHA1_AUTHENTICATION, 20, rtcp_tag, slen))


class SRTPEngine:
    """One MI355X device's engine: HBM tables of session keys and contexts."""

    _default = {}
    _lock = threading.Lock()

    def __init__(self, device: int = 0, check_replay: bool = True, abort_on_error: bool = True,
                 max_contexts: int = 1 << 20, max_factories: int = 1 << 14,
                 max_transformers: int = 1 << 16, max_batch: int = 1 << 16):
        L = N.lib()
        o = N.EngineOpts()
        L.srtp_engine_opts_default(C.byref(o))
        o.device, o.check_replay, o.abort_on_error = device, int(check_replay), int(abort_on_error)
        o.max_contexts, o.max_factories = max_contexts, max_factories
        o.max_transformers, o.max_batch = max_transformers, max_batch
        h = C.c_void_p()
        N.check(L.srtp_engine_create(C.byref(o), C.byref(h)), None, "srtp_engine_create")
        self.h = h
        self.device = device
        # test hook: SRTP_TEST_DEBUG=<flags> puts every engine of a test run on
        # e.g. the split path (N.DEBUG_FORCE_WIDE) or the fused one (N.DEBUG_NO_WIDE)
        self._env_debug = int(os.environ.get("SRTP_TEST_DEBUG", "0"), 0)
        if self._env_debug:
            self.set_debug(0)

    @classmethod
    def default(cls, device: int = 0) -> "SRTPEngine":
        with cls._lock:
            if device not in cls._default:
                cls._default[device] = SRTPEngine(device)
            return cls._default[device]

    def close(self):
        if self.h:
            _rp_close_all(self)
            N.lib().srtp_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self, stream=None):
        N.check(N.lib().srtp_engine_sync(self.h, stream), self.h, "srtp_engine_sync")

    @property
    def stream_ptr(self) -> int:
        """hipStream_t of the engine's own stream (transform_device's default)."""
        return N.lib().srtp_engine_stream(self.h) or 0

    def set_timing(self, enable: bool) -> None:
        N.check(N.lib().srtp_engine_set_timing(self.h, int(enable)), self.h, "set_timing")

    def set_debug(self, flags: int) -> None:
        """Test hooks (srtp_engine_set_debug), e.g. N.DEBUG_FORCE_CHAIN_STALL."""
        flags = int(flags) | getattr(self, "_env_debug", 0)
        N.check(N.lib().srtp_engine_set_debug(self.h, flags), self.h, "set_debug")

    def read_timing(self) -> dict:
        """{stage: (total ms, bundles)} since the last read (HIP events)."""
        ms = (C.c_double * len(N.STAGES))()
        cnt = (C.c_uint64 * len(N.STAGES))()
        N.check(N.lib().srtp_engine_read_timing(self.h, ms, cnt), self.h, "read_timing")
        return {name: (ms[i], cnt[i]) for i, name in enumerate(N.STAGES)}

    def num_contexts(self) -> int:
        return N.check(N.lib().srtp_engine_num_contexts(self.h), self.h, "num_contexts")

    def stats(self) -> dict:
        """srtp_engine_stats: cumulative per-status counts, ROC re-checks,
        repairs, context-table occupancy / overflow / rehashes."""
        st = N.Stats()
        N.check(N.lib().srtp_engine_stats(self.h, C.byref(st)), self.h, "stats")
        return st.as_dict()

    # -- control plane used by SRTPContextFactory / SRTPTransformer ----------
    def _factory_create(self, sender, key, salt, klen, slen, srtp, srtcp) -> int:
        fid = C.c_int32()
        rc = N.lib().srtp_factory_create(self.h, int(sender), key, klen, salt, slen, C.byref(srtp),
                                         C.byref(srtcp), C.byref(fid))
        N.check(rc, self.h, "SRTPContextFactory")
        return fid.value

    def _factory_close(self, fid: int) -> None:
        N.check(N.lib().srtp_factory_close(self.h, fid), self.h, "close")

    def _transformer_create(self, kind: int, fwd: int, rev: int) -> int:
        tid = C.c_int32()
        N.check(N.lib().srtp_transformer_create(self.h, kind, fwd, rev, C.byref(tid)), self.h,
                "transformer_create")
        return tid.value

    def _transformer_set_factory(self, tid: int, fid: int, forward: bool) -> None:
        N.check(N.lib().srtp_transformer_set_factory(self.h, tid, fid, int(forward)), self.h,
                "setFactory")

    def _transformer_close(self, tid: int) -> None:
        N.check(N.lib().srtp_transformer_close(self.h, tid), self.h, "close")

    def context_state(self, transformer: "_SRTPBase", ssrc: int) -> Optional[dict]:
        st = N.CtxState()
        rc = N.check(N.lib().srtp_get_context_state(self.h, transformer.tid, ssrc & 0xFFFFFFFF,
                                                    C.byref(st)), self.h, "get_context_state")
        if rc == 0:
            return None
        return {k: getattr(st, k) for k, _ in N.CtxState._fields_}

    def export_contexts(self, transformer: "_SRTPBase") -> dict:
        """{ssrc: state} of every context the transformer holds:
        ROC / s_l / replay window / SRTCP indices, to move a stream to another
        engine or GPU with srtp_set_context_state."""
        L = N.lib()
        cnt = C.c_uint32()
        N.check(L.srtp_export_contexts(self.h, transformer.tid, None, None, 0, C.byref(cnt)), self.h,
                "export_contexts")
        n = cnt.value
        ssrcs = (C.c_uint32 * max(n, 1))()
        states = (N.CtxState * max(n, 1))()
        N.check(L.srtp_export_contexts(self.h, transformer.tid, ssrcs, states, n, C.byref(cnt)),
                self.h, "export_contexts")
        return {int(ssrcs[i]): {k: getattr(states[i], k) for k, _ in N.CtxState._fields_}
                for i in range(min(n, cnt.value))}

    def import_context(self, transformer: "_SRTPBase", ssrc: int, state: dict,
                       forward: bool) -> None:
        """Create or overwrite the transformer's context for ssrc with an
        exported state, keyed by its forward or reverse factory."""
        st = N.CtxState(**{k: state.get(k, 0) for k, _ in N.CtxState._fields_})
        N.check(N.lib().srtp_set_context_state(self.h, transformer.tid, ssrc & 0xFFFFFFFF,
                                               int(forward), C.byref(st)), self.h, "import_context")

    # -- bundle entry points -------------------------------------------------
    def transform_host(self, reverse: bool, tid, seg: np.ndarray, off: np.ndarray,
                       length: np.ndarray, cap: np.ndarray, flags=None) -> np.ndarray:
        """Process a packed bundle held in host memory (copied to HBM and back).
        ``tid`` is one transformer id or an int32 array with one id per packet."""
        n = len(off)
        assert seg.dtype == np.uint8 and seg.flags.c_contiguous
        off = np.ascontiguousarray(off, np.uint32)
        cap = np.ascontiguousarray(cap, np.uint32)
        assert length.dtype == np.uint32 and length.flags.c_contiguous and len(length) == n
        status = np.zeros(n, np.int32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint32)
        if np.isscalar(tid):
            tids_p, tid0 = None, int(tid)
        else:
            tids = np.ascontiguousarray(tid, np.int32)
            tids_p, tid0 = tids.ctypes.data, -1
        rc = N.lib().srtp_transform_host(
            self.h, int(reverse), tids_p, tid0, seg.ctypes.data, seg.nbytes, off.ctypes.data,
            length.ctypes.data, cap.ctypes.data, None if fl is None else fl.ctypes.data,
            status.ctypes.data, n)
        N.check(rc, self.h, "srtp_transform_host")
        return status

    def transform_device(self, reverse: bool, tid, seg, off, length, cap, status, flags=None,
                         n: Optional[int] = None, stream=None) -> None:
        """Enqueue a bundle whose buffers are device tensors (torch, on this
        engine's GPU).  ``tid`` is an int or an int32 device tensor.  Async on
        ``stream`` (a torch.cuda.Stream or raw hipStream_t pointer); None =
        the device's default stream (torch's default stream too), ordered after
        the torch work that produced the tensors there.  ``stream_ptr`` is the
        engine's own stream (one hardware queue per engine)."""
        if n is None:
            n = off.numel()
        if np.isscalar(tid):
            tids_p, tid0 = None, int(tid)
        else:
            tids_p, tid0 = tid.data_ptr(), -1
        sp = getattr(stream, "cuda_stream", stream)
        rc = N.lib().srtp_transform_device(
            self.h, int(reverse), tids_p, tid0, seg.data_ptr(), off.data_ptr(), length.data_ptr(),
            cap.data_ptr(), None if flags is None else flags.data_ptr(), status.data_ptr(), n, sp)
        N.check(rc, self.h, "srtp_transform_device")


def host_register(arr: np.ndarray) -> None:
    """Pins ``arr``'s memory for DMA by every GPU (srtp_host_register): a
    long-lived buffer pool registered once, which the dispatcher then moves
    with no host copy (a one-shard bundle, or each shard's packets back to
    back).  Unregister before the array is freed."""
    assert arr.flags.c_contiguous and arr.nbytes > 0
    N.check(N.lib().srtp_host_register(arr.ctypes.data, arr.nbytes), None, "srtp_host_register")


def host_unregister(arr: np.ndarray) -> None:
    N.check(N.lib().srtp_host_unregister(arr.ctypes.data), None, "srtp_host_unregister")


class HostBuffer:
    """Pinned host memory of the engine's own (srtp_host_alloc), registered for
    in-place DMA like host_register's, at the full PCIe rate: ``array`` is a
    uint8 view of it.  close() frees it; no view may be used afterwards."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        N.check(N.lib().srtp_host_alloc(int(nbytes), C.byref(p)), None, "srtp_host_alloc")
        self._p = p
        self.array = np.ctypeslib.as_array((C.c_uint8 * int(nbytes)).from_address(p.value))

    def close(self):
        if self._p:
            self.array = None
            N.check(N.lib().srtp_host_free(self._p), None, "srtp_host_free")
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_is_registered(arr: np.ndarray) -> bool:
    return bool(N.lib().srtp_host_is_registered(arr.ctypes.data, arr.nbytes))


class SRTPDispatcher:
    """In-process multi-GPU engine (srtp_dispatch_*, C ABI): one engine per
    shard on ``devices[i]`` (several shards may share a GPU), each bundle split
    by SSRC (shard = srtp_shard_of(SSRC)), results identical to one engine.
    Usable wherever an SRTPEngine is (``engine=`` of SRTPContextFactory)."""

    def __init__(self, devices: Sequence[int], check_replay: bool = True,
                 abort_on_error: bool = True, max_contexts: int = 1 << 20,
                 max_factories: int = 1 << 14, max_transformers: int = 1 << 16,
                 max_batch: int = 1 << 16):
        L = N.lib()
        o = N.EngineOpts()
        L.srtp_engine_opts_default(C.byref(o))
        o.check_replay, o.abort_on_error = int(check_replay), int(abort_on_error)
        o.max_contexts, o.max_factories = max_contexts, max_factories
        o.max_transformers, o.max_batch = max_transformers, max_batch
        devs = (C.c_int32 * len(devices))(*devices)
        h = C.c_void_p()
        N.check(L.srtp_dispatch_create(devs, len(devices), C.byref(o), C.byref(h)), None,
                "srtp_dispatch_create")
        self.h = h
        self.devices = list(devices)

    @property
    def shards(self) -> int:
        return N.lib().srtp_dispatch_num_shards(self.h)

    def shard_of(self, ssrc: int) -> int:
        return N.lib().srtp_shard_of(ssrc & 0xFFFFFFFF, self.shards)

    def close(self):
        if self.h:
            _rp_close_all(self)
            N.lib().srtp_dispatch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        return N.check(rc, None, what, dispatch=self.h)

    def stats(self) -> dict:
        st = N.Stats()
        self._chk(N.lib().srtp_dispatch_stats(self.h, C.byref(st)), "stats")
        return st.as_dict()

    def host_times(self) -> dict:
        """srtp_dispatch_host_times in ms (plan, pack, wait, scatter, total) and calls."""
        ns = (C.c_uint64 * 6)()
        self._chk(N.lib().srtp_dispatch_host_times(self.h, ns), "host_times")
        d = {k: ns[i] / 1e6 for i, k in enumerate(("plan_ms", "pack_ms", "wait_ms", "scatter_ms",
                                                    "total_ms"))}
        d["calls"] = int(ns[5])
        return d

    def context_state(self, transformer: "_SRTPBase", ssrc: int) -> Optional[dict]:
        st = N.CtxState()
        rc = self._chk(N.lib().srtp_dispatch_get_context_state(self.h, transformer.tid,
                                                               ssrc & 0xFFFFFFFF, C.byref(st)),
                       "get_context_state")
        if rc == 0:
            return None
        return {k: getattr(st, k) for k, _ in N.CtxState._fields_}

    def import_context(self, transformer: "_SRTPBase", ssrc: int, state: dict,
                       forward: bool) -> None:
        st = N.CtxState(**{k: state.get(k, 0) for k, _ in N.CtxState._fields_})
        self._chk(N.lib().srtp_dispatch_set_context_state(self.h, transformer.tid, ssrc & 0xFFFFFFFF,
                                                          int(forward), C.byref(st)),
                  "import_context")

    def _factory_create(self, sender, key, salt, klen, slen, srtp, srtcp) -> int:
        fid = C.c_int32()
        self._chk(N.lib().srtp_dispatch_factory_create(self.h, int(sender), key, klen, salt, slen,
                                                       C.byref(srtp), C.byref(srtcp), C.byref(fid)),
                  "SRTPContextFactory")
        return fid.value

    def _factory_close(self, fid: int) -> None:
        self._chk(N.lib().srtp_dispatch_factory_close(self.h, fid), "close")

    def _transformer_create(self, kind: int, fwd: int, rev: int) -> int:
        tid = C.c_int32()
        self._chk(N.lib().srtp_dispatch_transformer_create(self.h, kind, fwd, rev, C.byref(tid)),
                  "transformer_create")
        return tid.value

    def _transformer_set_factory(self, tid: int, fid: int, forward: bool) -> None:
        self._chk(N.lib().srtp_dispatch_transformer_set_factory(self.h, tid, fid, int(forward)),
                  "setFactory")

    def _transformer_close(self, tid: int) -> None:
        self._chk(N.lib().srtp_dispatch_transformer_close(self.h, tid), "close")

    def transform_host(self, reverse: bool, tid, seg: np.ndarray, off: np.ndarray,
                       length: np.ndarray, cap: np.ndarray, flags=None) -> np.ndarray:
        """As SRTPEngine.transform_host, split across the shards."""
        n = len(off)
        assert seg.dtype == np.uint8 and seg.flags.c_contiguous
        off = np.ascontiguousarray(off, np.uint32)
        cap = np.ascontiguousarray(cap, np.uint32)
        assert length.dtype == np.uint32 and length.flags.c_contiguous and len(length) == n
        status = np.zeros(n, np.int32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint32)
        if np.isscalar(tid):
            tids_p, tid0 = None, int(tid)
        else:
            tids = np.ascontiguousarray(tid, np.int32)
            tids_p, tid0 = tids.ctypes.data, -1
        rc = N.lib().srtp_dispatch_transform_host(
            self.h, int(reverse), tids_p, tid0, seg.ctypes.data, seg.nbytes, off.ctypes.data,
            length.ctypes.data, cap.ctypes.data, None if fl is None else fl.ctypes.data,
            status.ctypes.data, n)
        self._chk(rc, "srtp_dispatch_transform_host")
        return status

    def submit_host(self, reverse: bool, tid, seg: np.ndarray, off: np.ndarray,
                    length: np.ndarray, cap: np.ndarray, flags=None) -> "HostTicket":
        """srtp_dispatch_submit_host: transform_host without waiting.  The
        arrays (kept alive by the returned ticket) must not be touched until
        ``ticket.wait()`` (srtp_dispatch_wait_host) returns the statuses."""
        n = len(off)
        assert seg.dtype == np.uint8 and seg.flags.c_contiguous
        off = np.ascontiguousarray(off, np.uint32)
        cap = np.ascontiguousarray(cap, np.uint32)
        assert length.dtype == np.uint32 and length.flags.c_contiguous and len(length) == n
        status = np.zeros(n, np.int32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint32)
        tids = None
        if np.isscalar(tid):
            tids_p, tid0 = None, int(tid)
        else:
            tids = np.ascontiguousarray(tid, np.int32)
            tids_p, tid0 = tids.ctypes.data, -1
        t = C.c_uint64()
        rc = N.lib().srtp_dispatch_submit_host(
            self.h, int(reverse), tids_p, tid0, seg.ctypes.data, seg.nbytes, off.ctypes.data,
            length.ctypes.data, cap.ctypes.data, None if fl is None else fl.ctypes.data,
            status.ctypes.data, n, C.byref(t))
        self._chk(rc, "srtp_dispatch_submit_host")
        return HostTicket(self, t.value, status, (seg, off, length, cap, fl, tids))


class HostTicket:
    """A host bundle in flight (SRTPDispatcher.submit_host)."""

    def __init__(self, d: SRTPDispatcher, ticket: int, status: np.ndarray, keep):
        self.d, self.ticket, self.status, self._keep = d, ticket, status, keep
        self.done = False

    def wait(self) -> np.ndarray:
        if not self.done:
            self.d._chk(N.lib().srtp_dispatch_wait_host(self.d.h, self.ticket), "srtp_dispatch_wait_host")
            self.done = True
            self._keep = None
        return self.status


class SRTPAggregator:
    """Per-packet submits from many threads -> bundles (srtp_aggregator_*,
    SURVEY.md 8f.2).  ``callback(cookie, status, data)`` runs on a dispatch
    thread once per packet, in bundle order; packets of one direction (and,
    over a dispatcher, of one shard) complete in the order they were
    accepted.  ``engine`` is an SRTPEngine or an SRTPDispatcher (one lane per
    shard, srtp_aggregator_create_dispatch).  Each packet is its own
    1-element RawPacket[] as in the reference's RTPConnector streams
    (RTPConnectorInputStream.java:425-452, RTPConnectorOutputStream.java
    :268-300,652-830), whatever the engine's abort_on_error.  ``callback``
    None: only synchronous ``transform`` calls.  ``seal_idle``: a lane with no
    bundle in flight seals at once (SRTP_AGG_SEAL_IDLE)."""

    def __init__(self, engine, callback, max_packets: int = 1 << 14,
                 max_bytes: int = 24 << 20, deadline_us: int = 1000, depth: int = 4,
                 seal_idle: bool = True):
        self.engine = engine
        o = N.AggregatorOpts(max_packets, max_bytes, deadline_us, depth,
                             N.AGG_SEAL_IDLE if seal_idle else 0)

        def _cb(user, cookie, status, data, length):
            callback(int(cookie), int(status), C.string_at(data, length) if length else b"")

        self._cb = N.AGG_CB(_cb) if callback is not None else N.AGG_CB()  # kept alive
        h = C.c_void_p()
        if isinstance(engine, SRTPDispatcher):
            rc = N.lib().srtp_aggregator_create_dispatch(engine.h, C.byref(o), self._cb, None,
                                                         C.byref(h))
            N.check(rc, None, "srtp_aggregator_create_dispatch")
        else:
            N.check(N.lib().srtp_aggregator_create(engine.h, C.byref(o), self._cb, None, C.byref(h)),
                    engine.h, "srtp_aggregator_create")
        self.h = h

    def submit(self, reverse: bool, transformer: "_SRTPBase", data: bytes, flags: int = 0,
               cookie: int = 0) -> int:
        """0, or N.EFULL for a submit from a callback that found no free slot."""
        data = bytes(data)
        rc = N.lib().srtp_aggregator_submit(self.h, int(reverse), transformer.tid, data, len(data),
                                            flags, cookie)
        if rc == N.EFULL:
            return rc
        return N.check(rc, None, "submit")

    def transform(self, reverse: bool, transformer: "_SRTPBase", data: bytes, flags: int = 0):
        """Synchronous (srtp_aggregator_transform): (status, bytes) of one
        packet, sharing bundles with concurrent callers."""
        data = bytes(data)
        cap = len(data) if reverse else len(data) + 16
        out = (C.c_uint8 * max(cap, 1))()
        st, ol = C.c_int32(), C.c_uint32()
        N.check(N.lib().srtp_aggregator_transform(self.h, int(reverse), transformer.tid, data, len(data),
                                                  len(data), cap, flags, out, C.byref(st), C.byref(ol)),
                None, "srtp_aggregator_transform")
        return int(st.value), bytes(out[:ol.value])

    def flush(self) -> None:
        N.check(N.lib().srtp_aggregator_flush(self.h), None, "flush")

    def stats(self) -> dict:
        a, c, b = C.c_uint64(), C.c_uint64(), C.c_uint64()
        N.lib().srtp_aggregator_stats(self.h, C.byref(a), C.byref(c), C.byref(b))
        return {"accepted": a.value, "completed": c.value, "bundles": b.value}

    def close(self) -> None:
        if self.h:
            N.lib().srtp_aggregator_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SRTPContextFactory:
    """SRTPContextFactory(sender, masterKey, masterSalt, srtpPolicy, srtcpPolicy)."""

    def __init__(self, sender: bool, masterKey: bytes, masterSalt: bytes, srtpPolicy: SRTPPolicy,
                 srtcpPolicy: SRTPPolicy, engine=None):
        self.engine = engine or SRTPEngine.default()
        key = (C.c_uint8 * len(masterKey)).from_buffer_copy(bytes(masterKey))
        salt = (C.c_uint8 * len(masterSalt)).from_buffer_copy(bytes(masterSalt))
        try:
            self.fid = self.engine._factory_create(sender, key, salt, len(masterKey),
                                                   len(masterSalt), srtpPolicy._c(),
                                                   srtcpPolicy._c())
        finally:
            C.memset(key, 0, len(masterKey))
            C.memset(salt, 0, len(masterSalt))
        self.sender = sender
        self.srtpPolicy, self.srtcpPolicy = srtpPolicy, srtcpPolicy

    def close(self):
        self.engine._factory_close(self.fid)


class RawPacket:
    """Packet view (nm/RawPacket.java): buffer, offset, length, flags."""

    FIXED_HEADER_SIZE = 12
    EXT_HEADER_SIZE = 4

    def __init__(self, buffer, offset: int = 0, length: Optional[int] = None, flags: int = 0):
        self.buffer = bytearray(buffer)
        self.offset = offset
        self.length = len(self.buffer) - offset if length is None else length
        self.flags = flags

    def getBuffer(self): return self.buffer
    def getOffset(self): return self.offset
    def getLength(self): return self.length
    def getFlags(self): return self.flags
    def setFlags(self, f): self.flags = f

    def data(self) -> bytes:
        return bytes(self.buffer[self.offset:self.offset + self.length])

    def readByte(self, off): return self.buffer[self.offset + off]

    def readInt(self, off):
        return int.from_bytes(self.buffer[self.offset + off:self.offset + off + 4], "big")

    def getSequenceNumber(self):
        return int.from_bytes(self.buffer[self.offset + 2:self.offset + 4], "big")

    def getSSRC(self): return self.readInt(8)
    def getRTCPSSRC(self): return self.readInt(4)

    def getHeaderLength(self):
        b0 = self.buffer[self.offset]
        h = 12 + 4 * (b0 & 0x0F)
        if b0 & 0x10:
            i = self.offset + 12 + 4 * (b0 & 0x0F) + 2
            hi = self.buffer[i] - 256 if self.buffer[i] >= 128 else self.buffer[i]
            h += 4 + ((hi << 8) | self.buffer[i + 1]) * 4
        return h

    def getPayloadLength(self): return self.length - self.getHeaderLength()

    def isInvalid(self):
        return len(self.buffer) < self.offset + self.length or self.length < 12


TRAILER_ROOM = 16  # largest trailer: SRTCP E|index (4) + 12-byte tag


def block_encrypt(enc_type: int, key: bytes, block: bytes) -> bytes:
    """One block of the policy's cipher on the host (AES-128/256, Twofish)."""
    out = (C.c_uint8 * 16)()
    N.check(N.lib().srtp_block_encrypt(enc_type, bytes(key), len(key), bytes(block)[:16], out), None,
            "block_encrypt")
    return bytes(out)


def derive_session_keys_for(enc_type: int, masterKey: bytes, masterSalt: bytes, rtcp: bool = False):
    """Session keys with the policy's cipher as the PRF (Twofish for the ZRTP
    Twofish policies, AES otherwise)."""
    mk = bytes(masterKey)
    klen = 32 if len(mk) >= 32 else 16
    enc, auth, salt = (C.c_uint8 * klen)(), (C.c_uint8 * 20)(), (C.c_uint8 * 14)()
    N.check(N.lib().srtp_derive_session_keys_for(enc_type, mk[:klen], klen, bytes(masterSalt)[:14],
                                                 int(rtcp), enc, auth, salt), None, "kdf")
    return bytes(enc), bytes(auth), bytes(salt)


def derive_session_keys_auth(enc_type: int, masterKey: bytes, masterSalt: bytes, rtcp: bool = False,
                             auth_len: int = 20):
    """Session keys with an auth key of `auth_len` bytes (ZRTP's Skein
    policies: 32, ZRTPTransformEngine.java:867-872)."""
    mk = bytes(masterKey)
    klen = 32 if len(mk) >= 32 else 16
    enc, auth, salt = (C.c_uint8 * klen)(), (C.c_uint8 * auth_len)(), (C.c_uint8 * 14)()
    N.check(N.lib().srtp_derive_session_keys_auth(enc_type, mk[:klen], klen, bytes(masterSalt)[:14],
                                                  int(rtcp), enc, auth, auth_len, salt), None, "kdf")
    return bytes(enc), bytes(auth), bytes(salt)


def skein512_mac(key: bytes, msg: bytes, out_bits: int = 512) -> bytes:
    """The engine's host Skein-512 (version 1.3): keyed like bccontrib's SkeinMac
    (plain hash for an empty key), out_bits output bits."""
    out = (C.c_uint8 * ((out_bits + 7) // 8))()
    N.check(N.lib().srtp_skein512_mac(bytes(key), len(key), out_bits, bytes(msg), len(msg), out), None,
            "skein512_mac")
    return bytes(out)


def derive_session_keys(masterKey: bytes, masterSalt: bytes, rtcp: bool = False):
    """The engine's host-side RFC 3711 4.3 key derivation (no GPU needed); a
    32-byte master key selects the AES-256 PRF and a 32-byte session key
    (RFC 6188 4.1)."""
    mk = bytes(masterKey)
    klen = 32 if len(mk) >= 32 else 16
    enc, auth, salt = (C.c_uint8 * klen)(), (C.c_uint8 * 20)(), (C.c_uint8 * 14)()
    N.check(N.lib().srtp_derive_session_keys_n(mk[:klen], klen, bytes(masterSalt)[:14], int(rtcp),
                                               enc, auth, salt), None, "kdf")
    return bytes(enc), bytes(auth), bytes(salt)


def pack(pkts: Sequence[Optional[RawPacket]], predicate=None, reverse: bool = False):
    """RawPacket[] -> (seg, off, len, cap, flags): the marshalling a JNI shim
    does.  Each packet region is 16-byte aligned and holds the
    packet's buffer bytes from its offset; ``cap`` is the Java buffer's length
    after the offset, so RawPacket.isInvalid and the bounds the reference
    reads against (getHeaderLength's extension field, readRegionToBuff) are the
    same.  For protect, ``cap`` also leaves room for the trailer (the in-place
    form of RawPacket.append / grow), so a packet whose header-extension
    length field lies past its buffer reads the zero padding there instead of
    throwing (the one protect-side difference from the reference's
    AIOOBE).  ``None`` elements and packets the predicate rejects are flagged
    SKIP (SinglePacketTransformer.java:121-216 never hands them to the
    transformer)."""
    n = len(pkts)
    off = np.zeros(n, np.uint32)
    length = np.zeros(n, np.uint32)
    cap = np.zeros(n, np.uint32)
    flags = np.zeros(n, np.uint32)
    pos = 0
    for i, p in enumerate(pkts):
        if p is None or (predicate is not None and not predicate(p)):
            flags[i] = N.PKT_FLAG_SKIP
            cap[i] = 16
        else:
            avail = len(p.buffer) - p.offset
            fits = p.length <= avail
            cap[i] = max(avail, p.length + TRAILER_ROOM) if fits and not reverse else max(avail, 0)
            length[i] = p.length
            flags[i] = p.flags & (N.PKT_FLAG_DISCARD | N.PKT_FLAG_SILENCE)
        off[i] = pos
        pos += (int(cap[i]) + 15) & ~15
    seg = np.zeros(max(pos, 16), np.uint8)
    for i, p in enumerate(pkts):
        if p is not None and not (flags[i] & N.PKT_FLAG_SKIP):
            src = np.frombuffer(bytes(p.buffer[p.offset:]), np.uint8)
            seg[off[i]:off[i] + len(src)] = src
    return seg, off, length, cap, flags


class PacketTransformer:
    """transform/PacketTransformer.java:28-53"""

    def close(self):
        raise NotImplementedError

    def transform(self, pkts):
        raise NotImplementedError

    def reverseTransform(self, pkts):
        raise NotImplementedError


_rp_lock = threading.Lock()


def _rp_batch(engine) -> C.c_void_p:
    """The calling thread's srtp_rawpacket_batch on `engine` (an SRTPEngine or
    SRTPDispatcher): the staging of the C marshalling, one per thread as a
    JNI shim keeps one per Java thread."""
    with _rp_lock:
        tl = engine.__dict__.get("_rp_tls")
        if tl is None:
            tl = engine._rp_tls = threading.local()
            engine._rp_all = []
    h = getattr(tl, "h", None)
    if h is None:
        h = C.c_void_p()
        L = N.lib()
        if isinstance(engine, SRTPDispatcher):
            N.check(L.srtp_rawpacket_batch_create_dispatch(engine.h, C.byref(h)), None, "rawpacket")
        else:
            N.check(L.srtp_rawpacket_batch_create(engine.h, C.byref(h)), engine.h, "rawpacket")
        tl.h = h
        with _rp_lock:
            engine._rp_all.append(h)
    return h


def _rp_close_all(engine) -> None:
    agg = engine.__dict__.pop("_pkt_agg", None)
    if agg is not None:
        agg.close()
    with _rp_lock:
        for h in engine.__dict__.get("_rp_all", []):
            N.lib().srtp_rawpacket_batch_destroy(h)
        engine.__dict__["_rp_all"] = []
        engine.__dict__.pop("_rp_tls", None)


def _packet_aggregator(engine) -> "SRTPAggregator":
    """The engine's (or dispatcher's: one lane per shard) aggregator for
    per-packet calls, created on first use -- what the JNI shim keeps one of
    per process."""
    with _rp_lock:
        agg = engine.__dict__.get("_pkt_agg")
        if agg is None:
            agg = engine._pkt_agg = SRTPAggregator(engine, None, max_packets=4096, max_bytes=8 << 20,
                                                   deadline_us=500, depth=4, seal_idle=True)
    return agg


_grow_tls = threading.local()
_GROW = 65536 + 16


def _rawpacket_one(engine, reverse: bool, tid: int, pkt: "RawPacket"):
    """SinglePacketTransformer.transform / reverseTransform(RawPacket)
    (SinglePacketTransformer.java:113,169; SRTPTransformer.java:185-219,
    SRTCPTransformer.java:175-207) through srtp_rawpacket_transform_one: the
    packet joins the bundles of concurrent callers (srtp_aggregator_transform)
    and is written back as the reference leaves it.  Returns the packet or
    None (dropped); raises where the reference throws."""
    g = getattr(_grow_tls, "buf", None)
    if g is None:
        g = _grow_tls.buf = (C.c_uint8 * _GROW)()
    agg = _packet_aggregator(engine)
    buf = pkt.buffer if len(pkt.buffer) else bytearray(1)
    v = (C.c_char * len(buf)).from_buffer(buf)
    length, st, need = C.c_uint32(pkt.length), C.c_int32(), C.c_uint32()
    rc = N.lib().srtp_rawpacket_transform_one(
        agg.h, int(reverse), int(tid), C.addressof(v), len(pkt.buffer), pkt.offset, C.byref(length),
        pkt.flags & (N.PKT_FLAG_DISCARD | N.PKT_FLAG_SILENCE), C.byref(st), C.byref(need), g, _GROW)
    del v
    N.check(rc, None, "srtp_rawpacket_transform_one")
    if need.value:  # the reference's new byte[] (RawPacket.append / grow): the result at offset 0
        nb = bytearray(need.value)
        nb[:length.value] = bytes(g[:length.value])
        pkt.buffer, pkt.offset = nb, 0
    pkt.length = int(length.value)
    s = int(st.value)
    if s == N.STATUS_ERR_MALFORMED:
        raise SRTPTransformException("Failed to transform RawPacket! (malformed for SRTP)")
    return pkt if s == N.STATUS_OK else None


def _rawpacket_run(engine, reverse: bool, tids, pkts, predicate=None):
    """transform / reverseTransform(RawPacket[]) through the C marshalling
    (srtp_rawpacket_transform, libjitsi_amd/csrc/rawpacket.cpp), with what a
    JNI shim does around it: hand over each RawPacket's buffer, offset, length
    and flags; afterwards move a packet the reference gives a new buffer
    (RawPacket.append without room, RawPacket.grow: need_len) to a new buffer
    at offset 0, replace dropped elements with None, and rethrow a throw after
    the whole array was written back (SinglePacketTransformer.java:121-216).
    ``tids`` is one transformer id or one per packet (-1: no transformer)."""
    n = len(pkts)
    L = N.lib()
    bufs = (C.c_void_p * n)()
    buf_len = np.zeros(n, np.uint32)
    offset = np.zeros(n, np.uint32)
    length = np.zeros(n, np.uint32)
    flags = np.zeros(n, np.uint32)
    views = []
    for i, p in enumerate(pkts):
        if p is None:
            continue
        if predicate is not None and not predicate(p):
            flags[i] = N.PKT_FLAG_SKIP
        else:
            flags[i] = p.flags & (N.PKT_FLAG_DISCARD | N.PKT_FLAG_SILENCE)
        buf = p.buffer if len(p.buffer) else bytearray(1)
        v = (C.c_char * len(buf)).from_buffer(buf)
        views.append(v)
        bufs[i] = C.addressof(v)
        buf_len[i] = len(p.buffer)
        offset[i] = p.offset
        length[i] = p.length
    status = np.zeros(n, np.int32)
    need = np.zeros(n, np.uint32)
    thrown = C.c_int32(-1)
    if np.isscalar(tids):
        tids_p, tid0 = None, int(tids)
    else:
        tids_a = np.ascontiguousarray(tids, np.int32)
        tids_p, tid0 = tids_a.ctypes.data, -1
    b = _rp_batch(engine)
    rc = L.srtp_rawpacket_transform(b, int(reverse), tids_p, tid0, bufs, buf_len.ctypes.data,
                                    offset.ctypes.data, length.ctypes.data, flags.ctypes.data,
                                    status.ctypes.data, need.ctypes.data, n, C.byref(thrown))
    del views
    N.check(rc, None, "srtp_rawpacket_transform")
    for i, p in enumerate(pkts):
        st = int(status[i])
        if p is None or st in (N.STATUS_SKIPPED, N.STATUS_NOT_PROCESSED):
            continue
        if need[i]:  # the reference's new byte[]: the result at offset 0
            data, dl = C.POINTER(C.c_uint8)(), C.c_uint32()
            N.check(L.srtp_rawpacket_result(b, i, C.byref(data), C.byref(dl)), None, "result")
            nb = bytearray(int(need[i]))
            nb[:dl.value] = C.string_at(data, dl.value)
            p.buffer, p.offset = nb, 0
        p.length = int(length[i])
        if st != N.STATUS_OK and st != N.STATUS_ERR_MALFORMED:
            pkts[i] = None
    if thrown.value >= 0:
        raise SRTPTransformException(
            f"Failed to transform RawPacket(s)! (packet {thrown.value}: malformed for SRTP)")
    return pkts


class _SRTPBase(PacketTransformer):
    KIND = N.KIND_RTP

    def __init__(self, forwardFactory: SRTPContextFactory,
                 reverseFactory: Optional[SRTPContextFactory] = None, packetPredicate=None):
        reverseFactory = reverseFactory or forwardFactory
        self.engine = forwardFactory.engine
        self.forwardFactory, self.reverseFactory = forwardFactory, reverseFactory
        self.packetPredicate = packetPredicate
        self.exceptionsInTransform = 0
        self.exceptionsInReverseTransform = 0
        self.tid = self.engine._transformer_create(self.KIND, forwardFactory.fid,
                                                   reverseFactory.fid)

    def _set_factory(self, factory: SRTPContextFactory, forward: bool):
        self.engine._transformer_set_factory(self.tid, factory.fid, forward)
        if forward:
            self.forwardFactory = factory
        else:
            self.reverseFactory = factory

    def close(self):
        self.engine._transformer_close(self.tid)

    def _count_exception(self, reverse):
        if reverse:
            self.exceptionsInReverseTransform += 1
        else:
            self.exceptionsInTransform += 1

    def _run(self, pkts, reverse):
        """RawPacket: SinglePacketTransformer's per-packet transform(RawPacket)
        (coalesced with concurrent callers).  An array of one element: the
        SinglePacketTransformer array loop over that per-packet call -- the
        connectors' 1-element arrays.  Longer arrays: one bundle
        (srtp_rawpacket_transform) with the loop's abort-on-throw."""
        if pkts is None:
            return None
        if isinstance(pkts, RawPacket):
            return _rawpacket_one(self.engine, reverse, self.tid, pkts)
        if len(pkts) == 0:
            return pkts
        if len(pkts) == 1:
            p = pkts[0]
            if p is not None and (self.packetPredicate is None or self.packetPredicate(p)):
                try:
                    pkts[0] = _rawpacket_one(self.engine, reverse, self.tid, p)
                except SRTPTransformException:
                    self._count_exception(reverse)
                    raise
            return pkts
        try:
            return _rawpacket_run(self.engine, reverse, self.tid, pkts, self.packetPredicate)
        except SRTPTransformException:
            self._count_exception(reverse)
            raise

    def transform(self, pkts):
        return self._run(pkts, False)

    def reverseTransform(self, pkts):
        return self._run(pkts, True)


class SRTPTransformer(_SRTPBase):
    """SRTPTransformer(forwardFactory, reverseFactory)"""

    KIND = N.KIND_RTP

    def setContextFactory(self, factory: SRTPContextFactory, forward: bool):
        self._set_factory(factory, forward)


class SRTCPTransformer(_SRTPBase):
    """SRTCPTransformer(forwardFactory, reverseFactory) or SRTCPTransformer(srtpTransformer)"""

    KIND = N.KIND_RTCP

    def __init__(self, forwardFactory, reverseFactory=None):
        if isinstance(forwardFactory, SRTPTransformer):
            t = forwardFactory
            forwardFactory, reverseFactory = t.forwardFactory, t.reverseFactory
        super().__init__(forwardFactory, reverseFactory)

    def updateFactory(self, factory: SRTPContextFactory, forward: bool):
        self._set_factory(factory, forward)


def transform_bundle(transformers: Sequence[Optional[_SRTPBase]], pkts, reverse: bool):
    """Process packets of many transformers in one GPU bundle (the batching the
    reference's 1-element arrays cannot express).  Equivalent to calling each
    transformer's transform()/reverseTransform() on its packets in order; a
    throw aborts the later packets of that transformer only, and is raised
    once every packet was written back."""
    eng = next(t for t in transformers if t is not None).engine
    pkts = list(pkts)
    masked = [p if t is not None else None for p, t in zip(pkts, transformers)]
    tids = np.array([t.tid if t is not None else -1 for t in transformers], np.int32)
    out = _rawpacket_run(eng, reverse, tids, masked)
    return [o if t is not None else p for o, p, t in zip(out, pkts, transformers)]
