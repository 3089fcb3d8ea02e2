"""ctypes binding of the C oracle (oracle/srtp_oracle.c).

TEST INFRASTRUCTURE ONLY: the parity checker and the CPU baseline.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module.  The product (``libjitsi_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_srtp.so")

# statuses / constants (srtp_oracle.h)
OK, DROP_REPLAY, DROP_AUTH, DROP_VERSION, DROP_NO_CONTEXT = 0, 1, 2, 3, 4
ERR_CAPACITY, ERR_MALFORMED, DROP_INVALID, NOT_PROCESSED, SKIPPED = 5, 6, 7, 8, 9
FLAG_DISCARD, FLAG_SILENCE, FLAG_SKIP = 0x2, 0x4, 0x80000000
KIND_RTP, KIND_RTCP = 0, 1
MODE_REF, MODE_TUNED = 0, 1


class Policy(C.Structure):
    """SRTPPolicy(encType, encKeyLength, authType, authKeyLength, authTagLength,
    saltKeyLength) -- srtp/SRTPPolicy.java:107-120."""

    _fields_ = [(n, C.c_int32) for n in (
        "enc_type", "enc_key_len", "auth_type", "auth_key_len", "auth_tag_len",
        "salt_key_len")]


class CtxState(C.Structure):
    _fields_ = [("roc", C.c_int32), ("s_l", C.c_int32), ("seq_num_set", C.c_int32),
                ("guessed_roc", C.c_int32), ("sent_index", C.c_int32),
                ("received_index", C.c_int32), ("replay_window", C.c_uint64)]


def build() -> str:
    """Compile the oracle with its Makefile (gcc + libcrypto)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, u8p, u32p, i32p = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_int32)
        L.orc_factory_new.restype = vp
        L.orc_factory_new.argtypes = [C.c_int, u8p, C.c_int, u8p, C.c_int, C.POINTER(Policy),
                                      C.POINTER(Policy), C.c_int]
        L.orc_factory_close.argtypes = [vp]
        L.orc_transformer_new.restype = vp
        L.orc_transformer_new.argtypes = [C.c_int, vp, vp]
        L.orc_transformer_set_factory.argtypes = [vp, vp, C.c_int]
        L.orc_transformer_close.argtypes = [vp]
        L.orc_transformer_free.argtypes = [vp]
        L.orc_set_check_replay.argtypes = [C.c_int]
        L.orc_process.restype = C.c_int
        L.orc_process.argtypes = [C.POINTER(vp), C.c_int, C.c_int, u8p, u32p, u32p, u32p, u32p,
                                  i32p, C.c_uint32, C.c_int]
        L.orc_get_state.restype = C.c_int
        L.orc_get_state.argtypes = [vp, C.c_uint32, C.POINTER(CtxState)]
        L.orc_num_contexts.restype = C.c_uint32
        L.orc_num_contexts.argtypes = [vp]
        L.orc_tls_export.restype = C.c_int
        L.orc_tls_export.argtypes = [C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p,
                                     C.c_char_p, C.c_char_p, C.c_int]
        L.orc_export_contexts.restype = C.c_uint32
        L.orc_export_contexts.argtypes = [vp, u32p, C.POINTER(CtxState), C.c_uint32]
        L.orc_set_context_state.restype = C.c_int
        L.orc_set_context_state.argtypes = [vp, C.c_uint32, C.c_int, C.POINTER(CtxState)]
        L.orc_remove_context.restype = C.c_int
        L.orc_remove_context.argtypes = [vp, C.c_uint32]
        L.orc_aes128_encrypt_block.argtypes = [u8p, u8p, u8p]
        L.orc_hmac_sha1.argtypes = [u8p, C.c_int, u8p, C.c_size_t, u8p]
        L.orc_derive_keys.argtypes = [u8p, u8p, C.c_int, u8p, u8p, u8p]
        L.orc_derive_keys_n.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, u8p, u8p]
        L.orc_derive_keys_twofish.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, u8p, u8p]
        L.orc_twofish_encrypt_block.argtypes = [u8p, C.c_int, u8p, u8p]
        L.orc_derive_keys_auth.argtypes = [C.c_int, u8p, C.c_int, u8p, C.c_int, u8p, u8p, C.c_int, u8p]
        L.orc_skein512_mac.argtypes = [u8p, C.c_int, C.c_int, u8p, C.c_size_t, u8p]
        L.orc_skein512_state0.argtypes = [u8p, C.c_int, C.c_int, C.POINTER(C.c_uint64)]
        L.orc_aes_f8.argtypes = [u8p, u8p, C.c_int, u8p, u8p, C.c_int]
        L.orc_bench_round_trips.restype = C.c_int64
        L.orc_bench_round_trips.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, C.c_int,
                                            C.c_uint32, C.POINTER(C.c_double)]
        _lib = L
    return _lib


def _u8(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8).copy()
    return a, a.ctypes.data_as(C.POINTER(C.c_uint8))


def aes128_block(key: bytes, block: bytes) -> bytes:
    k, kp = _u8(key)
    i, ip = _u8(block)
    o = np.zeros(16, np.uint8)
    lib().orc_aes128_encrypt_block(kp, ip, o.ctypes.data_as(C.POINTER(C.c_uint8)))
    return o.tobytes()


def hmac_sha1(key: bytes, msg: bytes) -> bytes:
    k, kp = _u8(key)
    m, mp = _u8(msg if msg else b"\0")
    o = np.zeros(20, np.uint8)
    lib().orc_hmac_sha1(kp, len(key), mp, len(msg), o.ctypes.data_as(C.POINTER(C.c_uint8)))
    return o.tobytes()


def derive_keys(master_key: bytes, master_salt: bytes, rtcp: bool = False):
    """RFC 3711 4.3 session keys (a 32-byte master key: the AES-256 PRF and a
    32-byte cipher key, RFC 6188 4.1)."""
    klen = 32 if len(master_key) >= 32 else 16
    k, kp = _u8(master_key[:klen])
    s, sp = _u8(master_salt)
    enc, auth, salt = np.zeros(klen, np.uint8), np.zeros(20, np.uint8), np.zeros(14, np.uint8)
    P = C.POINTER(C.c_uint8)
    lib().orc_derive_keys_n(kp, klen, sp, int(rtcp), enc.ctypes.data_as(P),
                            auth.ctypes.data_as(P), salt.ctypes.data_as(P))
    return enc.tobytes(), auth.tobytes(), salt.tobytes()


def twofish_block(key: bytes, block: bytes) -> bytes:
    k, kp = _u8(key)
    i, ip = _u8(block)
    o = np.zeros(16, np.uint8)
    lib().orc_twofish_encrypt_block(kp, len(key), ip, o.ctypes.data_as(C.POINTER(C.c_uint8)))
    return o.tobytes()


def derive_keys_twofish(master_key: bytes, master_salt: bytes, rtcp: bool = False):
    """Session keys of a Twofish policy (Twofish PRF, key length = master key's)."""
    klen = 32 if len(master_key) >= 32 else 16
    k, kp = _u8(master_key[:klen])
    s, sp = _u8(master_salt)
    enc, auth, salt = np.zeros(klen, np.uint8), np.zeros(20, np.uint8), np.zeros(14, np.uint8)
    P = C.POINTER(C.c_uint8)
    lib().orc_derive_keys_twofish(kp, klen, sp, int(rtcp), enc.ctypes.data_as(P),
                                  auth.ctypes.data_as(P), salt.ctypes.data_as(P))
    return enc.tobytes(), auth.tobytes(), salt.tobytes()


def skein512(msg: bytes, out_bits: int = 512, key: bytes = b"") -> bytes:
    """Skein-512 (version 1.3) of `msg`, keyed (Skein-MAC, as bccontrib's
    SkeinMac) when `key` is non-empty."""
    k, kp = _u8(key if key else b"\0")
    m, mp = _u8(msg if msg else b"\0")
    o = np.zeros((out_bits + 7) // 8, np.uint8)
    lib().orc_skein512_mac(kp, len(key), out_bits, mp, len(msg), o.ctypes.data_as(C.POINTER(C.c_uint8)))
    return o.tobytes()


def skein512_iv(out_bits: int) -> list:
    """Skein-512's chaining value after the config UBI (unkeyed): the IV."""
    k, kp = _u8(b"\0")
    o = np.zeros(8, np.uint64)
    lib().orc_skein512_state0(kp, 0, out_bits, o.ctypes.data_as(C.POINTER(C.c_uint64)))
    return [int(x) for x in o]


def derive_keys_auth(master_key: bytes, master_salt: bytes, rtcp: bool = False, auth_len: int = 20,
                     twofish: bool = False):
    """Session keys with an auth key of `auth_len` bytes (Skein policies: 32)."""
    klen = 32 if len(master_key) >= 32 else 16
    k, kp = _u8(master_key[:klen])
    s, sp = _u8(master_salt)
    enc, auth, salt = np.zeros(klen, np.uint8), np.zeros(auth_len, np.uint8), np.zeros(14, np.uint8)
    P = C.POINTER(C.c_uint8)
    lib().orc_derive_keys_auth(int(twofish), kp, klen, sp, int(rtcp), enc.ctypes.data_as(P),
                               auth.ctypes.data_as(P), auth_len, salt.ctypes.data_as(P))
    return enc.tobytes(), auth.tobytes(), salt.tobytes()


def aes_f8(key: bytes, salt: bytes, iv: bytes, data: bytes) -> bytes:
    """SRTPCipherF8 (deriveForIV + process) over `data` with IV `iv`."""
    k, kp = _u8(key)
    s, sp = _u8(salt)
    i, ip = _u8(iv)
    d, dp = _u8(data if data else b"\0")
    lib().orc_aes_f8(kp, sp, len(salt), ip, dp, len(data))
    return d.tobytes()[:len(data)]


def bench_round_trips(mode: int, threads: int, seconds: float, pkt_len: int, ssrcs: int,
                      seed: int = 0x5EED0002):
    """(packets protected+unprotected, wall seconds) of the pinned C timing
    loop (oracle_bench.c)."""
    el = C.c_double()
    n = lib().orc_bench_round_trips(mode, threads, seconds, pkt_len, ssrcs, seed, C.byref(el))
    if n < 0:
        raise RuntimeError("oracle benchmark rejected a packet")
    return int(n), el.value


def set_check_replay(enabled: bool) -> None:
    lib().orc_set_check_replay(int(enabled))


class Factory:
    def __init__(self, sender, master_key, master_salt, srtp_policy, srtcp_policy, mode=MODE_REF):
        k, kp = _u8(master_key)
        s, sp = _u8(master_salt)
        self.h = lib().orc_factory_new(int(sender), kp, len(master_key), sp, len(master_salt),
                                       C.byref(srtp_policy), C.byref(srtcp_policy), mode)
        if not self.h:
            raise ValueError("unsupported policy")

    def close(self):
        lib().orc_factory_close(self.h)


class Transformer:
    def __init__(self, kind, fwd: Factory, rev: Factory):
        self.kind = kind
        self.h = lib().orc_transformer_new(kind, fwd.h, rev.h)

    def set_factory(self, f: Factory, forward: bool):
        lib().orc_transformer_set_factory(self.h, f.h, int(forward))

    def close(self):
        lib().orc_transformer_close(self.h)

    def state(self, ssrc: int):
        st = CtxState()
        if not lib().orc_get_state(self.h, ssrc & 0xFFFFFFFF, C.byref(st)):
            return None
        return {k: getattr(st, k) for k, _ in CtxState._fields_}

    def num_contexts(self) -> int:
        return lib().orc_num_contexts(self.h)

    def export_contexts(self) -> dict:
        """{ssrc: state} of every context (orc_export_contexts)."""
        n = lib().orc_export_contexts(self.h, None, None, 0)
        ssrcs = (C.c_uint32 * max(n, 1))()
        states = (CtxState * max(n, 1))()
        lib().orc_export_contexts(self.h, ssrcs, states, n)
        return {int(ssrcs[i]): {k: getattr(states[i], k) for k, _ in CtxState._fields_}
                for i in range(n)}

    def import_context(self, ssrc: int, state: dict, forward: bool) -> None:
        st = CtxState(**{k: state.get(k, 0) for k, _ in CtxState._fields_})
        if lib().orc_set_context_state(self.h, ssrc & 0xFFFFFFFF, int(forward), C.byref(st)) != 0:
            raise ValueError("factory closed")

    def remove_context(self, ssrc: int) -> bool:
        return bool(lib().orc_remove_context(self.h, ssrc & 0xFFFFFFFF))

    def __del__(self):
        try:
            lib().orc_transformer_free(self.h)
        except Exception:
            pass


def process(transformers, reverse: bool, seg: np.ndarray, off: np.ndarray, length: np.ndarray,
            cap: np.ndarray, flags=None, abort_on_error: bool = True):
    """Run one transform()/reverseTransform() bundle in place.

    ``transformers`` is one Transformer (whole bundle) or a sequence with one
    entry per packet.  Returns the status array; ``length`` is updated."""
    n = len(off)
    assert seg.dtype == np.uint8 and seg.flags.c_contiguous
    off = np.ascontiguousarray(off, np.uint32)
    cap = np.ascontiguousarray(cap, np.uint32)
    assert length.dtype == np.uint32 and length.flags.c_contiguous
    fl = np.zeros(n, np.uint32) if flags is None else np.ascontiguousarray(flags, np.uint32)
    status = np.zeros(n, np.int32)
    if isinstance(transformers, Transformer):
        arr = (C.c_void_p * 1)(transformers.h)
        stride = 0
    else:
        arr = (C.c_void_p * n)(*[t.h if t is not None else None for t in transformers])
        stride = 1
    u32 = C.POINTER(C.c_uint32)
    lib().orc_process(arr, stride, int(reverse), seg.ctypes.data_as(C.POINTER(C.c_uint8)),
                      off.ctypes.data_as(u32), length.ctypes.data_as(u32), cap.ctypes.data_as(u32),
                      fl.ctypes.data_as(u32), status.ctypes.data_as(C.POINTER(C.c_int32)),
                      n, int(abort_on_error))
    return status


def tls_export(prf: int, secret: bytes, client_random: bytes, server_random: bytes,
               label: bytes, n: int) -> bytes:
    """RFC 5705 exporter over the TLS PRF (OpenSSL TLS1-PRF; prf 0 = TLS 1.0
    MD5-SHA1, 1 = TLS 1.2 SHA256) -- orc_tls_export."""
    out = C.create_string_buffer(max(n, 1))
    if lib().orc_tls_export(prf, secret, len(secret), client_random, server_random, label, out, n):
        raise RuntimeError("TLS1-PRF failed")
    return out.raw[:n]
