"""ctypes binding of the C ABI in include/srtp_mi355x.h (libsrtp_mi355x.so).

The shared library is built in-tree (``libjitsi_amd/csrc/Makefile``, driven by
``__graft_entry__.build()``).  There is no CPU fallback: if the library is
missing or no GPU is visible, engine creation raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SRTP_MI355X_LIB: another in-tree build of the same ABI (diagnostic variants)
LIB_PATH = os.environ.get("SRTP_MI355X_LIB") or os.path.join(_HERE, "libsrtp_mi355x.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "srtp_mi355x.h")

# include/srtp_mi355x.h
NULL_ENCRYPTION, AESCM_ENCRYPTION, AESF8_ENCRYPTION, TWOFISH_ENCRYPTION, TWOFISHF8_ENCRYPTION = range(5)
NULL_AUTHENTICATION, HMACSHA1_AUTHENTICATION = 0, 1
KIND_RTP, KIND_RTCP = 0, 1
(STATUS_OK, STATUS_DROP_REPLAY, STATUS_DROP_AUTH, STATUS_DROP_VERSION, STATUS_DROP_NO_CONTEXT,
 STATUS_ERR_CAPACITY, STATUS_ERR_MALFORMED, STATUS_DROP_INVALID, STATUS_NOT_PROCESSED,
 STATUS_SKIPPED, STATUS_ERR_INTERNAL) = range(11)
STATUS_NAMES = ["OK", "DROP_REPLAY", "DROP_AUTH", "DROP_VERSION", "DROP_NO_CONTEXT",
                "ERR_CAPACITY", "ERR_MALFORMED", "DROP_INVALID", "NOT_PROCESSED", "SKIPPED",
                "ERR_INTERNAL"]
NUM_STATUS = len(STATUS_NAMES)
DEBUG_FORCE_CHAIN_STALL = 0x1
DEBUG_FORCE_WIDE = 0x2  # every bundle on the split path (k_ctr_wide + k_mac_wide)
DEBUG_NO_WIDE = 0x4     # every bundle on the fused kernels
DEBUG_NO_SMALL = 0x8    # bundles of up to 255 packets off k_small (one launch per bundle)
ABI_VERSION = 3
AGG_SEAL_IDLE = 0x1
PKT_FLAG_DISCARD, PKT_FLAG_SILENCE, PKT_FLAG_SKIP = 0x2, 0x4, 0x80000000
RC = {0: "SRTP_OK", -1: "SRTP_EINVAL", -2: "SRTP_ENOMEM", -3: "SRTP_EFULL", -4: "SRTP_EDEVICE",
      -5: "SRTP_EPOLICY", -6: "SRTP_EAGAIN"}
EFULL = -3
EAGAIN = -6

EXPORTED = [
    "srtp_engine_opts_default", "srtp_engine_create", "srtp_engine_destroy",
    "srtp_engine_last_error", "srtp_factory_create", "srtp_factory_close",
    "srtp_transformer_create", "srtp_transformer_set_factory", "srtp_transformer_close",
    "srtp_transform_device", "srtp_transform_host", "srtp_engine_sync",
    "srtp_get_context_state", "srtp_engine_num_contexts", "srtp_engine_set_timing",
    "srtp_engine_read_timing", "srtp_derive_session_keys", "srtp_export_contexts",
    "srtp_set_context_state", "srtp_pipeline_create", "srtp_pipeline_destroy",
    "srtp_pipeline_slot_get", "srtp_pipeline_submit", "srtp_pipeline_wait",
    "srtp_engine_stats", "srtp_engine_stream", "srtp_shard_of", "srtp_dispatch_plan", "srtp_dispatch_create",
    "srtp_dispatch_destroy", "srtp_dispatch_last_error", "srtp_dispatch_num_shards",
    "srtp_dispatch_engine", "srtp_dispatch_factory_create", "srtp_dispatch_factory_close",
    "srtp_dispatch_transformer_create", "srtp_dispatch_transformer_set_factory",
    "srtp_dispatch_transformer_close", "srtp_dispatch_transform_host", "srtp_dispatch_submit_host",
    "srtp_dispatch_wait_host",
    "srtp_dispatch_get_context_state", "srtp_dispatch_set_context_state", "srtp_dispatch_stats",
    "srtp_tls_export_keying_material", "srtp_dtls_profile_keys", "srtp_dtls_transformer_create",
    "srtp_engine_get_opts", "srtp_derive_session_keys_n", "srtp_derive_session_keys_for",
    "srtp_block_encrypt", "srtp_aggregator_opts_default", "srtp_aggregator_create",
    "srtp_aggregator_submit", "srtp_aggregator_flush", "srtp_aggregator_stats",
    "srtp_aggregator_destroy", "srtp_derive_session_keys_auth", "srtp_skein512_mac",
    "srtp_engine_set_debug", "srtp_contexts_save", "srtp_contexts_restore",
    "srtp_dispatch_route", "srtp_aggregator_create_dispatch", "srtp_transformer_info",
    "srtp_rawpacket_batch_create", "srtp_rawpacket_batch_create_dispatch",
    "srtp_rawpacket_batch_destroy", "srtp_rawpacket_transform", "srtp_rawpacket_result",
    "srtp_dispatch_host_times", "srtp_pipeline_submit_ex", "srtp_aggregator_transform",
    "srtp_aggregator_transformer_info", "srtp_rawpacket_transform_one", "srtp_device_count",
    "srtp_host_register", "srtp_host_unregister", "srtp_host_is_registered", "srtp_pipeline_submit_host",
    "srtp_pipeline_submit_gather",
    "srtp_pipeline_create_ex", "srtp_host_alloc", "srtp_host_free",
    "srtp_queue_create", "srtp_queue_submit", "srtp_queue_reap", "srtp_queue_outstanding",
    "srtp_queue_aggregator", "srtp_queue_destroy", "srtp_queue_release", "srtp_packet_may_throw",
    "srtp_rawpacket_batch_set_aggregator", "srtp_rawpacket_submit", "srtp_rawpacket_complete",
    "srtp_pipeline_query",
]
STAGES = ["parse", "sort", "verify", "walk", "protect", "decrypt"]


# Sources that decide what the crypto kernels execute: the key that ties
# committed PMC counters (profiles/pmc_traffic.json) to the build they measured.
KERNEL_SOURCES = ["srtp_kernels.hip", "aes_rounds_asm.inc", "srtp_kernels.h", "srtp_types.h", "engine.cpp"]


def kernel_source_sha16() -> str:
    import hashlib
    h = hashlib.sha256()
    for name in KERNEL_SOURCES:
        with open(os.path.join(_HERE, "csrc", name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


class SrtpError(RuntimeError):
    pass


class Policy(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "enc_type", "enc_key_len", "auth_type", "auth_key_len", "auth_tag_len", "salt_key_len")]


class EngineOpts(C.Structure):
    _fields_ = [("device", C.c_int32), ("check_replay", C.c_int32),
                ("abort_on_error", C.c_int32), ("max_contexts", C.c_uint32),
                ("max_factories", C.c_uint32), ("max_transformers", C.c_uint32),
                ("max_batch", C.c_uint32)]


class CtxState(C.Structure):
    _fields_ = [("roc", C.c_int32), ("s_l", C.c_int32), ("seq_num_set", C.c_int32),
                ("guessed_roc", C.c_int32), ("sent_index", C.c_int32),
                ("received_index", C.c_int32), ("replay_window", C.c_uint64),
                ("key_set", C.c_uint32)]


class Stats(C.Structure):
    """srtp_stats (include/srtp_mi355x.h)"""
    _fields_ = ([("bundles", C.c_uint64), ("packets", C.c_uint64),
                 ("status", C.c_uint64 * NUM_STATUS)] +
                [(n, C.c_uint64) for n in ("roc_rechecks", "repaired", "ctx_overflow", "ctx_live",
                                           "ctx_tombstones", "ctx_slots", "rehashes", "chain_stalls", "long_walked",
                                           "holes", "small_bundles")])

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "status"}
        d["status"] = {STATUS_NAMES[i]: int(self.status[i]) for i in range(NUM_STATUS)}
        return d


class DtlsKeys(C.Structure):
    """srtp_dtls_keys (include/srtp_mi355x.h)"""
    _fields_ = [("srtp", Policy), ("srtcp", Policy), ("key_len", C.c_int32),
                ("salt_len", C.c_int32), ("keying_material_len", C.c_int32),
                ("client_key", C.c_uint8 * 16), ("server_key", C.c_uint8 * 16),
                ("client_salt", C.c_uint8 * 14), ("server_salt", C.c_uint8 * 14)]


class AggregatorOpts(C.Structure):
    _fields_ = [("max_packets", C.c_uint32), ("max_bytes", C.c_size_t), ("deadline_us", C.c_uint32),
                ("depth", C.c_int32), ("flags", C.c_uint32)]


class Completion(C.Structure):
    """srtp_completion (include/srtp_mi355x.h)"""
    _fields_ = [("cookie", C.c_uint64), ("status", C.c_int32), ("len", C.c_uint32),
                ("in_len", C.c_uint32), ("reverse", C.c_int32), ("tid", C.c_int32),
                ("data", C.POINTER(C.c_uint8))]


AGG_CB = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_int32, C.POINTER(C.c_uint8), C.c_uint32)


class PipelineSlot(C.Structure):
    _fields_ = [("seg", C.c_void_p), ("seg_cap", C.c_size_t), ("off", C.c_void_p),
                ("len", C.c_void_p), ("cap", C.c_void_p), ("flags", C.c_void_p),
                ("tids", C.c_void_p), ("status", C.c_void_p), ("max_packets", C.c_uint32)]


_lib = None


def lib() -> C.CDLL:
    """Load libsrtp_mi355x.so, failing loudly when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SrtpError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; "
                        f"g.build()'` (make -C libjitsi_amd/csrc)")
    L = C.CDLL(LIB_PATH)
    vp, i32, u32 = C.c_void_p, C.c_int32, C.c_uint32
    pi32, pu32, pu8 = C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)
    L.srtp_engine_opts_default.argtypes = [C.POINTER(EngineOpts)]
    L.srtp_engine_create.argtypes = [C.POINTER(EngineOpts), C.POINTER(vp)]
    L.srtp_engine_destroy.argtypes = [vp]
    L.srtp_engine_destroy.restype = None
    L.srtp_engine_last_error.argtypes = [vp]
    L.srtp_engine_last_error.restype = C.c_char_p
    L.srtp_factory_create.argtypes = [vp, i32, pu8, i32, pu8, i32, C.POINTER(Policy),
                                      C.POINTER(Policy), pi32]
    L.srtp_factory_close.argtypes = [vp, i32]
    L.srtp_transformer_create.argtypes = [vp, i32, i32, i32, pi32]
    L.srtp_transformer_set_factory.argtypes = [vp, i32, i32, i32]
    L.srtp_transformer_close.argtypes = [vp, i32]
    L.srtp_transform_device.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, u32, vp]
    L.srtp_transform_host.argtypes = [vp, i32, vp, i32, vp, C.c_size_t, vp, vp, vp, vp, vp, u32]
    L.srtp_engine_sync.argtypes = [vp, vp]
    L.srtp_get_context_state.argtypes = [vp, i32, u32, C.POINTER(CtxState)]
    L.srtp_engine_num_contexts.argtypes = [vp]
    L.srtp_engine_num_contexts.restype = C.c_int64
    L.srtp_engine_set_timing.argtypes = [vp, i32]
    L.srtp_engine_set_debug.argtypes = [vp, u32]
    L.srtp_engine_read_timing.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]
    L.srtp_derive_session_keys.argtypes = [pu8, pu8, i32, pu8, pu8, pu8]
    L.srtp_derive_session_keys_n.argtypes = [C.c_char_p, i32, C.c_char_p, i32, pu8, pu8, pu8]
    L.srtp_derive_session_keys_for.argtypes = [i32, C.c_char_p, i32, C.c_char_p, i32, pu8, pu8, pu8]
    L.srtp_block_encrypt.argtypes = [i32, C.c_char_p, i32, C.c_char_p, pu8]
    L.srtp_derive_session_keys_auth.argtypes = [i32, C.c_char_p, i32, C.c_char_p, i32, pu8, pu8, i32, pu8]
    L.srtp_skein512_mac.argtypes = [C.c_char_p, i32, i32, C.c_char_p, C.c_size_t, pu8]
    L.srtp_export_contexts.argtypes = [vp, i32, pu32, C.POINTER(CtxState), u32, pu32]
    L.srtp_set_context_state.argtypes = [vp, i32, u32, i32, C.POINTER(CtxState)]
    L.srtp_contexts_save.argtypes = [vp, u32, vp, vp, vp, vp]
    L.srtp_transformer_info.argtypes = [vp, i32, pi32, pi32]
    L.srtp_rawpacket_batch_create.argtypes = [vp, C.POINTER(vp)]
    L.srtp_rawpacket_batch_create_dispatch.argtypes = [vp, C.POINTER(vp)]
    L.srtp_rawpacket_batch_destroy.argtypes = [vp]
    L.srtp_rawpacket_batch_destroy.restype = None
    L.srtp_rawpacket_transform.argtypes = [vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, vp, u32, pi32]
    L.srtp_rawpacket_result.argtypes = [vp, u32, C.POINTER(C.POINTER(C.c_uint8)), pu32]
    L.srtp_contexts_restore.argtypes = [vp, u32, vp, vp, vp, vp]
    L.srtp_pipeline_create.argtypes = [vp, u32, C.c_size_t, i32, C.POINTER(vp)]
    L.srtp_pipeline_destroy.argtypes = [vp]
    L.srtp_pipeline_destroy.restype = None
    L.srtp_pipeline_slot_get.argtypes = [vp, i32, C.POINTER(PipelineSlot)]
    L.srtp_pipeline_submit.argtypes = [vp, i32, i32, i32, i32, i32, u32, C.c_size_t]
    L.srtp_pipeline_wait.argtypes = [vp, i32]
    L.srtp_pipeline_query.argtypes = [vp, i32]
    L.srtp_pipeline_submit_ex.argtypes = [vp, i32, i32, i32, i32, i32, u32, C.c_size_t, i32]
    L.srtp_aggregator_transform.argtypes = [vp, i32, i32, vp, u32, u32, u32, u32, vp, pi32, pu32]
    L.srtp_aggregator_transformer_info.argtypes = [vp, i32, pi32, pi32]
    L.srtp_rawpacket_transform_one.argtypes = [vp, i32, i32, vp, u32, u32, pu32, u32, pi32, pu32, vp, u32]
    L.srtp_pipeline_create_ex.argtypes = [vp, u32, C.c_size_t, i32, u32, C.POINTER(vp)]
    L.srtp_host_register.argtypes = [vp, C.c_size_t]
    L.srtp_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
    L.srtp_host_free.argtypes = [vp]
    L.srtp_host_unregister.argtypes = [vp]
    L.srtp_host_is_registered.argtypes = [vp, C.c_size_t]
    L.srtp_host_is_registered.restype = i32
    L.srtp_pipeline_submit_host.argtypes = [vp, i32, i32, i32, i32, i32, u32, C.c_size_t, i32, vp]
    L.srtp_pipeline_submit_gather.argtypes = [vp, i32, i32, i32, i32, i32, u32, C.c_size_t, i32, vp, C.c_size_t, vp]
    L.srtp_device_count.argtypes = []
    L.srtp_device_count.restype = i32
    L.srtp_engine_stats.argtypes = [vp, C.POINTER(Stats)]
    L.srtp_engine_get_opts.argtypes = [vp, C.POINTER(EngineOpts)]
    L.srtp_aggregator_opts_default.argtypes = [C.POINTER(AggregatorOpts)]
    L.srtp_aggregator_create.argtypes = [vp, C.POINTER(AggregatorOpts), AGG_CB, vp, C.POINTER(vp)]
    L.srtp_aggregator_create_dispatch.argtypes = [vp, C.POINTER(AggregatorOpts), AGG_CB, vp,
                                                   C.POINTER(vp)]
    L.srtp_dispatch_route.argtypes = [vp, i32, C.c_char_p, u32]
    L.srtp_dispatch_route.restype = i32
    L.srtp_aggregator_submit.argtypes = [vp, i32, i32, C.c_char_p, u32, u32, C.c_uint64]
    L.srtp_aggregator_flush.argtypes = [vp]
    L.srtp_aggregator_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]
    L.srtp_aggregator_destroy.argtypes = [vp]
    L.srtp_aggregator_destroy.restype = None
    L.srtp_tls_export_keying_material.argtypes = [i32, C.c_char_p, i32, C.c_char_p, C.c_char_p,
                                                  C.c_char_p, vp, i32]
    L.srtp_dtls_profile_keys.argtypes = [i32, C.c_char_p, i32, C.POINTER(DtlsKeys)]
    L.srtp_dtls_transformer_create.argtypes = [vp, i32, i32, i32, C.c_char_p, i32, pi32, pi32]
    L.srtp_engine_stream.argtypes = [vp]
    L.srtp_engine_stream.restype = vp
    L.srtp_shard_of.argtypes = [u32, i32]
    L.srtp_shard_of.restype = i32
    L.srtp_dispatch_plan.argtypes = [i32, i32, i32, vp, i32, u32, vp, i32, vp, C.c_size_t, vp, vp, vp,
                                     vp, u32, vp, vp]
    L.srtp_dispatch_plan.restype = i32
    L.srtp_dispatch_create.argtypes = [vp, i32, C.POINTER(EngineOpts), C.POINTER(vp)]
    L.srtp_dispatch_destroy.argtypes = [vp]
    L.srtp_dispatch_destroy.restype = None
    L.srtp_dispatch_last_error.argtypes = [vp]
    L.srtp_dispatch_last_error.restype = C.c_char_p
    L.srtp_dispatch_num_shards.argtypes = [vp]
    L.srtp_dispatch_num_shards.restype = i32
    L.srtp_dispatch_engine.argtypes = [vp, i32]
    L.srtp_dispatch_engine.restype = vp
    L.srtp_dispatch_factory_create.argtypes = [vp, i32, pu8, i32, pu8, i32, C.POINTER(Policy),
                                               C.POINTER(Policy), pi32]
    L.srtp_dispatch_factory_close.argtypes = [vp, i32]
    L.srtp_dispatch_transformer_create.argtypes = [vp, i32, i32, i32, pi32]
    L.srtp_dispatch_transformer_set_factory.argtypes = [vp, i32, i32, i32]
    L.srtp_dispatch_transformer_close.argtypes = [vp, i32]
    L.srtp_dispatch_transform_host.argtypes = [vp, i32, vp, i32, vp, C.c_size_t, vp, vp, vp, vp, vp,
                                               u32]
    L.srtp_dispatch_submit_host.argtypes = [vp, i32, vp, i32, vp, C.c_size_t, vp, vp, vp, vp, vp, u32,
                                            C.POINTER(C.c_uint64)]
    L.srtp_dispatch_wait_host.argtypes = [vp, C.c_uint64]
    L.srtp_dispatch_get_context_state.argtypes = [vp, i32, u32, C.POINTER(CtxState)]
    L.srtp_dispatch_set_context_state.argtypes = [vp, i32, u32, i32, C.POINTER(CtxState)]
    L.srtp_dispatch_stats.argtypes = [vp, C.POINTER(Stats)]
    L.srtp_dispatch_host_times.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.srtp_queue_create.argtypes = [vp, u32, C.POINTER(vp)]
    L.srtp_queue_submit.argtypes = [vp, i32, i32, vp, u32, u32, u32, u32, C.c_uint64]
    L.srtp_queue_reap.argtypes = [vp, C.POINTER(Completion), u32, i32]
    L.srtp_queue_outstanding.argtypes = [vp]
    L.srtp_queue_outstanding.restype = i32
    L.srtp_queue_aggregator.argtypes = [vp]
    L.srtp_queue_aggregator.restype = vp
    L.srtp_queue_release.argtypes = [vp]
    L.srtp_queue_release.restype = None
    L.srtp_queue_destroy.argtypes = [vp]
    L.srtp_queue_destroy.restype = None
    L.srtp_packet_may_throw.argtypes = [i32, i32, C.c_char_p, u32, u32, u32, u32]
    L.srtp_packet_may_throw.restype = i32
    L.srtp_rawpacket_batch_set_aggregator.argtypes = [vp, vp]
    L.srtp_rawpacket_submit.argtypes = [vp, i32, i32, vp, u32, u32, u32, u32, C.c_uint64]
    L.srtp_rawpacket_complete.argtypes = [vp, C.POINTER(Completion), u32, pu32, pu32]
    _lib = L
    return L


def check(rc: int, engine=None, what: str = "", dispatch=None) -> int:
    if rc < 0:
        msg = RC.get(rc, str(rc))
        if engine or dispatch:
            detail = (lib().srtp_dispatch_last_error(dispatch) if dispatch
                      else lib().srtp_engine_last_error(engine))
            if detail:
                msg += ": " + detail.decode(errors="replace")
        raise SrtpError(f"{what}: {msg}")
    return rc
