"""DTLS-SRTP keying: from a finished handshake to SRTP / SRTCP transformers.

Mirrors DtlsPacketTransformer.initializeSRTPTransformer
(transform/dtls/DtlsPacketTransformer.java:549-690) over the engine's C ABI
(libjitsi_amd/csrc/dtls_keys.cpp): the negotiated protection profile's
policies (:574-612), the RFC 5705 export of 2 * (key + salt) bytes with the
label "EXTRACTOR-dtls_srtp" (:614-617), the client key | server key | client
salt | server salt split (:618-638), and the client / server factories with the
forward factory being this side's own (:639-690).  The DTLS handshake itself
(BouncyCastle's DTLSClientProtocol / DTLSServerProtocol) is out of scope
(SURVEY.md 8): the caller supplies its master secret and randoms.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

from . import _native as N
from .srtp import SRTCPTransformer, SRTPContextFactory, SRTPPolicy, SRTPTransformer

# SRTPProtectionProfile ids (RFC 5764 4.1.2), the four DtlsPacketTransformer handles
SRTP_AES128_CM_HMAC_SHA1_80 = 0x0001
SRTP_AES128_CM_HMAC_SHA1_32 = 0x0002
SRTP_NULL_HMAC_SHA1_80 = 0x0005
SRTP_NULL_HMAC_SHA1_32 = 0x0006
PROFILES = (SRTP_AES128_CM_HMAC_SHA1_80, SRTP_AES128_CM_HMAC_SHA1_32, SRTP_NULL_HMAC_SHA1_80,
            SRTP_NULL_HMAC_SHA1_32)
# TLS PRF of the negotiated version: DTLS 1.0 (the reference's offer,
# TlsClientImpl.java:148-155) or DTLS 1.2
PRF_TLS10, PRF_SHA256 = 0, 1
EXPORTER_LABEL = b"EXTRACTOR-dtls_srtp"  # ExporterLabel.dtls_srtp


def export_keying_material(master_secret: bytes, client_random: bytes, server_random: bytes,
                           length: int, label: bytes = EXPORTER_LABEL,
                           prf: int = PRF_TLS10) -> bytes:
    """TlsContext.exportKeyingMaterial(label, null, length) (RFC 5705, no
    context value) for a session with this master secret and randoms."""
    assert len(client_random) == 32 and len(server_random) == 32
    out = (C.c_uint8 * max(length, 1))()
    N.check(N.lib().srtp_tls_export_keying_material(prf, bytes(master_secret), len(master_secret),
                                                    bytes(client_random), bytes(server_random),
                                                    bytes(label), out, length),
            None, "exportKeyingMaterial")
    return bytes(out)[:length]


def profile_keys(profile: int, keying_material: Optional[bytes] = None) -> dict:
    """Policies and split keys of a protection profile (:574-638).  Without
    keying material: only the policies and keying_material_len."""
    k = N.DtlsKeys()
    km = None if keying_material is None else bytes(keying_material)
    rc = N.lib().srtp_dtls_profile_keys(profile, km, 0 if km is None else len(km), C.byref(k))
    if rc == -5:
        raise ValueError("srtpProtectionProfile")  # the reference's IllegalArgumentException
    N.check(rc, None, "profile_keys")
    pol = [SRTPPolicy(p.enc_type, p.enc_key_len, p.auth_type, p.auth_key_len, p.auth_tag_len,
                      p.salt_key_len) for p in (k.srtp, k.srtcp)]
    d = {"srtpPolicy": pol[0], "srtcpPolicy": pol[1],
         "keying_material_len": k.keying_material_len}
    if km is not None:
        d.update(client_key=bytes(k.client_key)[:k.key_len],
                 server_key=bytes(k.server_key)[:k.key_len],
                 client_salt=bytes(k.client_salt)[:k.salt_len],
                 server_salt=bytes(k.server_salt)[:k.salt_len])
    return d


def initialize_srtp_transformer(profile: int, is_client: bool, rtcp: bool,
                                keying_material: bytes, engine=None):
    """DtlsPacketTransformer.initializeSRTPTransformer(profile, tlsContext)
    given the exported keying material: an SRTPTransformer (rtcp False) or
    SRTCPTransformer whose forward factory is this side's."""
    k = profile_keys(profile, keying_material)
    if not k["client_key"]:  # NULL-cipher profiles: no master key
        raise ValueError("profile exports no master key; the reference fails deriving keys")
    sp, cp = k["srtpPolicy"], k["srtcpPolicy"]
    client = SRTPContextFactory(is_client, k["client_key"], k["client_salt"], sp, cp, engine=engine)
    server = SRTPContextFactory(not is_client, k["server_key"], k["server_salt"], sp, cp,
                                engine=engine)
    fwd, rev = (client, server) if is_client else (server, client)
    return (SRTCPTransformer if rtcp else SRTPTransformer)(fwd, rev)
