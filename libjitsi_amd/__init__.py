"""libjitsi_amd -- MI355X-native SRTP/SRTCP packet-crypto engine.

A drop-in for the per-packet hot path of libjitsi's SRTPTransformer /
SRTCPTransformer (AES_CM_128_HMAC_SHA1_80/_32, F8_128_HMAC_SHA1_80 and NULL-cipher
profiles):
bundles of packets from many SSRC contexts are protected/unprotected by
hand-written gfx950 kernels behind the C ABI in include/srtp_mi355x.h.
"""
from .srtp import (PacketTransformer, RawPacket, SRTCPTransformer, SRTPAggregator,  # noqa: F401
                   SRTPContextFactory, SRTPDispatcher,
                   SRTPEngine, SRTPPipeline, SRTPPolicy, SRTPTransformer, SRTPTransformException, pack,
                   HostBuffer, host_is_registered, host_register, host_unregister, profile_policies, transform_bundle)
from . import _native  # noqa: F401

__all__ = ["PacketTransformer", "RawPacket", "SRTCPTransformer", "SRTPAggregator", "SRTPContextFactory", "SRTPDispatcher", "SRTPEngine",
           "SRTPPipeline", "SRTPPolicy", "SRTPTransformer", "SRTPTransformException", "pack", "profile_policies",
           "transform_bundle", "host_register", "host_unregister", "host_is_registered", "HostBuffer"]
