"""CPU: pin the oracle (and the engine's host-side key derivation) to published
known-answer vectors.  The reference ships no SRTP test vectors, so
parity is pinned by the standards' KATs and libsrtp's published SRTP/SRTCP
vectors for the same profile and RFC 3711 B.3 master key."""
import hashlib
import hmac

import numpy as np
import pytest

B3_KEY = bytes.fromhex("E1F97A0D3E018BE0D64FA32C06DE4139")
B3_SALT = bytes.fromhex("0EC675AD498AFEEBB6960B3AABE6")


def test_fips197_c1(oracle):
    out = oracle.aes128_block(bytes(range(16)), bytes.fromhex("00112233445566778899aabbccddeeff"))
    assert out.hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


RFC2202 = [
    (b"\x0b" * 20, b"Hi There", "b617318655057264e28bc0b6fb378c8ef146be00"),
    (b"Jefe", b"what do ya want for nothing?", "effcdf6ae5eb2fa2d27416d5f184df9c259a7c79"),
    (b"\xaa" * 20, b"\xdd" * 50, "125d7342b9ac11cd91a39af48aa17b4f63f175d3"),
    (bytes(range(1, 26)), b"\xcd" * 50, "4c9007f4026250c6bc8414f9bf50c86c2d7235da"),
    (b"\x0c" * 20, b"Test With Truncation", "4c1a03424b55e07fe7f27be1d58bb9324a9a5a04"),
    (b"\xaa" * 80, b"Test Using Larger Than Block-Size Key - Hash Key First",
     "aa4ae5e15272d00e95705637ce8a3b55ed402112"),
    (b"\xaa" * 80, b"Test Using Larger Than Block-Size Key and Larger Than One Block-Size Data",
     "e8e99d0f45237d786d6bbaa7965c7808bbff1a91"),
]


@pytest.mark.parametrize("key,msg,mac", RFC2202)
def test_rfc2202_hmac_sha1(oracle, key, msg, mac):
    assert oracle.hmac_sha1(key, msg).hex() == mac
    assert hmac.new(key, msg, hashlib.sha1).hexdigest() == mac


def test_rfc3711_b2_keystream(oracle):
    """AES-CM keystream, RFC 3711 App. B.2 (counter in IV bytes 14-15)."""
    key = bytes.fromhex("2B7E151628AED2A6ABF7158809CF4F3C")
    iv = bytearray.fromhex("F0F1F2F3F4F5F6F7F8F9FAFBFCFD0000")
    ks = b""
    for j in range(3):
        iv[14], iv[15] = j >> 8, j & 0xFF
        ks += oracle.aes128_block(key, bytes(iv))
    assert ks.hex().upper() == ("E03EAD0935C95E80E166B16DD92B4EB4"
                                "D23513162B02D0F72A43A2FE4A5F97AB"
                                "41E95B3BB0A2E8DD477901E4FCA894C0")


# RFC 3711 App. B.1: AES-f8 (IV' = E(k_e ^ (k_s || 0x55..), IV), chained S(j))
B1_KEY = bytes.fromhex("234829008467be186c3de14aae72d62c")
B1_SALT = bytes.fromhex("32f2870d")
B1_IV = bytes.fromhex("006e5cba50681de55c621599d462564a")  # 0 || RTP header[1..11] || ROC
B1_PT = b"pseudorandomness is the next best thing"
B1_CT = ("019ce7a26e7854014a6366aa95d4eefd" "1ad4172a14f9faf455b7f1d4b62bd08f" "562c0eef7c4802")


def test_rfc3711_b1_aes_f8(oracle):
    mask = bytes(k ^ (B1_SALT[i] if i < 4 else 0x55) for i, k in enumerate(B1_KEY))
    assert oracle.aes128_block(mask, B1_IV).hex() == "595b699bbd3bc0df26062093c1ad8f73"  # IV'
    assert oracle.aes_f8(B1_KEY, B1_SALT, B1_IV, B1_PT).hex() == B1_CT
    # F8 is an involution on the same IV
    assert oracle.aes_f8(B1_KEY, B1_SALT, B1_IV, bytes.fromhex(B1_CT)) == B1_PT


def test_rfc3711_b1_aes_f8_pyref():
    from oracle import pyref as R
    buf = bytearray(B1_PT)
    R.f8_process(R.expand_key(B1_KEY), R.expand_key(R.f8_key_mask(B1_KEY, B1_SALT)), buf, 0,
                 len(buf), B1_IV)
    assert buf.hex() == B1_CT


def test_rfc3711_b3_key_derivation(oracle):
    enc, auth, salt = oracle.derive_keys(B3_KEY, B3_SALT)
    assert enc.hex().upper() == "C61E7A93744F39EE10734AFE3FF7A087"
    assert salt.hex().upper() == "30CBBC08863D8C85D49DB34A9AE1"
    assert auth.hex().upper() == "CEBE321F6FF7716B6FD4AB49AF256A156D38BAA4"


def test_engine_host_kdf_matches_rfc3711_b3():
    """The product's own host-side PRF (no GPU needed)."""
    from libjitsi_amd.srtp import derive_session_keys
    enc, auth, salt = derive_session_keys(B3_KEY, B3_SALT)
    assert enc.hex().upper() == "C61E7A93744F39EE10734AFE3FF7A087"
    assert salt.hex().upper() == "30CBBC08863D8C85D49DB34A9AE1"
    assert auth.hex().upper() == "CEBE321F6FF7716B6FD4AB49AF256A156D38BAA4"


def test_engine_host_kdf_matches_oracle_srtcp(oracle):
    from libjitsi_amd.srtp import derive_session_keys
    rng = np.random.default_rng(5)
    for _ in range(20):
        k, s = rng.bytes(16), rng.bytes(14)
        for rtcp in (False, True):
            assert derive_session_keys(k, s, rtcp) == oracle.derive_keys(k, s, rtcp)


def _one(oracle, kind, pkts, warm=0):
    pol = oracle.Policy(1, 16, 1, 20, 10, 14)
    f = oracle.Factory(True, B3_KEY, B3_SALT, pol, pol)
    t = oracle.Transformer(kind, f, f)
    seg = np.zeros(64 * len(pkts), np.uint8)
    for i, p in enumerate(pkts):
        seg[64 * i:64 * i + len(p)] = np.frombuffer(p, np.uint8)
    ln = np.array([len(p) for p in pkts], np.uint32)
    st = oracle.process(t, False, seg, np.arange(len(pkts)) * 64, ln, np.full(len(pkts), 64))
    return seg, ln, st


def test_libsrtp_srtp_vector(oracle):
    """libsrtp test/srtp_driver.c srtp_validate (AES_CM_128_HMAC_SHA1_80)."""
    seg, ln, st = _one(oracle, oracle.KIND_RTP,
                       [bytes.fromhex("800f1234decafbadcafebabe") + b"\xab" * 16])
    assert st[0] == 0 and ln[0] == 38
    assert seg[:38].tobytes().hex() == (
        "800f1234decafbadcafebabe4e55dc4ce79978d88ca4d215949d2402b78d6acc99ea179b8dbb")


def test_libsrtp_srtcp_vector(oracle):
    """libsrtp srtcp vector (SRTCP index 1: the second packet of the context)."""
    p = bytes.fromhex("81c8000bcafebabe") + b"\xab" * 16
    seg, ln, st = _one(oracle, oracle.KIND_RTCP, [p, p])
    assert (st == 0).all() and ln[1] == 38
    assert seg[64:64 + 38].tobytes().hex() == (
        "81c8000bcafebabe7128035be487b9bdbef89041f977a5a880000001993e08cd54d6c1230798")


def test_abi_exports_every_declared_symbol():
    """libsrtp_mi355x.so loads on a CPU-only host and exports every function
    include/srtp_mi355x.h declares."""
    import ctypes
    import re
    from libjitsi_amd import _native
    decl = re.findall(r"^\s*(?:int|void|void \*|int32_t|int64_t|const char \*|srtp_\w+ \*)\s*\*?(srtp_\w+)\(",
                      open(_native.HEADER_PATH).read(), re.M)
    assert set(decl) == set(_native.EXPORTED)
    lib = ctypes.CDLL(_native.LIB_PATH)
    for sym in decl:
        assert hasattr(lib, sym), sym
