"""Independent pure-Python restatement of the reference SRTP/SRTCP path.

TEST INFRASTRUCTURE ONLY -- a second oracle used to cross-check the C oracle
(oracle/srtp_oracle.c) on small bundles.  It shares no code with it: AES-128 is
implemented here from FIPS-197, HMAC-SHA1 comes from Python's hashlib/hmac,
Skein-512 is restated here from the Skein 1.3 paper,
and the context state machine is restated directly from

  srtp/SRTPCryptoContext.java:237-744, srtp/SRTCPCryptoContext.java:106-451,
  srtp/SRTPCipherCTR.java:68-121, srtp/SRTPCipherF8.java:66-183,
  srtp/BaseSRTPCryptoContext.java:269-278,
  srtp/SRTPTransformer.java:100-219, srtp/SRTCPTransformer.java:92-207,
  nm/RawPacket.java, tf/SinglePacketTransformer.java:121-216

with Java int/long arithmetic emulated by explicit masking.
"""
from __future__ import annotations

import hashlib
import hmac

M32, M64 = 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF


def i32(x):
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


def i64(x):
    x &= M64
    return x - (1 << 64) if x & (1 << 63) else x


def lshl(v, n):  # Java long << n
    return i64(v << (n & 63))


def ishl1(n):  # Java int 1 << n
    return i32(1 << (n & 31))


# ---------------------------------------------------------------- AES-128
def _xt(a):
    return ((a << 1) ^ (0x1B if a & 0x80 else 0)) & 0xFF


def _sbox():
    # S-box via log/antilog tables over generator 3
    exp, log = [0] * 256, [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x ^= _xt(x)
    s = []
    for a in range(256):
        inv = 0 if a == 0 else exp[(255 - log[a]) % 255]
        b = inv
        r = inv
        for _ in range(4):
            b = ((b << 1) | (b >> 7)) & 0xFF
            r ^= b
        s.append(r ^ 0x63)
    return s


SBOX = _sbox()


def expand_key(key: bytes):
    w = [list(key[4 * i:4 * i + 4]) for i in range(4)]
    rcon = 1
    for i in range(4, 44):
        t = list(w[i - 1])
        if i % 4 == 0:
            t = [SBOX[t[1]] ^ rcon, SBOX[t[2]], SBOX[t[3]], SBOX[t[0]]]
            rcon = _xt(rcon)
        w.append([w[i - 4][k] ^ t[k] for k in range(4)])
    return [bytes(sum(w[4 * r:4 * r + 4], [])) for r in range(11)]


def aes_block(rks, block: bytes) -> bytes:
    s = [b ^ k for b, k in zip(block, rks[0])]
    for r in range(1, 11):
        s = [SBOX[s[4 * ((c + row) % 4) + row]] for c in range(4) for row in range(4)]
        if r < 10:
            t = []
            for c in range(4):
                a0, a1, a2, a3 = s[4 * c:4 * c + 4]
                t += [_xt(a0) ^ _xt(a1) ^ a1 ^ a2 ^ a3, a0 ^ _xt(a1) ^ _xt(a2) ^ a2 ^ a3,
                      a0 ^ a1 ^ _xt(a2) ^ _xt(a3) ^ a3, _xt(a0) ^ a0 ^ a1 ^ a2 ^ _xt(a3)]
            s = t
        s = [b ^ k for b, k in zip(s, rks[r])]
    return bytes(s)


class Throw(Exception):
    """A Java exception escaping the context method."""


def cipher_stream(rks, length, iv):
    """SRTPCipherCTR.getCipherStream :68-92 (Java division/remainder)."""
    ctr_end = int(length / 16) if length >= 0 else -((-length) // 16)
    out = bytearray()
    inb = bytearray(iv[:14]) + b"\0\0"
    ctr = 0
    while ctr < ctr_end:
        inb[14], inb[15] = (ctr >> 8) & 0xFF, ctr & 0xFF
        out += aes_block(rks, bytes(inb))
        ctr += 1
    inb[14], inb[15] = (ctr >> 8) & 0xFF, ctr & 0xFF
    tail = aes_block(rks, bytes(inb))
    rem = length - 16 * ctr_end  # Java %: sign of the dividend
    if rem < 0:
        raise Throw("arraycopy")
    return bytes(out) + tail[:rem]


def ctr_process(rks, buf: bytearray, buflen, off, length, iv):
    """SRTPCipherCTR.process :94-121 on a buffer of buflen bytes."""
    if off + length > buflen:
        return
    ks = cipher_stream(rks, length, iv)
    for i in range(length):
        if i + off < 0:
            raise Throw("AIOOBE")
        buf[i + off] ^= ks[i]


def f8_process(rks, f8rks, buf: bytearray, off, length, iv):
    """SRTPCipherF8.process :97-128 / processBlock :145-183: IV' = E(k_e ^ m, IV),
    S(j) = E(k_e, IV' ^ S(j-1) ^ j), S(-1) = 0, j big-endian in bytes 12..15."""
    ivp = aes_block(f8rks, bytes(iv))
    s = bytes(16)
    j = pos = 0
    while pos < length:
        n = min(16, length - pos)
        x = bytearray(a ^ b for a, b in zip(s, ivp))
        for k in range(4):
            x[12 + k] ^= (j >> (24 - 8 * k)) & 0xFF
        s = aes_block(rks, bytes(x))
        j += 1
        if off < 0:
            raise Throw("AIOOBE")
        for i in range(n):
            buf[off + pos + i] ^= s[i]
        pos += n


def f8_key_mask(key, salt):
    """SRTPCipherF8.deriveForIV :66-95: key ^ (salt || 0x55..)."""
    return bytes(k ^ (salt[i] if i < len(salt) else 0x55) for i, k in enumerate(key))


# ---------------------------------------------------------------- Skein-512
# Skein 1.3 (Threefish-512 + UBI), restated here independently of oracle/skein.c
# for SKEIN_AUTHENTICATION (BaseSRTPCryptoContext.java:244-248).
_SK_R = ((46, 36, 19, 37), (33, 27, 14, 42), (17, 49, 36, 39), (44, 9, 54, 56),
         (39, 30, 34, 24), (13, 50, 10, 17), (25, 29, 39, 43), (8, 35, 56, 22))
_SK_PI = (2, 1, 4, 7, 6, 5, 0, 3)


def threefish512(key, tweak, words):
    k = list(key) + [0x1BD11BDAA9FC1A22]
    for w in key:
        k[8] ^= w
    t = (tweak[0], tweak[1], tweak[0] ^ tweak[1])

    def subkey(s):
        sk = [k[(s + i) % 9] for i in range(8)]
        sk[5] += t[s % 3]
        sk[6] += t[(s + 1) % 3]
        sk[7] += s
        return [x & M64 for x in sk]

    v = list(words)
    for d in range(72):
        if d % 4 == 0:
            v = [(a + b) & M64 for a, b in zip(v, subkey(d // 4))]
        e = []
        for j in range(4):
            x0 = (v[2 * j] + v[2 * j + 1]) & M64
            r = _SK_R[d % 8][j]
            x1 = (((v[2 * j + 1] << r) | (v[2 * j + 1] >> (64 - r))) & M64) ^ x0
            e += [x0, x1]
        v = [e[_SK_PI[i]] for i in range(8)]
    return [(a + b) & M64 for a, b in zip(v, subkey(18))]


def _ubi(g, msg: bytes, typ: int):
    n = len(msg)
    padded = msg + bytes(-n % 64 if n else 64)
    for i in range(0, len(padded), 64):
        blk = [int.from_bytes(padded[i + 8 * w:i + 8 * w + 8], "little") for w in range(8)]
        pos = min(i + 64, n)
        t1 = (typ << 56) | ((1 << 62) if i == 0 else 0) | ((1 << 63) if i + 64 >= len(padded) else 0)
        c = threefish512(g, (pos, t1), blk)
        g = [a ^ b for a, b in zip(c, blk)]
    return g


def skein512_mac(key: bytes, msg: bytes, out_bits: int) -> bytes:
    g = [0] * 8
    if key:
        g = _ubi(g, key, 0)
    cfg = b"SHA3" + (1).to_bytes(2, "little") + bytes(2) + out_bits.to_bytes(8, "little") + bytes(16)
    g = _ubi(g, cfg, 4)
    g = _ubi(g, msg, 48)
    g = _ubi(g, bytes(8), 63)
    return b"".join(w.to_bytes(8, "little") for w in g)[:(out_bits + 7) // 8]


def derive(mk, ms, rtcp, auth_len=20):
    """RFC 3711 4.3 with kdr = 0 (computeIv label << 48 -> byte 7)."""
    rks = expand_key(mk)
    out = []
    for lab, n in zip((3, 4, 5) if rtcp else (0, 1, 2), (16, auth_len, 14)):
        iv = bytearray(ms[:14]) + b"\0\0"
        iv[7] ^= lab
        out.append(cipher_stream(rks, n, bytes(iv)))
    return out


# ---------------------------------------------------------------- contexts
class Ctx:
    def __init__(self, policy, mk, ms, rtcp):
        self.policy = policy  # (enc, enc_len, auth, auth_len, tag, salt_len)
        enc, auth, salt = derive(mk, ms, rtcp, policy[3] if policy[2] == 2 else 20)
        self.rks = expand_key(enc)
        self.f8rks = expand_key(f8_key_mask(enc, salt)) if policy[0] == 2 else None
        self.auth = auth
        self.salt = salt
        self.roc = self.s_l = self.guessed = 0
        self.seq_set = False
        self.sent = self.recv = 0
        self.window = 0

    def mac(self, data: bytes, roc: int) -> bytes:
        if self.policy[2] == 2:  # SkeinMac, tag_len * 8 output bits (SRTPCryptoContext.java:421-428)
            return skein512_mac(self.auth, data + (roc & M32).to_bytes(4, "big"), 8 * self.policy[4])
        return hmac.new(self.auth, data + (roc & M32).to_bytes(4, "big"), hashlib.sha1).digest()


class Factory:
    def __init__(self, sender, mk, ms, srtp, srtcp):
        self.mk, self.ms, self.srtp, self.srtcp, self.closed = mk, ms, srtp, srtcp, False

    def close(self):
        self.closed = True


class Transformer:
    def __init__(self, kind, fwd, rev):
        self.kind, self.fwd, self.rev, self.ctx = kind, fwd, rev, {}

    def set_factory(self, f, forward):
        cur = self.fwd if forward else self.rev
        if cur is not None and cur is not f:
            cur.close()
        if forward:
            self.fwd = f
        else:
            self.rev = f

    def close(self):
        self.fwd.close()
        if self.rev is not self.fwd:
            self.rev.close()
        self.ctx = {}

    def get(self, ssrc, f):
        c = self.ctx.get(ssrc)
        if c is None and f is not None and not f.closed:
            rtcp = self.kind == 1
            c = Ctx(f.srtcp if rtcp else f.srtp, f.mk, f.ms, rtcp)
            self.ctx[ssrc] = c
        return c


CHECK_REPLAY = [True]


def header_len(buf, cap):
    cc = buf[0] & 0x0F
    h = 12 + 4 * cc
    if buf[0] & 0x10:
        i = 12 + 4 * cc + 2
        if i + 1 >= cap:
            raise Throw("ext")
        hi = buf[i] - 256 if buf[i] >= 128 else buf[i]
        h += 4 + ((hi * 256) | buf[i + 1]) * 4
    return h


def guess(c, seq):
    if c.s_l < 32768:
        c.guessed = i32(c.roc - 1) if seq - c.s_l > 32768 else c.roc
    else:
        c.guessed = i32(c.roc + 1) if c.s_l - 32768 > seq else c.roc
    return lshl(c.guessed, 16) | seq


def replay_ok(c, gi):
    if not CHECK_REPLAY[0]:
        return True
    delta = gi - (lshl(c.roc, 16) | c.s_l)
    if delta > 0:
        return True
    if -delta > 64:
        return False
    return not ((c.window & M64) >> ((-delta) & 63)) & 1


def update(c, seq, gi):
    delta = gi - (lshl(c.roc, 16) | c.s_l)
    if delta > 0:
        c.window = lshl(c.window, delta) | 1
    else:
        c.window = i64(c.window | ishl1(-delta))
    if c.guessed == c.roc:
        if seq > c.s_l:
            c.s_l = seq & 0xFFFF
    elif c.guessed == i32(c.roc + 1):
        c.s_l = seq & 0xFFFF
        c.roc = c.guessed


def rtp_iv(c, buf):
    ssrc = buf[8:12]
    index = (lshl(c.guessed, 16) | ((buf[2] << 8) | buf[3])) & ((1 << 48) - 1)
    ib = index.to_bytes(6, "big")
    return bytes([c.salt[0], c.salt[1], c.salt[2], c.salt[3]] +
                 [ssrc[k] ^ c.salt[4 + k] for k in range(4)] +
                 [ib[k] ^ c.salt[8 + k] for k in range(6)] + [0, 0])


def rtp_f8_iv(c, buf):
    """SRTPCryptoContext.processPacketAESF8 :532-555: 0 || header[1..11] || ROC."""
    return bytes([0]) + bytes(buf[1:12]) + (c.guessed & M32).to_bytes(4, "big")


def rtcp_f8_iv(buf, index):
    """SRTCPCryptoContext.processPacketAESF8 :267-298: 0^4 || E|index || header[0..7]."""
    return bytes(4) + ((index | 0x80000000) & M32).to_bytes(4, "big") + bytes(buf[0:8])


def rtcp_iv(c, buf, index):
    ib = (index & M32).to_bytes(4, "big")
    return bytes(list(c.salt[:4]) + [buf[4 + k] ^ c.salt[4 + k] for k in range(4)] +
                 [c.salt[8], c.salt[9]] + [ib[k] ^ c.salt[10 + k] for k in range(4)] + [0, 0])


def process_one(t, reverse, buf: bytearray, L, cap, flags):
    """Returns (status, new length)."""
    if L < 12 or L > cap:
        return 7, L
    if t.kind == 0:
        if reverse and (buf[0] & 0xC0) != 0x80:
            return 3, L
        c = t.get(int.from_bytes(buf[8:12], "big"), t.rev if reverse else t.fwd)
        if c is None:
            return 4, L
        enc, _, auth, _, T, _ = c.policy
        seq = (buf[2] << 8) | buf[3]
        if not reverse:
            if L + (T if auth else 0) > cap:
                return 5, L
            if not c.seq_set:
                c.seq_set, c.s_l = True, seq
            gi = guess(c, seq)
            if not replay_ok(c, gi):
                return 1, L
            if enc in (1, 2):
                try:
                    h = header_len(buf, cap)
                    if enc == 1:
                        ctr_process(c.rks, buf, cap, h, L - h, rtp_iv(c, buf))
                    else:
                        f8_process(c.rks, c.f8rks, buf, h, L - h, rtp_f8_iv(c, buf))
                except Throw:
                    return 6, L
            if auth:
                tag = c.mac(bytes(buf[:L]), c.guessed)[:T]
                buf[L:L + T] = tag
                L += T
            update(c, seq, gi)
            return 0, L
        if not c.seq_set:
            c.seq_set, c.s_l = True, seq
        gi = guess(c, seq)
        if not replay_ok(c, gi):
            return 1, L
        if auth:
            got = bytes(buf[L - T:L])
            L = max(0, L - T) if T > 0 else L
            if c.mac(bytes(buf[:L]), c.guessed)[:T] != got:
                return 2, L
        if not (flags & 0x6) and enc in (1, 2):
            try:
                h = header_len(buf, cap)
                if enc == 1:
                    ctr_process(c.rks, buf, cap, h, L - h, rtp_iv(c, buf))
                else:
                    f8_process(c.rks, c.f8rks, buf, h, L - h, rtp_f8_iv(c, buf))
            except Throw:
                return 6, L
        update(c, seq, gi)
        return 0, L
    # SRTCP
    c = t.get(int.from_bytes(buf[4:8], "big"), t.rev if reverse else t.fwd)
    if c is None:
        return 4, L
    enc, _, auth, _, T, _ = c.policy
    if not reverse:
        if L + ((4 + T) if auth else 0) > cap:
            return 5, L
        if enc == 1:
            ctr_process(c.rks, buf, cap, 8, L - 8, rtcp_iv(c, buf, c.sent))
        elif enc == 2:
            f8_process(c.rks, c.f8rks, buf, 8, L - 4 - T, rtcp_f8_iv(buf, c.sent))
        index = (c.sent | 0x80000000) if enc in (1, 2) else 0
        if auth:
            tag = c.mac(bytes(buf[:L]), index)[:T]
            buf[L:L + 4] = (index & M32).to_bytes(4, "big")
            buf[L + 4:L + 4 + T] = tag
            L += 4 + T
        c.sent = (c.sent + 1) & 0x7FFFFFFF
        return 0, L
    io = L - 4 - T
    if io < 0:
        return 6, L
    ie = int.from_bytes(buf[io:io + 4], "big")
    decrypt = bool(ie & 0x80000000)
    index = ie & 0x7FFFFFFF
    delta = i32(index - c.recv)
    if not (delta > 0 or (-delta <= 64 and not ((c.window & M64) >> ((-delta) & 63)) & 1)):
        return 1, L
    if auth:
        got = bytes(buf[L - T:L])
        L = max(0, L - T - 4)
        if c.mac(bytes(buf[:L]), ie)[:T] != got:
            return 2, L
    if decrypt and enc == 1:
        try:
            ctr_process(c.rks, buf, cap, 8, L - 8, rtcp_iv(c, buf, index))
        except Throw:
            return 6, L
    if decrypt and enc == 2:
        f8_process(c.rks, c.f8rks, buf, 8, L - 4 - T, rtcp_f8_iv(buf, index))
    d2 = i32(c.recv - index)
    if d2 > 0:
        c.window = lshl(c.window, d2) | 1
    else:
        c.window = i64(c.window | ishl1(d2))
    c.recv = index
    return 0, L


def process(ts, reverse, seg, off, length, cap, flags=None, abort_on_error=True):
    """Same contract as oracle.process (numpy arrays, in place)."""
    n = len(off)
    status = [0] * n
    aborted = set()
    for i in range(n):
        t = ts[i] if isinstance(ts, (list, tuple)) else ts
        fl = int(flags[i]) if flags is not None else 0
        if t is None or fl & 0x80000000:
            status[i] = 9
            continue
        if id(t) in aborted:
            status[i] = 8
            continue
        o, C = int(off[i]), int(cap[i])
        buf = bytearray(seg[o:o + C].tobytes())
        st, L = process_one(t, reverse, buf, int(length[i]), C, fl)
        seg[o:o + C] = list(buf[:C])
        length[i] = L
        status[i] = st
        if st == 6 and abort_on_error:
            aborted.add(id(t))
    return status
