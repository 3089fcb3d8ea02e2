// host_crypto.cpp -- see host_crypto.h.  FIPS-197 AES-128/256 and FIPS 180-4
// SHA-1, written for clarity (control plane only).
#include "host_crypto.h"

#include <string.h>

namespace srtp {

namespace {

uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return r;
}

struct SBox {
    uint8_t s[256];
    SBox() {
        // multiplicative inverse in GF(2^8) followed by the affine map
        for (int x = 0; x < 256; x++) {
            uint8_t inv = 0;
            if (x) {
                for (int y = 1; y < 256; y++)
                    if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
            }
            uint8_t b = inv, r = inv;
            for (int i = 0; i < 4; i++) {
                b = (uint8_t)((b << 1) | (b >> 7));
                r ^= b;
            }
            s[x] = (uint8_t)(r ^ 0x63);
        }
    }
};

const SBox &sbox() {
    static const SBox sb;
    return sb;
}

inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

} // namespace

const uint32_t kSha1Init[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};

void aes_te0_le(uint32_t te0[256]) {
    const uint8_t *S = sbox().s;
    for (int x = 0; x < 256; x++) {
        uint8_t s = S[x], s2 = xtime(s), s3 = (uint8_t)(s2 ^ s);
        te0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
}

// FIPS-197 5.2 key expansion for Nk = 4 (AES-128) or 8 (AES-256) words.
int aes_expand_le(const uint8_t *key, int key_len, uint32_t rk[60]) {
    const uint8_t *S = sbox().s;
    const int nk = key_len / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint8_t w[240];
    memcpy(w, key, (size_t)key_len);
    uint8_t rcon = 1;
    for (int i = nk; i < total; i++) {
        uint8_t t[4] = {w[4 * i - 4], w[4 * i - 3], w[4 * i - 2], w[4 * i - 1]};
        if (i % nk == 0) {
            uint8_t t0 = t[0];
            t[0] = (uint8_t)(S[t[1]] ^ rcon);
            t[1] = S[t[2]];
            t[2] = S[t[3]];
            t[3] = S[t0];
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int k = 0; k < 4; k++) t[k] = S[t[k]];
        }
        for (int k = 0; k < 4; k++) w[4 * i + k] = (uint8_t)(w[4 * (i - nk) + k] ^ t[k]);
    }
    for (int i = 0; i < total; i++)
        rk[i] = (uint32_t)w[4 * i] | ((uint32_t)w[4 * i + 1] << 8) | ((uint32_t)w[4 * i + 2] << 16) |
                ((uint32_t)w[4 * i + 3] << 24);
    memset(w, 0, sizeof w);
    return nr;
}

void aes128_expand_le(const uint8_t key[16], uint32_t rk[44]) {
    uint32_t t[60];
    aes_expand_le(key, 16, t);
    memcpy(rk, t, 44 * 4);
    memset(t, 0, sizeof t);
}

void aes_encrypt_block_nr(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    const uint8_t *S = sbox().s;
    uint8_t st[16];
    for (int i = 0; i < 16; i++) st[i] = (uint8_t)(in[i] ^ (rk[i / 4] >> (8 * (i % 4))));
    for (int r = 1; r <= nr; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int row = 0; row < 4; row++) t[4 * c + row] = S[st[4 * ((c + row) % 4) + row]];
        if (r != nr) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                t[4 * c + 0] = (uint8_t)(xtime(a0) ^ (xtime(a1) ^ a1) ^ a2 ^ a3);
                t[4 * c + 1] = (uint8_t)(a0 ^ xtime(a1) ^ (xtime(a2) ^ a2) ^ a3);
                t[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xtime(a2) ^ (xtime(a3) ^ a3));
                t[4 * c + 3] = (uint8_t)((xtime(a0) ^ a0) ^ a1 ^ a2 ^ xtime(a3));
            }
        }
        for (int i = 0; i < 16; i++) st[i] = (uint8_t)(t[i] ^ (rk[4 * r + i / 4] >> (8 * (i % 4))));
    }
    memcpy(out, st, 16);
}

void aes128_encrypt_block(const uint32_t rk[44], const uint8_t in[16], uint8_t out[16]) {
    aes_encrypt_block_nr(rk, 10, in, out);
}

void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
    uint32_t w[80];
    for (int t = 0; t < 16; t++)
        w[t] = ((uint32_t)blk[4 * t] << 24) | ((uint32_t)blk[4 * t + 1] << 16) |
               ((uint32_t)blk[4 * t + 2] << 8) | blk[4 * t + 3];
    for (int t = 16; t < 80; t++) w[t] = rotl(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
        uint32_t f, k;
        if (t < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
        else if (t < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
        else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
        uint32_t tmp = rotl(a, 5) + f + e + k + w[t];
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// SRTPCipherCTR.getCipherStream (:68-92) for the short key-derivation streams.
static void cipher_stream(const uint32_t *rk, int nr, uint8_t *out, int length, const uint8_t iv[16]) {
    uint8_t in[16], blk[16];
    memcpy(in, iv, 14);
    for (int ctr = 0; ctr * 16 < length; ctr++) {
        in[14] = (uint8_t)(ctr >> 8);
        in[15] = (uint8_t)ctr;
        aes_encrypt_block_nr(rk, nr, in, blk);
        int n = length - ctr * 16 < 16 ? length - ctr * 16 : 16;
        memcpy(out + ctr * 16, blk, (size_t)n);
    }
}

void derive_session_keys(const uint8_t mk[16], const uint8_t ms[14], bool rtcp, uint8_t enc[16],
                         uint8_t auth[20], uint8_t salt[14]) {
    derive_session_keys_n(mk, 16, ms, rtcp, enc, auth, salt);
}

void derive_session_keys_n(const uint8_t *mk, int key_len, const uint8_t ms[14], bool rtcp,
                           uint8_t *enc, uint8_t auth[20], uint8_t salt[14]) {
    uint32_t rk[60];
    const int nr = aes_expand_le(mk, key_len, rk);
    uint8_t iv[16];
    const int base = rtcp ? 3 : 0;
    uint8_t *outs[3] = {enc, auth, salt};
    const int lens[3] = {key_len, 20, 14};
    for (int lab = 0; lab < 3; lab++) {
        memcpy(iv, ms, 14);
        iv[7] ^= (uint8_t)(base + lab); // computeIv: key_id = label << 48 lands in byte 7
        iv[14] = iv[15] = 0;
        cipher_stream(rk, nr, outs[lab], lens[lab], iv);
    }
    memset(rk, 0, sizeof rk);
}

void hmac_sha1_midstates(const uint8_t key[20], uint32_t ipad[5], uint32_t opad[5]) {
    uint8_t bi[64], bo[64];
    memset(bi, 0x36, 64);
    memset(bo, 0x5c, 64);
    for (int i = 0; i < 20; i++) {
        bi[i] ^= key[i];
        bo[i] ^= key[i];
    }
    memcpy(ipad, kSha1Init, 20);
    memcpy(opad, kSha1Init, 20);
    sha1_compress(ipad, bi);
    sha1_compress(opad, bo);
    memset(bi, 0, 64);
    memset(bo, 0, 64);
}

} // namespace srtp
