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

// ------------------------------------------------------------------ Twofish
// Schneier et al., "Twofish: A 128-Bit Block Cipher" (1998), 4.1-4.3, for the
// ZRTP "2FS" policies (TWOFISH_ENCRYPTION / TWOFISHF8_ENCRYPTION, run by
// BouncyCastle's TwofishEngine in the reference, BaseSRTPCryptoContext.java
// :217-225).  The key schedule folds the key-dependent S-boxes and the MDS
// matrix into four 256-word tables, which the GPU reads for g().
namespace {

struct TwofishQ {
    uint8_t q[2][256];
    TwofishQ() {
        static const uint8_t t[2][4][16] = {
            {{8, 1, 7, 13, 6, 15, 3, 2, 0, 11, 5, 9, 14, 12, 10, 4},
             {14, 12, 11, 8, 1, 2, 3, 5, 15, 4, 10, 6, 7, 0, 9, 13},
             {11, 10, 5, 14, 6, 13, 9, 0, 12, 8, 15, 3, 2, 4, 7, 1},
             {13, 7, 15, 4, 1, 2, 6, 14, 9, 11, 3, 0, 8, 5, 12, 10}},
            {{2, 8, 11, 13, 15, 7, 6, 14, 3, 1, 9, 4, 0, 10, 12, 5},
             {1, 14, 2, 11, 4, 12, 3, 7, 6, 13, 10, 5, 15, 9, 0, 8},
             {4, 12, 7, 5, 1, 6, 9, 10, 0, 14, 13, 8, 2, 11, 3, 15},
             {11, 9, 5, 1, 12, 3, 13, 14, 6, 4, 7, 15, 2, 0, 8, 10}}};
        auto r4 = [](unsigned v) { return ((v >> 1) | (v << 3)) & 15u; };
        for (int w = 0; w < 2; w++)
            for (unsigned x = 0; x < 256; x++) {
                unsigned a = x >> 4, b = x & 15;
                unsigned a1 = a ^ b, b1 = (a ^ r4(b) ^ (a << 3)) & 15;
                unsigned a2 = t[w][0][a1], b2 = t[w][1][b1];
                unsigned a3 = a2 ^ b2, b3 = (a2 ^ r4(b2) ^ (a2 << 3)) & 15;
                q[w][x] = (uint8_t)((t[w][3][b3] << 4) | t[w][2][a3]);
            }
    }
};

const TwofishQ &tfq() {
    static const TwofishQ t;
    return t;
}

uint8_t gf_mul_poly(unsigned a, unsigned b, unsigned poly) {
    unsigned r = 0;
    for (; b; b >>= 1, a <<= 1) {
        if (a & 0x100) a ^= poly;
        if (b & 1) r ^= a;
    }
    return (uint8_t)r;
}

// which q each of the h stages applies to byte j: [k=4 stage, k>=3 stage,
// before L1, before L0, last]
const int kHq[4][5] = {{1, 1, 0, 0, 1}, {0, 1, 1, 0, 0}, {0, 0, 0, 1, 1}, {1, 0, 1, 1, 0}};
const uint8_t kMds[4][4] = {
    {0x01, 0xEF, 0x5B, 0x5B}, {0x5B, 0xEF, 0xEF, 0x01}, {0xEF, 0x5B, 0x01, 0xEF}, {0xEF, 0x01, 0xEF, 0x5B}};
const uint8_t kRs[4][8] = {{0x01, 0xA4, 0x55, 0x87, 0x5A, 0x58, 0xDB, 0x9E},
                           {0xA4, 0x56, 0x82, 0xF3, 0x1E, 0xC6, 0x68, 0xE5},
                           {0x02, 0xA1, 0xFC, 0xC1, 0x47, 0xAE, 0x3D, 0x19},
                           {0xA4, 0x55, 0x87, 0x5A, 0x58, 0xDB, 0x9E, 0x03}};

uint8_t h_sbox(int j, uint8_t y, const uint32_t *L, int k) {
    const uint8_t(*q)[256] = tfq().q;
    auto lb = [&](int i) { return (uint8_t)(L[i] >> (8 * j)); };
    if (k == 4) y = (uint8_t)(q[kHq[j][0]][y] ^ lb(3));
    if (k >= 3) y = (uint8_t)(q[kHq[j][1]][y] ^ lb(2));
    y = (uint8_t)(q[kHq[j][2]][y] ^ lb(1));
    y = (uint8_t)(q[kHq[j][3]][y] ^ lb(0));
    return q[kHq[j][4]][y];
}

uint32_t mds_col(int j, uint8_t y) {
    return (uint32_t)gf_mul_poly(kMds[0][j], y, 0x169) | (uint32_t)gf_mul_poly(kMds[1][j], y, 0x169) << 8 |
           (uint32_t)gf_mul_poly(kMds[2][j], y, 0x169) << 16 |
           (uint32_t)gf_mul_poly(kMds[3][j], y, 0x169) << 24;
}

uint32_t h_word(uint32_t x, const uint32_t *L, int k) {
    uint32_t z = 0;
    for (int j = 0; j < 4; j++) z ^= mds_col(j, h_sbox(j, (uint8_t)(x >> (8 * j)), L, k));
    return z;
}

} // namespace

void twofish_schedule(const uint8_t *key, int key_len, uint32_t K[40], uint32_t T[4][256]) {
    const int k = key_len / 8;
    uint32_t even[4], odd[4], sv[4];
    for (int i = 0; i < k; i++) {
        const uint8_t *m = key + 8 * i;
        even[i] = (uint32_t)m[0] | (uint32_t)m[1] << 8 | (uint32_t)m[2] << 16 | (uint32_t)m[3] << 24;
        odd[i] = (uint32_t)m[4] | (uint32_t)m[5] << 8 | (uint32_t)m[6] << 16 | (uint32_t)m[7] << 24;
        uint32_t w = 0;
        for (int r = 0; r < 4; r++) {
            uint8_t v = 0;
            for (int c = 0; c < 8; c++) v ^= gf_mul_poly(kRs[r][c], m[c], 0x14D);
            w |= (uint32_t)v << (8 * r);
        }
        sv[k - 1 - i] = w;
    }
    for (int i = 0; i < 20; i++) {
        const uint32_t a = h_word(0x02020202u * (uint32_t)i, even, k);
        const uint32_t b = rotl(h_word(0x02020202u * (uint32_t)i + 0x01010101u, odd, k), 8);
        K[2 * i] = a + b;
        K[2 * i + 1] = rotl(a + 2 * b, 9);
    }
    for (int j = 0; j < 4; j++)
        for (int x = 0; x < 256; x++) T[j][x] = mds_col(j, h_sbox(j, (uint8_t)x, sv, k));
    memset(even, 0, sizeof even);
    memset(odd, 0, sizeof odd);
    memset(sv, 0, sizeof sv);
}

void twofish_encrypt_block(const uint32_t K[40], const uint32_t T[4][256], const uint8_t in[16],
                           uint8_t out[16]) {
    auto g = [&](uint32_t x) {
        return T[0][x & 255] ^ T[1][(x >> 8) & 255] ^ T[2][(x >> 16) & 255] ^ T[3][x >> 24];
    };
    uint32_t r[4];
    for (int i = 0; i < 4; i++) {
        uint32_t w;
        memcpy(&w, in + 4 * i, 4); // little-endian host
        r[i] = w ^ K[i];
    }
    for (int rd = 0; rd < 16; rd++) {
        const uint32_t t0 = g(r[0]), t1 = g(rotl(r[1], 8));
        const uint32_t f0 = t0 + t1 + K[2 * rd + 8], f1 = t0 + 2 * t1 + K[2 * rd + 9];
        const uint32_t x = r[2] ^ f0;
        const uint32_t n0 = (x >> 1) | (x << 31), n1 = rotl(r[3], 1) ^ f1;
        r[2] = r[0];
        r[3] = r[1];
        r[0] = n0;
        r[1] = n1;
    }
    for (int i = 0; i < 4; i++) {
        const uint32_t c = r[(i + 2) & 3] ^ K[i + 4];
        memcpy(out + 4 * i, &c, 4);
    }
}

// SRTPCipherCTR.getCipherStream (:68-92) for the short key-derivation streams,
// over AES (nr rounds of rk) or Twofish (tf_K / tf_T).
struct PrfCipher {
    const uint32_t *rk = nullptr;
    int nr = 0;
    const uint32_t *tf_K = nullptr;
    const uint32_t (*tf_T)[256] = nullptr;
    void encrypt(const uint8_t in[16], uint8_t out[16]) const {
        if (tf_K) twofish_encrypt_block(tf_K, tf_T, in, out);
        else aes_encrypt_block_nr(rk, nr, in, out);
    }
};

static void cipher_stream(const PrfCipher &c, uint8_t *out, int length, const uint8_t iv[16]) {
    uint8_t in[16], blk[16];
    memcpy(in, iv, 14);
    for (int ctr = 0; ctr * 16 < length; ctr++) {
        in[14] = (uint8_t)(ctr >> 8);
        in[15] = (uint8_t)ctr;
        c.encrypt(in, blk);
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
    derive_session_keys_cipher(false, mk, key_len, ms, rtcp, enc, auth, salt);
}

void derive_session_keys_cipher(bool twofish, const uint8_t *mk, int key_len, const uint8_t ms[14],
                                bool rtcp, uint8_t *enc, uint8_t *auth, uint8_t salt[14], int auth_len) {
    uint32_t rk[60];
    static thread_local uint32_t tK[40], tT[4][256];
    PrfCipher prf;
    if (twofish) {
        twofish_schedule(mk, key_len, tK, tT);
        prf.tf_K = tK;
        prf.tf_T = tT;
    } else {
        prf.nr = aes_expand_le(mk, key_len, rk);
        prf.rk = rk;
    }
    uint8_t iv[16];
    const int base = rtcp ? 3 : 0;
    uint8_t *outs[3] = {enc, auth, salt};
    const int lens[3] = {key_len, auth_len, 14};
    for (int lab = 0; lab < 3; lab++) {
        memcpy(iv, ms, 14);
        iv[7] ^= (uint8_t)(base + lab); // computeIv: key_id = label << 48 lands in byte 7
        iv[14] = iv[15] = 0;
        cipher_stream(prf, outs[lab], lens[lab], iv);
    }
    memset(rk, 0, sizeof rk);
    memset(tK, 0, sizeof tK);
    memset(tT, 0, sizeof tT);
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

// ------------------------------------------------------------ Skein-512
// "The Skein Hash Function Family" 1.3: Threefish-512 (72 rounds, a subkey
// every 4), UBI chaining, and the keyed form SkeinMac uses.  The host only
// runs the key and config UBIs once per key set (plus whole MACs for the C
// ABI's srtp_skein512_mac); the per-packet MAC is on the GPU.
namespace {

const int kSkR[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                        {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};

inline uint64_t rol64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

// h = Threefish-512(key h, tweak {t0, t1}, m) ^ m
void skein_block(uint64_t h[8], const uint64_t m[8], uint64_t t0, uint64_t t1) {
    uint64_t k[9], t[3] = {t0, t1, t0 ^ t1}, v[8];
    k[8] = kSkeinParity;
    for (int i = 0; i < 8; i++) {
        k[i] = h[i];
        k[8] ^= h[i];
        v[i] = m[i];
    }
    for (int s = 0; s <= 18; s++) {
        for (int i = 0; i < 8; i++) v[i] += k[(s + i) % 9];
        v[5] += t[s % 3];
        v[6] += t[(s + 1) % 3];
        v[7] += (uint64_t)s;
        if (s == 18) break;
        for (int r = 0; r < 4; r++) {
            const int *R = kSkR[(4 * s + r) % 8];
            // MIX on (0,1) (2,3) (4,5) (6,7), then the word permutation
            // {2, 1, 4, 7, 6, 5, 0, 3}
            for (int j = 0; j < 4; j++) {
                v[2 * j] += v[2 * j + 1];
                v[2 * j + 1] = rol64(v[2 * j + 1], R[j]) ^ v[2 * j];
            }
            const uint64_t w0 = v[0], w3 = v[3];
            v[0] = v[2]; v[2] = v[4]; v[4] = v[6]; v[6] = w0;
            v[3] = v[7]; v[7] = w3;
        }
    }
    for (int i = 0; i < 8; i++) h[i] = v[i] ^ m[i];
}

// UBI(h, msg[0..n), type) over the whole message (zero-padded; one block of
// zeros for an empty message)
void skein_ubi(uint64_t h[8], const uint8_t *msg, size_t n, uint64_t type) {
    size_t pos = 0;
    bool first = true;
    do {
        uint8_t blk[64] = {0};
        const size_t take = n - pos < 64 ? n - pos : 64;
        if (take) memcpy(blk, msg + pos, take);
        pos += take;
        uint64_t m[8];
        for (int i = 0; i < 8; i++) {
            m[i] = 0;
            for (int b = 7; b >= 0; b--) m[i] = (m[i] << 8) | blk[8 * i + b];
        }
        const uint64_t t1 = (type << 56) | (first ? 1ull << 62 : 0) | (pos == n ? 1ull << 63 : 0);
        skein_block(h, m, pos, t1);
        first = false;
    } while (pos < n);
}

} // namespace

void skein512_key_state(const uint8_t *key, int key_len, int out_bits, uint64_t g0[8]) {
    memset(g0, 0, 64);
    if (key_len > 0) skein_ubi(g0, key, (size_t)key_len, kSkeinTypeKey);
    uint8_t cfg[32] = {'S', 'H', 'A', '3', 1, 0, 0, 0};
    for (int i = 0; i < 8; i++) cfg[8 + i] = (uint8_t)((uint64_t)out_bits >> (8 * i));
    skein_ubi(g0, cfg, sizeof cfg, kSkeinTypeCfg);
}

void skein512_mac(const uint8_t *key, int key_len, int out_bits, const uint8_t *msg, size_t n,
                  uint8_t *out) {
    uint64_t h[8];
    skein512_key_state(key, key_len, out_bits, h);
    skein_ubi(h, msg, n, kSkeinTypeMsg);
    const uint8_t zero8[8] = {0};
    skein_ubi(h, zero8, 8, kSkeinTypeOut);
    for (int i = 0; i < (out_bits + 7) / 8; i++) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

} // namespace srtp
