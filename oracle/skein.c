/* skein.c -- Skein-512 (version 1.3) for the oracle.  TEST INFRASTRUCTURE ONLY:
 * see skein.h for what it restates and how it is pinned. */
#include "skein.h"

#include <string.h>

#define C240 0x1BD11BDAA9FC1A22ull

/* Skein 1.3 Table 4: rotation constants R(d mod 8, j) of Threefish-512 */
static const int R512[8][4] = {
    {46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
    {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22},
};
/* Table 3: the word permutation pi of Nw = 8 (f_i = e_pi(i)) */
static const int PI512[8] = {2, 1, 4, 7, 6, 5, 0, 3};

/* UBI block types (Table 6) */
enum { T_KEY = 0, T_CFG = 4, T_MSG = 48, T_OUT = 63 };
#define FLAG_FIRST (1ull << 62) /* tweak bit 126 */
#define FLAG_FINAL (1ull << 63) /* tweak bit 127 */

static inline uint64_t rotl64(uint64_t x, int n) { return (x << n) | (x >> (64 - n)); }

static inline uint64_t ld64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
    return v;
}

void sk_threefish512(const uint64_t k[8], const uint64_t t[2], const uint64_t in[8], uint64_t out[8]) {
    uint64_t ks[9], ts[3], v[8], e[8];
    ks[8] = C240;
    for (int i = 0; i < 8; i++) { ks[i] = k[i]; ks[8] ^= k[i]; }
    ts[0] = t[0]; ts[1] = t[1]; ts[2] = t[0] ^ t[1];
    memcpy(v, in, sizeof v);
    for (int d = 0; d < 72; d++) {
        if (d % 4 == 0) { /* subkey s = d / 4 (section 3.3.2) */
            const int s = d / 4;
            for (int i = 0; i < 8; i++) v[i] += ks[(s + i) % 9];
            v[5] += ts[s % 3];
            v[6] += ts[(s + 1) % 3];
            v[7] += (uint64_t)s;
        }
        for (int j = 0; j < 4; j++) { /* MIX */
            e[2 * j] = v[2 * j] + v[2 * j + 1];
            e[2 * j + 1] = rotl64(v[2 * j + 1], R512[d % 8][j]) ^ e[2 * j];
        }
        for (int i = 0; i < 8; i++) v[i] = e[PI512[i]];
    }
    for (int i = 0; i < 8; i++) v[i] += ks[(18 + i) % 9];
    v[5] += ts[18 % 3];
    v[6] += ts[19 % 3];
    v[7] += 18u;
    memcpy(out, v, sizeof v);
}

/* one UBI step: h = E(h, tweak, block) ^ block */
static void ubi_block(uint64_t h[8], const uint8_t blk[64], uint64_t pos, int type, int first,
                      int final) {
    uint64_t m[8], t[2], c[8];
    for (int i = 0; i < 8; i++) m[i] = ld64(blk + 8 * i);
    t[0] = pos;
    t[1] = ((uint64_t)type << 56) | (first ? FLAG_FIRST : 0) | (final ? FLAG_FINAL : 0);
    sk_threefish512(h, t, m, c);
    for (int i = 0; i < 8; i++) h[i] = c[i] ^ m[i];
}

/* UBI(h, msg, type) over a whole message (section 3.4) */
static void ubi(uint64_t h[8], const uint8_t *msg, size_t n, int type) {
    uint8_t blk[64];
    size_t done = 0;
    int first = 1;
    do {
        const size_t take = (n - done > 64) ? 64 : n - done;
        memset(blk, 0, sizeof blk);
        memcpy(blk, msg + done, take);
        done += take;
        ubi_block(h, blk, done, type, first, done == n);
        first = 0;
    } while (done < n);
}

void sk_init(sk_ctx *c, const uint8_t *key, int key_len, int out_bits) {
    memset(c, 0, sizeof *c);
    if (key_len > 0) ubi(c->g0, key, (size_t)key_len, T_KEY); /* K' = UBI(0, K, Tkey) */
    uint8_t cfg[32] = {0x53, 0x48, 0x41, 0x33, 1, 0, 0, 0}; /* "SHA3", version 1 */
    for (int i = 0; i < 8; i++) cfg[8 + i] = (uint8_t)((uint64_t)out_bits >> (8 * i));
    ubi(c->g0, cfg, sizeof cfg, T_CFG); /* tree parameters 0: sequential */
    c->out_bits = out_bits;
    sk_reset(c);
}

void sk_reset(sk_ctx *c) {
    memcpy(c->h, c->g0, sizeof c->h);
    c->nbuf = 0;
    c->pos = 0;
    c->first = 1;
}

void sk_update(sk_ctx *c, const uint8_t *msg, size_t n) {
    while (n > 0) {
        if (c->nbuf == 64) { /* more data follows: the held block is not the last */
            c->pos += 64;
            ubi_block(c->h, c->buf, c->pos, T_MSG, c->first, 0);
            c->first = 0;
            c->nbuf = 0;
        }
        const size_t take = (n < (size_t)(64 - c->nbuf)) ? n : (size_t)(64 - c->nbuf);
        memcpy(c->buf + c->nbuf, msg, take);
        c->nbuf += (int)take;
        msg += take;
        n -= take;
    }
}

void sk_final(sk_ctx *c, uint8_t *out) {
    memset(c->buf + c->nbuf, 0, (size_t)(64 - c->nbuf));
    c->pos += (uint64_t)c->nbuf;
    ubi_block(c->h, c->buf, c->pos, T_MSG, c->first, 1);
    /* Output(G, No) = UBI(G, ToBytes(0, 8), Tout) for No <= 512 */
    uint8_t ctr[64] = {0};
    uint64_t o[8];
    memcpy(o, c->h, sizeof o);
    ubi_block(o, ctr, 8, T_OUT, 1, 1);
    const int nbytes = (c->out_bits + 7) / 8;
    for (int i = 0; i < nbytes; i++) out[i] = (uint8_t)(o[i / 8] >> (8 * (i % 8)));
    sk_reset(c);
}
