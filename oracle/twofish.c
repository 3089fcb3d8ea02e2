/* twofish.c -- Twofish block cipher (Schneier et al., "Twofish: A 128-Bit
 * Block Cipher", 1998, sections 4.1-4.3), restated from the specification for
 * the oracle.  TEST INFRASTRUCTURE ONLY (see srtp_oracle.c).
 *
 * The reference's ZRTP "2FS" cipher is BouncyCastle's TwofishEngine
 * (BaseSRTPCryptoContext.java:217-225, bccontrib/bcprov); that jar is absent,
 * so this restatement is pinned by the specification's known answers
 * (tests/test_twofish.py). */
#include "twofish.h"

#include <string.h>

/* q0 / q1 (section 4.3.5): 4-bit t-tables */
static const uint8_t Q0T[4][16] = {
    {8, 1, 7, 13, 6, 15, 3, 2, 0, 11, 5, 9, 14, 12, 10, 4},
    {14, 12, 11, 8, 1, 2, 3, 5, 15, 4, 10, 6, 7, 0, 9, 13},
    {11, 10, 5, 14, 6, 13, 9, 0, 12, 8, 15, 3, 2, 4, 7, 1},
    {13, 7, 15, 4, 1, 2, 6, 14, 9, 11, 3, 0, 8, 5, 12, 10}};
static const uint8_t Q1T[4][16] = {
    {2, 8, 11, 13, 15, 7, 6, 14, 3, 1, 9, 4, 0, 10, 12, 5},
    {1, 14, 2, 11, 4, 12, 3, 7, 6, 13, 10, 5, 15, 9, 0, 8},
    {4, 12, 7, 5, 1, 6, 9, 10, 0, 14, 13, 8, 2, 11, 3, 15},
    {11, 9, 5, 1, 12, 3, 13, 14, 6, 4, 7, 15, 2, 0, 8, 10}};

static uint8_t ror4(uint8_t x, int n) { return (uint8_t)(((x >> n) | (x << (4 - n))) & 15); }

static uint8_t qperm(const uint8_t t[4][16], uint8_t x) {
    uint8_t a0 = x >> 4, b0 = x & 15;
    uint8_t a1 = a0 ^ b0, b1 = (uint8_t)((a0 ^ ror4(b0, 1) ^ (8 * a0)) & 15);
    uint8_t a2 = t[0][a1], b2 = t[1][b1];
    uint8_t a3 = a2 ^ b2, b3 = (uint8_t)((a2 ^ ror4(b2, 1) ^ (8 * a2)) & 15);
    uint8_t a4 = t[2][a3], b4 = t[3][b3];
    return (uint8_t)(16 * b4 + a4);
}

static uint8_t q0(uint8_t x) { return qperm(Q0T, x); }
static uint8_t q1(uint8_t x) { return qperm(Q1T, x); }

/* multiplication in GF(2^8) modulo the given primitive polynomial */
static uint8_t gf_mul(uint8_t a, uint8_t b, unsigned poly) {
    unsigned r = 0, x = a;
    while (b) {
        if (b & 1) r ^= x;
        x <<= 1;
        if (x & 0x100) x ^= poly;
        b >>= 1;
    }
    return (uint8_t)r;
}

static const uint8_t MDS[4][4] = {{0x01, 0xEF, 0x5B, 0x5B},
                                  {0x5B, 0xEF, 0xEF, 0x01},
                                  {0xEF, 0x5B, 0x01, 0xEF},
                                  {0xEF, 0x01, 0xEF, 0x5B}};
static const uint8_t RS[4][8] = {{0x01, 0xA4, 0x55, 0x87, 0x5A, 0x58, 0xDB, 0x9E},
                                 {0xA4, 0x56, 0x82, 0xF3, 0x1E, 0xC6, 0x68, 0xE5},
                                 {0x02, 0xA1, 0xFC, 0xC1, 0x47, 0xAE, 0x3D, 0x19},
                                 {0xA4, 0x55, 0x87, 0x5A, 0x58, 0xDB, 0x9E, 0x03}};

static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

/* the four key-dependent byte permutations of h (section 4.3.2) applied to
 * byte y of position j, with the k words of L */
static uint8_t h_byte(int j, uint8_t y, const uint32_t *L, int k) {
#define LB(i) ((uint8_t)(L[i] >> (8 * j)))
    static const int first[4] = {1, 0, 0, 1};  /* k == 4: q1 q0 q0 q1 */
    static const int second[4] = {1, 1, 0, 0}; /* k >= 3: q1 q1 q0 q0 */
    if (k == 4) y = (uint8_t)((first[j] ? q1(y) : q0(y)) ^ LB(3));
    if (k >= 3) y = (uint8_t)((second[j] ? q1(y) : q0(y)) ^ LB(2));
    switch (j) {
    case 0: y = q1((uint8_t)(q0((uint8_t)(q0(y) ^ LB(1))) ^ LB(0))); break;
    case 1: y = q0((uint8_t)(q0((uint8_t)(q1(y) ^ LB(1))) ^ LB(0))); break;
    case 2: y = q1((uint8_t)(q1((uint8_t)(q0(y) ^ LB(1))) ^ LB(0))); break;
    default: y = q0((uint8_t)(q1((uint8_t)(q1(y) ^ LB(1))) ^ LB(0))); break;
    }
#undef LB
    return y;
}

static uint32_t mds_column(int j, uint8_t y) {
    uint32_t z = 0;
    for (int i = 0; i < 4; i++) z |= (uint32_t)gf_mul(MDS[i][j], y, 0x169) << (8 * i);
    return z;
}

static uint32_t h_fn(uint32_t X, const uint32_t *L, int k) {
    uint32_t z = 0;
    for (int j = 0; j < 4; j++) z ^= mds_column(j, h_byte(j, (uint8_t)(X >> (8 * j)), L, k));
    return z;
}

int tf_set_key(tf_key *t, const uint8_t *key, int key_len) {
    if (key_len != 16 && key_len != 24 && key_len != 32) return -1;
    const int k = key_len / 8;
    uint32_t M[8], Me[4], Mo[4], S[4];
    for (int i = 0; i < 2 * k; i++)
        M[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 |
               (uint32_t)key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
    for (int i = 0; i < k; i++) {
        Me[i] = M[2 * i];
        Mo[i] = M[2 * i + 1];
        uint32_t s = 0;
        for (int r = 0; r < 4; r++) {
            uint8_t v = 0;
            for (int c = 0; c < 8; c++) v ^= gf_mul(RS[r][c], key[8 * i + c], 0x14D);
            s |= (uint32_t)v << (8 * r);
        }
        S[k - 1 - i] = s; /* S = (S_{k-1}, ..., S_0) */
    }
    const uint32_t rho = 0x01010101u;
    for (int i = 0; i < 20; i++) {
        uint32_t A = h_fn(2 * i * rho, Me, k);
        uint32_t B = rol(h_fn((2 * i + 1) * rho, Mo, k), 8);
        t->K[2 * i] = A + B;
        t->K[2 * i + 1] = rol(A + 2 * B, 9);
    }
    /* g = h(., S): the full key-dependent tables, g(X) = ^_j T_j[byte j of X] */
    for (int j = 0; j < 4; j++)
        for (int x = 0; x < 256; x++) t->T[j][x] = mds_column(j, h_byte(j, (uint8_t)x, S, k));
    memset(M, 0, sizeof M);
    return 0;
}

static uint32_t g_fn(const tf_key *t, uint32_t X) {
    return t->T[0][X & 255] ^ t->T[1][(X >> 8) & 255] ^ t->T[2][(X >> 16) & 255] ^ t->T[3][X >> 24];
}

void tf_encrypt(const tf_key *t, const uint8_t in[16], uint8_t out[16]) {
    uint32_t R[4];
    for (int i = 0; i < 4; i++)
        R[i] = ((uint32_t)in[4 * i] | (uint32_t)in[4 * i + 1] << 8 | (uint32_t)in[4 * i + 2] << 16 |
                (uint32_t)in[4 * i + 3] << 24) ^ t->K[i];
    for (int r = 0; r < 16; r++) {
        uint32_t T0 = g_fn(t, R[0]), T1 = g_fn(t, rol(R[1], 8));
        uint32_t F0 = T0 + T1 + t->K[2 * r + 8], F1 = T0 + 2 * T1 + t->K[2 * r + 9];
        uint32_t n0 = ror(R[2] ^ F0, 1), n1 = rol(R[3], 1) ^ F1;
        R[2] = R[0];
        R[3] = R[1];
        R[0] = n0;
        R[1] = n1;
    }
    for (int i = 0; i < 4; i++) {
        uint32_t c = R[(i + 2) & 3] ^ t->K[i + 4];
        out[4 * i] = (uint8_t)c; out[4 * i + 1] = (uint8_t)(c >> 8);
        out[4 * i + 2] = (uint8_t)(c >> 16); out[4 * i + 3] = (uint8_t)(c >> 24);
    }
}
