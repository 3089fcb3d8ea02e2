/*
 * srtp_oracle.c -- CPU restatement of libjitsi's SRTP/SRTCP hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).  See the header
 * for scope, the reference files it follows and the packet model.  Every
 * function below names the reference lines it restates; Java integer
 * semantics are reproduced explicitly (wrapping i32, JLS 15.19 shift masks).
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include "srtp_oracle.h"
#include "skein.h"
#include "twofish.h"

#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/kdf.h>
#include <openssl/core_names.h>
#include <openssl/params.h>
#include <stdlib.h>
#include <string.h>

#define THROW (-1) /* a Java exception escaped the context method */

static int g_check_replay = 1; /* SRTPCryptoContext.java:87, read at :110-121 */

void orc_set_check_replay(int enabled) { g_check_replay = enabled ? 1 : 0; }

/* ---------- Java integer helpers ---------------------------------------- */
static inline int32_t j_add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
static inline int32_t j_sub(int32_t a, int32_t b) { return (int32_t)((uint32_t)a - (uint32_t)b); }
/* long << n (distance & 63) */
static inline int64_t j_lshl(int64_t v, int64_t n) { return (int64_t)((uint64_t)v << (n & 63)); }
/* int 1 << n (distance & 31), result int */
static inline int32_t j_ishl1(int64_t n) { return (int32_t)(1u << (n & 31)); }
/* bit ((v >> n) & 1) for long v, distance & 63 */
static inline int j_lbit(int64_t v, int64_t n) { return (int)(((uint64_t)v >> (n & 63)) & 1u); }

/* ---------- structures -------------------------------------------------- */
struct orc_factory {
    int sender, mode, closed;
    uint8_t master_key[32], master_salt[14];
    orc_policy srtp, srtcp;
};

typedef struct orc_ctx {
    uint32_t ssrc;
    int kind;
    orc_policy policy;
    int mode;
    uint8_t enc_key[32], auth_key[64], salt_key[14];
    int key_len; /* 16 or 32 (AES-256-CM) */
    sk_ctx skein;         /* SKEIN_AUTHENTICATION: keyed Skein-512, tag_len * 8 output bits */
    struct blk *ecb;      /* AES-128/256 or Twofish keyed with the session key */
    EVP_CIPHER_CTX *ctr;  /* tuned mode (AES) */
    struct blk *f8;       /* F8: IV' cipher keyed with encKey ^ (salt || 0x55..) */
    HMAC_CTX *hmac;       /* ref: re-keyed per packet; tuned: pre-keyed template */
    HMAC_CTX *hmac_work;
    /* SRTPCryptoContext state (:130-164) */
    int32_t roc, s_l, guessed_roc;
    int seq_num_set;
    /* SRTCPCryptoContext state (:54-59) */
    int32_t sent_index, received_index;
    int64_t replay_window; /* BaseSRTPCryptoContext.java:138 */
    uint8_t tag_store[64];
    uint8_t temp_store[100];
} orc_ctx;

typedef struct {
    uint32_t *keys;
    orc_ctx **vals;
    uint32_t cap, count;
} ctx_map;

struct orc_transformer {
    int kind;
    orc_factory *fwd, *rev;
    ctx_map map;
};

/* ---------- primitives -------------------------------------------------- */
static EVP_CIPHER_CTX *aes_ecb_new(const uint8_t key[16]) {
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(c, EVP_aes_128_ecb(), NULL, key, NULL);
    EVP_CIPHER_CTX_set_padding(c, 0);
    return c;
}

/* AES-128 or AES-256 (key_len 32) ECB, for AES-256-CM and its PRF */
static EVP_CIPHER_CTX *aes_ecb_new_n(const uint8_t *key, int key_len) {
    if (key_len != 32) return aes_ecb_new(key);
    EVP_CIPHER_CTX *c = EVP_CIPHER_CTX_new();
    EVP_EncryptInit_ex(c, EVP_aes_256_ecb(), NULL, key, NULL);
    EVP_CIPHER_CTX_set_padding(c, 0);
    return c;
}

static inline void aes_block(EVP_CIPHER_CTX *c, const uint8_t in[16], uint8_t out[16]) {
    int outl = 0;
    EVP_EncryptUpdate(c, out, &outl, in, 16);
}

/* A block cipher instance: AES through OpenSSL, or Twofish (twofish.c) --
 * BaseSRTPCryptoContext picks AES.createBlockCipher() or TwofishEngine by the
 * policy's cipher (:197-226). */
typedef struct blk {
    EVP_CIPHER_CTX *evp;
    tf_key *tf;
} blk_t;

static int is_twofish(int enc) {
    return enc == ORC_TWOFISH_ENCRYPTION || enc == ORC_TWOFISHF8_ENCRYPTION;
}
static int is_ctr(int enc) { return enc == ORC_AESCM_ENCRYPTION || enc == ORC_TWOFISH_ENCRYPTION; }
static int is_f8(int enc) { return enc == ORC_AESF8_ENCRYPTION || enc == ORC_TWOFISHF8_ENCRYPTION; }

static blk_t *blk_new(int twofish, const uint8_t *key, int key_len) {
    blk_t *b = (blk_t *)calloc(1, sizeof *b);
    if (twofish) {
        b->tf = (tf_key *)calloc(1, sizeof *b->tf);
        tf_set_key(b->tf, key, key_len);
    } else {
        b->evp = aes_ecb_new_n(key, key_len);
    }
    return b;
}

static void blk_free(blk_t *b) {
    if (!b) return;
    if (b->evp) EVP_CIPHER_CTX_free(b->evp);
    if (b->tf) {
        memset(b->tf, 0, sizeof *b->tf);
        free(b->tf);
    }
    free(b);
}

static inline void blk_enc(blk_t *b, const uint8_t in[16], uint8_t out[16]) {
    if (b->tf) tf_encrypt(b->tf, in, out);
    else aes_block(b->evp, in, out);
}

void orc_twofish_encrypt_block(const uint8_t *key, int key_len, const uint8_t in[16],
                               uint8_t out[16]) {
    tf_key t;
    tf_set_key(&t, key, key_len);
    tf_encrypt(&t, in, out);
    memset(&t, 0, sizeof t);
}

void orc_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    EVP_CIPHER_CTX *c = aes_ecb_new(key);
    aes_block(c, in, out);
    EVP_CIPHER_CTX_free(c);
}

void orc_hmac_sha1(const uint8_t *key, int key_len, const uint8_t *msg, size_t n, uint8_t out[20]) {
    unsigned int ol = 20;
    HMAC(EVP_sha1(), key, key_len, msg, n, out, &ol);
}

/* SRTPCipherCTR.getCipherStream, SRTPCipherCTR.java:68-92: block j of the
 * keystream is AES(iv[0..13] || u16_be(j)); one extra tail block is always
 * computed; a negative, non-multiple-of-16 length makes the tail arraycopy
 * throw (IndexOutOfBoundsException). */
static int get_cipher_stream(blk_t *c, uint8_t *out, int length, const uint8_t iv[16]) {
    uint8_t in[16], tmp[16];
    memcpy(in, iv, 14);
    int ctr, ctr_end = length / 16; /* Java int division truncates like C99 */
    for (ctr = 0; ctr < ctr_end; ctr++) {
        in[14] = (uint8_t)((ctr & 0xFF00) >> 8);
        in[15] = (uint8_t)(ctr & 0x00FF);
        blk_enc(c, in, out + ctr * 16);
    }
    in[14] = (uint8_t)((ctr & 0xFF00) >> 8);
    in[15] = (uint8_t)(ctr & 0x00FF);
    blk_enc(c, in, tmp);
    int rem = length % 16; /* Java remainder has the dividend's sign, like C99 */
    if (rem < 0)
        return THROW;
    memcpy(out + ctr * 16, tmp, (size_t)rem);
    return 0;
}

/* SRTPCipherCTR.process, SRTPCipherCTR.java:94-121, on a buffer of length
 * buf_len (== RawPacket buffer.length, offset 0). */
static int cipher_ctr_process(orc_ctx *x, uint8_t *data, int buf_len, int off, int len,
                              const uint8_t iv[16]) {
    if ((int64_t)off + len > buf_len)
        return 0; /* silently skipped (:99-100) */
    if (len < 0) {
        /* getCipherStream: no blocks, tail arraycopy length len % 16 */
        return (len % 16 != 0) ? THROW : 0;
    }
    if (len > 0 && off < 0)
        return THROW; /* data[i + off] AIOOBE on the first XOR (:119-120) */
    if (len == 0)
        return 0;
    if (x->mode == ORC_MODE_TUNED && x->ctr) {
        int outl = 0;
        EVP_EncryptInit_ex(x->ctr, NULL, NULL, NULL, iv);
        EVP_EncryptUpdate(x->ctr, data + off, &outl, data + off, len);
        return 0;
    }
    uint8_t sbuf[1040];
    uint8_t *stream = (len + 16 <= (int)sizeof sbuf) ? sbuf : (uint8_t *)malloc((size_t)len + 16);
    get_cipher_stream(x->ecb, stream, len, iv);
    for (int i = 0; i < len; i++)
        data[i + off] ^= stream[i];
    if (stream != sbuf)
        free(stream);
    return 0;
}

/* SRTPCipherF8.deriveForIV, SRTPCipherF8.java:66-95: the IV' cipher is keyed
 * with key ^ (salt || 0x55 0x55 ..) (the salt copied, the rest 0x55). */
static blk_t *f8_iv_cipher_new(int twofish, const uint8_t *key, int key_len, const uint8_t *salt,
                               int salt_len) {
    uint8_t mk[32];
    for (int i = 0; i < key_len; i++)
        mk[i] = (uint8_t)(key[i] ^ (i < salt_len ? salt[i] : 0x55));
    blk_t *c = blk_new(twofish, mk, key_len);
    memset(mk, 0, sizeof mk);
    return c;
}

/* SRTPCipherF8.process :97-128 and processBlock :145-183: IV' = E(k_e ^ m, IV);
 * S(j) = E(k_e, IV' ^ S(j-1) ^ j) with S(-1) = 0 and j (a long) XORed into
 * bytes 12..15 big-endian; data[off + 16j + i] ^= S(j)[i].  The XOR loop
 * throws (AIOOBE) at a negative offset before touching the block; a negative
 * length processes nothing. */
static int cipher_f8_process(blk_t *c, blk_t *f8c, uint8_t *data, int off, int len,
                             const uint8_t iv[16]) {
    uint8_t ivp[16], S[16];
    blk_enc(f8c, iv, ivp);
    memset(S, 0, sizeof S);
    int64_t J = 0;
    int in_len = len;
    while (in_len > 0) {
        int n = in_len >= 16 ? 16 : in_len;
        for (int i = 0; i < 16; i++) S[i] ^= ivp[i];
        S[12] ^= (uint8_t)(J >> 24); S[13] ^= (uint8_t)(J >> 16);
        S[14] ^= (uint8_t)(J >> 8);  S[15] ^= (uint8_t)J;
        J++;
        blk_enc(c, S, S);
        if (off < 0) return THROW;
        for (int i = 0; i < n; i++) data[off + i] ^= S[i];
        in_len -= n;
        off += n;
    }
    return 0;
}

void orc_aes_f8(const uint8_t key[16], const uint8_t *salt, int salt_len, const uint8_t iv[16],
                uint8_t *data, int len) {
    blk_t *c = blk_new(0, key, 16), *f = f8_iv_cipher_new(0, key, 16, salt, salt_len);
    cipher_f8_process(c, f, data, 0, len, iv);
    blk_free(c);
    blk_free(f);
}

/* BaseSRTPCryptoContext.authenticatePacketHMAC, :269-278: tag_store =
 * HMAC-SHA1(authKey, buffer[0..len) || u32_be(rocIn)).  Reference mode re-keys
 * on every packet (OpenSSLHMAC.doFinal -> reset -> HMAC_Init_ex with the key,
 * OpenSSLHMAC.java:222,293-318). */
static void authenticate_packet_hmac(orc_ctx *x, const uint8_t *buf, int len, int32_t roc_in) {
    uint8_t rb[4] = {(uint8_t)(roc_in >> 24), (uint8_t)(roc_in >> 16), (uint8_t)(roc_in >> 8),
                     (uint8_t)roc_in};
    if (x->policy.auth_type == ORC_SKEIN_AUTHENTICATION) {
        /* the same update/update/doFinal sequence on bccontrib's SkeinMac; doFinal
         * resets it to the keyed, configured state (skein.c) */
        sk_update(&x->skein, buf, (size_t)len);
        sk_update(&x->skein, rb, 4);
        sk_final(&x->skein, x->tag_store);
        return;
    }
    unsigned int ol = 20;
    HMAC_CTX *h;
    if (x->mode == ORC_MODE_TUNED) {
        h = x->hmac_work;
        HMAC_CTX_copy(h, x->hmac);
    } else {
        h = x->hmac;
        HMAC_Init_ex(h, x->auth_key, 20, EVP_sha1(), NULL);
    }
    HMAC_Update(h, buf, (size_t)len);
    HMAC_Update(h, rb, 4);
    HMAC_Final(h, x->tag_store, &ol);
}

/* RFC 3711 4.3 PRF as SRTPCryptoContext.computeIv/deriveSrtpKeys
 * (:333-359, :393-447; kdr == 0 so key_id = label << 48, i.e. only IV byte 7
 * is XORed with the label) and SRTCPCryptoContext.computeIv/deriveSrtcpKeys
 * (:128-136, :158-211). */
void orc_derive_keys(const uint8_t mk[16], const uint8_t ms[14], int rtcp, uint8_t enc[16],
                     uint8_t auth[20], uint8_t salt[14]) {
    orc_derive_keys_n(mk, 16, ms, rtcp, enc, auth, salt);
}

/* deriveSrtpKeys :393-447 / deriveSrtcpKeys with a master key of key_len
 * bytes: the PRF is AES-128 or AES-256 (RFC 6188 4.1), the session key key_len
 * bytes. */
static void derive_keys_prf(int twofish, const uint8_t *mk, int key_len, const uint8_t ms[14],
                            int rtcp, uint8_t *enc, uint8_t *auth, int auth_len, uint8_t salt[14]);

void orc_derive_keys_n(const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                       uint8_t *enc, uint8_t auth[20], uint8_t salt[14]) {
    derive_keys_prf(0, mk, key_len, ms, rtcp, enc, auth, 20, salt);
}

/* with the policy's auth key length (32 for ZRTP's Skein, ZRTPTransformEngine.java:867-872) */
void orc_derive_keys_auth(int twofish, const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                          uint8_t *enc, uint8_t *auth, int auth_len, uint8_t salt[14]) {
    derive_keys_prf(twofish, mk, key_len, ms, rtcp, enc, auth, auth_len, salt);
}

/* the chaining value after the key (if any) and config UBIs: for key_len 0
 * the paper's precomputed IV of Skein-512-out_bits */
void orc_skein512_state0(const uint8_t *key, int key_len, int out_bits, uint64_t g0[8]) {
    sk_ctx c;
    sk_init(&c, key, key_len, out_bits);
    memcpy(g0, c.g0, sizeof c.g0);
    memset(&c, 0, sizeof c);
}

void orc_skein512_mac(const uint8_t *key, int key_len, int out_bits, const uint8_t *msg, size_t n,
                      uint8_t *out) {
    sk_ctx c;
    sk_init(&c, key, key_len, out_bits);
    sk_update(&c, msg, n);
    sk_final(&c, out);
    memset(&c, 0, sizeof c);
}

/* Twofish policies: deriveSrtpKeys keys the TwofishEngine `cipher` with the
 * master key, so the PRF is Twofish (BaseSRTPCryptoContext :217-225). */
void orc_derive_keys_twofish(const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                             uint8_t *enc, uint8_t auth[20], uint8_t salt[14]) {
    derive_keys_prf(1, mk, key_len, ms, rtcp, enc, auth, 20, salt);
}

static void derive_keys_prf(int twofish, const uint8_t *mk, int key_len, const uint8_t ms[14],
                            int rtcp, uint8_t *enc, uint8_t *auth, int auth_len, uint8_t salt[14]) {
    blk_t *c = blk_new(twofish, mk, key_len);
    uint8_t iv[16];
    int base = rtcp ? 3 : 0;
    for (int lab = 0; lab < 3; lab++) {
        memcpy(iv, ms, 14);
        iv[7] ^= (uint8_t)(base + lab);
        iv[14] = iv[15] = 0;
        if (lab == 0)
            get_cipher_stream(c, enc, key_len, iv);
        else if (lab == 1)
            get_cipher_stream(c, auth, auth_len, iv);
        else
            get_cipher_stream(c, salt, 14, iv);
    }
    blk_free(c);
}

/* ---------- RawPacket accessors (nm/RawPacket.java) --------------------- */
static inline int32_t read_int(const uint8_t *b, int o) { /* :951-957 */
    return (int32_t)(((uint32_t)b[o] << 24) | ((uint32_t)b[o + 1] << 16) |
                     ((uint32_t)b[o + 2] << 8) | b[o + 3]);
}
static inline int read_u16(const uint8_t *b, int o) { return (b[o] << 8) | b[o + 1]; } /* :1069 */

/* getHeaderLength :602-614 + getExtensionLength :544-556 (signed high byte).
 * Reading the extension length past the buffer throws. */
static int header_length(const uint8_t *b, int buf_len, int *h) {
    int cc = b[0] & 0x0f;
    int hl = 12 + 4 * cc;
    if ((b[0] & 0x10) == 0x10) {
        int idx = 12 + cc * 4 + 2;
        if (idx + 1 >= buf_len)
            return THROW;
        int ext = ((int)(int8_t)b[idx] * 256) | (b[idx + 1] & 0xFF);
        hl += 4 + ext * 4;
    }
    *h = hl;
    return 0;
}

/* ---------- context map ------------------------------------------------- */
static uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

static void map_init(ctx_map *m) {
    m->cap = 64; m->count = 0;
    m->keys = (uint32_t *)calloc(m->cap, sizeof(uint32_t));
    m->vals = (orc_ctx **)calloc(m->cap, sizeof(orc_ctx *));
}

static orc_ctx *map_get(ctx_map *m, uint32_t k) {
    uint32_t mask = m->cap - 1;
    for (uint32_t i = mix32(k) & mask;; i = (i + 1) & mask) {
        if (!m->vals[i]) return NULL;
        if (m->keys[i] == k) return m->vals[i];
    }
}

static void map_put(ctx_map *m, uint32_t k, orc_ctx *v);
static void map_grow(ctx_map *m) {
    ctx_map n;
    n.cap = m->cap * 2; n.count = 0;
    n.keys = (uint32_t *)calloc(n.cap, sizeof(uint32_t));
    n.vals = (orc_ctx **)calloc(n.cap, sizeof(orc_ctx *));
    for (uint32_t i = 0; i < m->cap; i++)
        if (m->vals[i]) map_put(&n, m->keys[i], m->vals[i]);
    free(m->keys); free(m->vals);
    *m = n;
}

static void map_put(ctx_map *m, uint32_t k, orc_ctx *v) {
    if (2 * (m->count + 1) > m->cap) map_grow(m);
    uint32_t mask = m->cap - 1;
    uint32_t i = mix32(k) & mask;
    while (m->vals[i]) i = (i + 1) & mask;
    m->keys[i] = k; m->vals[i] = v; m->count++;
}

static void ctx_free(orc_ctx *x) {
    if (!x) return;
    blk_free(x->ecb);
    if (x->ctr) EVP_CIPHER_CTX_free(x->ctr);
    blk_free(x->f8);
    if (x->hmac) HMAC_CTX_free(x->hmac);
    if (x->hmac_work) HMAC_CTX_free(x->hmac_work);
    memset(x, 0, sizeof *x);
    free(x);
}

static void map_clear(ctx_map *m) {
    for (uint32_t i = 0; i < m->cap; i++) {
        ctx_free(m->vals[i]);
        m->vals[i] = NULL;
    }
    m->count = 0;
}

/* ---------- factory / transformer -------------------------------------- */
static int policy_ok(const orc_policy *p, int rtcp) {
    if (p->enc_type != ORC_NULL_ENCRYPTION && !is_ctr(p->enc_type) && !is_f8(p->enc_type))
        return 0;
    if (p->enc_type != ORC_NULL_ENCRYPTION && p->salt_key_len != 14) return 0;
    if (p->enc_type == ORC_AESF8_ENCRYPTION && p->enc_key_len != 16) return 0;
    if ((p->enc_type == ORC_AESCM_ENCRYPTION || is_twofish(p->enc_type)) && p->enc_key_len != 16 &&
        p->enc_key_len != 32)
        return 0;
    /* SRTCP F8 ciphers [8, 8 + length - 4 - tag) (SRTCPCryptoContext :285-291),
     * which leaves the packet unless an HMAC trailer of >= 4 tag bytes follows */
    if (rtcp && is_f8(p->enc_type) &&
        (p->auth_type == ORC_NULL_AUTHENTICATION || p->auth_tag_len < 4))
        return 0;
    if (p->auth_type != ORC_NULL_AUTHENTICATION && p->auth_type != ORC_HMACSHA1_AUTHENTICATION &&
        p->auth_type != ORC_SKEIN_AUTHENTICATION)
        return 0;
    if (p->auth_type == ORC_HMACSHA1_AUTHENTICATION && p->auth_key_len != 20) return 0;
    /* Skein: a key of one UBI block at most, and a tag of >= 1 byte (the MAC's
     * output length is tag_len * 8 bits, SRTPCryptoContext.java:421-428) */
    if (p->auth_type == ORC_SKEIN_AUTHENTICATION &&
        (p->auth_key_len < 1 || p->auth_key_len > 64 || p->auth_tag_len < 1))
        return 0;
    /* <= 12 keeps readRegionToBuff in range for every packet of >= 12 bytes */
    if (p->auth_tag_len < 0 || p->auth_tag_len > 12) return 0;
    return 1;
}

orc_factory *orc_factory_new(int sender, const uint8_t *mk, int key_len, const uint8_t *ms,
                             int salt_len, const orc_policy *srtp, const orc_policy *srtcp,
                             int mode) {
    /* NULL-cipher profiles: the reference throws in key derivation;
     * here they keep a 16-B master key + 14-B salt for the AES-CM PRF, as RFC 3711
     * 4.3 prescribes -- behaviour "parity unpinned". */
    if (salt_len < 14 || !policy_ok(srtp, 0) || !policy_ok(srtcp, 1)) return NULL;
    /* BaseSRTPCryptoContext copies encKeyLength bytes of the master key (:187-190) */
    const int need = (srtp->enc_type != ORC_NULL_ENCRYPTION && srtp->enc_key_len == 32) ||
                     (srtcp->enc_type != ORC_NULL_ENCRYPTION && srtcp->enc_key_len == 32) ? 32 : 16;
    if (key_len < need) return NULL;
    orc_factory *f = (orc_factory *)calloc(1, sizeof *f);
    f->sender = sender; f->mode = mode;
    memcpy(f->master_key, mk, (size_t)need);
    memcpy(f->master_salt, ms, 14);
    f->srtp = *srtp; f->srtcp = *srtcp;
    return f;
}

/* SRTPContextFactory.close :74-86 (zeroes master keys, default contexts null) */
void orc_factory_close(orc_factory *f) {
    if (!f || f->closed) return;
    f->closed = 1;
    memset(f->master_key, 0, sizeof f->master_key);
    memset(f->master_salt, 0, 14);
}

orc_transformer *orc_transformer_new(int kind, orc_factory *fwd, orc_factory *rev) {
    orc_transformer *t = (orc_transformer *)calloc(1, sizeof *t);
    t->kind = kind; t->fwd = fwd; t->rev = rev;
    map_init(&t->map);
    return t;
}

/* SRTPTransformer.setContextFactory :100-125 / SRTCPTransformer.updateFactory :92-117 */
void orc_transformer_set_factory(orc_transformer *t, orc_factory *f, int forward) {
    orc_factory **slot = forward ? &t->fwd : &t->rev;
    if (*slot && *slot != f) orc_factory_close(*slot);
    *slot = f;
}

/* SRTPTransformer.close :132-150 */
void orc_transformer_close(orc_transformer *t) {
    orc_factory_close(t->fwd);
    if (t->rev != t->fwd) orc_factory_close(t->rev);
    map_clear(&t->map);
}

void orc_transformer_free(orc_transformer *t) {
    if (!t) return;
    map_clear(&t->map);
    free(t->map.keys); free(t->map.vals);
    free(t);
}

/* SRTPTransformer.getContext :152-175 / SRTCPTransformer.getContext :144-167:
 * lazily derive a context from the factory's default context (roc 0, kdr 0 ->
 * the session keys depend only on the master key/salt and the label). */
static orc_ctx *make_context(orc_transformer *t, uint32_t ssrc, orc_factory *f) {
    orc_ctx *x = (orc_ctx *)calloc(1, sizeof *x);
    x->ssrc = ssrc; x->kind = t->kind; x->mode = f->mode;
    x->policy = (t->kind == ORC_KIND_RTP) ? f->srtp : f->srtcp;
    const int tf = is_twofish(x->policy.enc_type);
    x->key_len = x->policy.enc_type != ORC_NULL_ENCRYPTION && x->policy.enc_key_len == 32 ? 32 : 16;
    const int skein = x->policy.auth_type == ORC_SKEIN_AUTHENTICATION;
    const int auth_len = skein ? x->policy.auth_key_len : 20;
    derive_keys_prf(tf, f->master_key, x->key_len, f->master_salt, t->kind == ORC_KIND_RTCP,
                    x->enc_key, x->auth_key, auth_len, x->salt_key);
    if (skein) sk_init(&x->skein, x->auth_key, auth_len, 8 * x->policy.auth_tag_len);
    x->ecb = blk_new(tf, x->enc_key, x->key_len);
    if (is_f8(x->policy.enc_type)) /* deriveSrtpKeys :443-444 */
        x->f8 = f8_iv_cipher_new(tf, x->enc_key, x->key_len, x->salt_key, 14);
    if (x->mode == ORC_MODE_TUNED && !tf) {
        x->ctr = EVP_CIPHER_CTX_new();
        EVP_EncryptInit_ex(x->ctr, x->key_len == 32 ? EVP_aes_256_ctr() : EVP_aes_128_ctr(), NULL,
                           x->enc_key, NULL);
    }
    x->hmac = HMAC_CTX_new();
    x->hmac_work = HMAC_CTX_new();
    HMAC_Init_ex(x->hmac, x->auth_key, 20, EVP_sha1(), NULL);
    return x;
}

static orc_ctx *get_context(orc_transformer *t, uint32_t ssrc, orc_factory *f) {
    orc_ctx *x = map_get(&t->map, ssrc);
    if (x) return x;
    if (!f || f->closed) return NULL;
    x = make_context(t, ssrc, f);
    map_put(&t->map, ssrc, x);
    return x;
}

/* ---------- SRTPCryptoContext ------------------------------------------ */
/* guessIndex :457-475 */
static int64_t guess_index(orc_ctx *x, int seq) {
    if (x->s_l < 32768)
        x->guessed_roc = (seq - x->s_l > 32768) ? j_sub(x->roc, 1) : x->roc;
    else
        x->guessed_roc = (x->s_l - 32768 > seq) ? j_add(x->roc, 1) : x->roc;
    return j_lshl((int64_t)x->guessed_roc, 16) | seq;
}

/* checkReplay :279-323 */
static int srtp_check_replay(orc_ctx *x, int64_t guessed_index) {
    if (!g_check_replay) return 1;
    int64_t local = j_lshl((int64_t)x->roc, 16) | x->s_l;
    int64_t delta = guessed_index - local;
    if (delta > 0) return 1;
    if (-delta > 64) return 0;
    if (j_lbit(x->replay_window, -delta)) return 0;
    return 1;
}

/* update :719-744 (note: `1 << -delta` is an int shift, sign-extended) */
static void srtp_update(orc_ctx *x, int seq, int64_t guessed_index) {
    int64_t delta = guessed_index - (j_lshl((int64_t)x->roc, 16) | x->s_l);
    if (delta > 0) {
        x->replay_window = j_lshl(x->replay_window, delta);
        x->replay_window |= 1;
    } else {
        x->replay_window |= (int64_t)j_ishl1(-delta);
    }
    if (x->guessed_roc == x->roc) {
        if (seq > x->s_l) x->s_l = seq & 0xffff;
    } else if (x->guessed_roc == j_add(x->roc, 1)) {
        x->s_l = seq & 0xffff;
        x->roc = x->guessed_roc;
    }
}

/* processPacketAESCM :482-525 */
static int srtp_process_aescm(orc_ctx *x, uint8_t *b, int len, int cap) {
    int32_t ssrc = read_int(b, 8);
    int seq = read_u16(b, 2);
    int64_t index = j_lshl((int64_t)x->guessed_roc, 16) | seq;
    uint8_t iv[16];
    for (int i = 0; i < 4; i++) iv[i] = x->salt_key[i];
    for (int i = 4; i < 8; i++) iv[i] = (uint8_t)((0xFF & (ssrc >> ((7 - i) * 8))) ^ x->salt_key[i]);
    for (int i = 8; i < 14; i++)
        iv[i] = (uint8_t)((0xFF & (uint8_t)(index >> ((13 - i) * 8))) ^ x->salt_key[i]);
    iv[14] = iv[15] = 0;
    int h;
    if (header_length(b, cap, &h) == THROW) return THROW;
    int payload_len = len - h; /* RawPacket.getPayloadLength :723-729 */
    return cipher_ctr_process(x, b, cap, h, payload_len, iv);
}

/* processPacketAESF8 :532-555: IV = 0x00 || header bytes 1..11 || ROC_be. */
static int srtp_process_aesf8(orc_ctx *x, uint8_t *b, int len, int cap) {
    uint8_t iv[16];
    memcpy(iv, b, 12);
    iv[0] = 0;
    int32_t roc = x->guessed_roc;
    iv[12] = (uint8_t)(roc >> 24); iv[13] = (uint8_t)(roc >> 16);
    iv[14] = (uint8_t)(roc >> 8);  iv[15] = (uint8_t)roc;
    int h;
    if (header_length(b, cap, &h) == THROW) return THROW;
    return cipher_f8_process(x->ecb, x->f8, b, h, len - h, iv);
}

static int srtp_encrypt(orc_ctx *x, uint8_t *b, int len, int cap) {
    if (is_ctr(x->policy.enc_type)) return srtp_process_aescm(x, b, len, cap);
    if (is_f8(x->policy.enc_type)) return srtp_process_aesf8(x, b, len, cap);
    return 0;
}

/* transformPacket :658-705 */
static int srtp_transform(orc_ctx *x, uint8_t *b, uint32_t *len, int cap) {
    int L = (int)*len;
    int seq = read_u16(b, 2);
    if (!x->seq_num_set) { x->seq_num_set = 1; x->s_l = seq; }
    int64_t gi = guess_index(x, seq);
    if (!srtp_check_replay(x, gi)) return ORC_DROP_REPLAY;
    if (srtp_encrypt(x, b, L, cap) == THROW) return ORC_ERR_MALFORMED;
    if (x->policy.auth_type != ORC_NULL_AUTHENTICATION) {
        authenticate_packet_hmac(x, b, L, x->guessed_roc);
        int T = x->policy.auth_tag_len;
        if (T > 0) { memcpy(b + L, x->tag_store, (size_t)T); L += T; } /* RawPacket.append */
    }
    srtp_update(x, seq, gi);
    *len = (uint32_t)L;
    return ORC_OK;
}

/* authenticatePacket :237-266 (readRegionToBuff :988-999, shrink :1284-1292) */
static int srtp_authenticate(orc_ctx *x, uint8_t *b, int *L, int cap) {
    if (x->policy.auth_type == ORC_NULL_AUTHENTICATION) return 1;
    int T = x->policy.auth_tag_len;
    int o = *L - T;
    if (!(o < 0 || T <= 0 || o + T > cap || (int)sizeof x->temp_store < T))
        memcpy(x->temp_store, b + o, (size_t)T);
    if (T > 0) { *L -= T; if (*L < 0) *L = 0; }
    authenticate_packet_hmac(x, b, *L, x->guessed_roc);
    for (int i = 0; i < T; i++)
        if (x->temp_store[i] != x->tag_store[i]) return 0;
    return 1;
}

/* reverseTransformPacket :572-642 */
static int srtp_reverse(orc_ctx *x, uint8_t *b, uint32_t *len, int cap, uint32_t flags) {
    int L = (int)*len;
    int seq = read_u16(b, 2);
    if (!x->seq_num_set) { x->seq_num_set = 1; x->s_l = seq; }
    int64_t gi = guess_index(x, seq);
    if (!srtp_check_replay(x, gi)) return ORC_DROP_REPLAY;
    int ok = srtp_authenticate(x, b, &L, cap);
    *len = (uint32_t)L;
    if (!ok) return ORC_DROP_AUTH;
    if ((flags & (ORC_FLAG_DISCARD | ORC_FLAG_SILENCE)) == 0)
        if (srtp_encrypt(x, b, L, cap) == THROW) return ORC_ERR_MALFORMED;
    srtp_update(x, seq, gi);
    return ORC_OK;
}

/* ---------- SRTCPCryptoContext ----------------------------------------- */
/* checkReplay :106-120 (int subtraction widened to long; not config-gated) */
static int srtcp_check_replay(orc_ctx *x, int32_t index) {
    int64_t delta = (int64_t)j_sub(index, x->received_index);
    if (delta > 0) return 1;
    if (-delta > 64) return 0;
    if (j_lbit(x->replay_window, -delta)) return 0;
    return 1;
}

/* update :435-451 (reversed delta; int shift in the else branch) */
static void srtcp_update(orc_ctx *x, int32_t index) {
    int32_t delta = j_sub(x->received_index, index);
    if (delta > 0) {
        x->replay_window = j_lshl(x->replay_window, delta);
        x->replay_window |= 1;
    } else {
        x->replay_window |= (int64_t)j_ishl1(delta);
    }
    x->received_index = index;
}

/* processPacketAESCM :218-260 (encrypts [8, length)) */
static int srtcp_process_aescm(orc_ctx *x, uint8_t *b, int L, int cap, int32_t index) {
    int32_t ssrc = read_int(b, 4);
    uint8_t iv[16];
    for (int i = 0; i < 4; i++) iv[i] = x->salt_key[i];
    iv[4] = (uint8_t)(((ssrc >> 24) & 0xff) ^ x->salt_key[4]);
    iv[5] = (uint8_t)(((ssrc >> 16) & 0xff) ^ x->salt_key[5]);
    iv[6] = (uint8_t)(((ssrc >> 8) & 0xff) ^ x->salt_key[6]);
    iv[7] = (uint8_t)((ssrc & 0xff) ^ x->salt_key[7]);
    iv[8] = x->salt_key[8];
    iv[9] = x->salt_key[9];
    iv[10] = (uint8_t)(((index >> 24) & 0xff) ^ x->salt_key[10]);
    iv[11] = (uint8_t)(((index >> 16) & 0xff) ^ x->salt_key[11]);
    iv[12] = (uint8_t)(((index >> 8) & 0xff) ^ x->salt_key[12]);
    iv[13] = (uint8_t)((index & 0xff) ^ x->salt_key[13]);
    iv[14] = iv[15] = 0;
    return cipher_ctr_process(x, b, cap, 8, L - 8, iv);
}

/* processPacketAESF8 :267-298: IV = 0 (4 B) || (index | E)_be || packet bytes
 * 0..7; ciphers [8, 8 + length - (4 + tag)) of the length at the call (before
 * the trailer on protect, after shrinking it on unprotect). */
static int srtcp_process_aesf8(orc_ctx *x, uint8_t *b, int L, int32_t index) {
    uint8_t iv[16] = {0};
    uint32_t ie = (uint32_t)index | 0x80000000u;
    iv[4] = (uint8_t)(ie >> 24); iv[5] = (uint8_t)(ie >> 16);
    iv[6] = (uint8_t)(ie >> 8);  iv[7] = (uint8_t)ie;
    memcpy(iv + 8, b, 8);
    return cipher_f8_process(x->ecb, x->f8, b, 8, L - (4 + x->policy.auth_tag_len), iv);
}

/* transformPacket :391-427 */
static int srtcp_transform(orc_ctx *x, uint8_t *b, uint32_t *len, int cap) {
    int L = (int)*len;
    int encrypt = 0;
    if (is_ctr(x->policy.enc_type)) {
        if (srtcp_process_aescm(x, b, L, cap, x->sent_index) == THROW) return ORC_ERR_MALFORMED;
        encrypt = 1;
    } else if (is_f8(x->policy.enc_type)) {
        if (srtcp_process_aesf8(x, b, L, x->sent_index) == THROW) return ORC_ERR_MALFORMED;
        encrypt = 1;
    }
    int32_t index = encrypt ? (int32_t)((uint32_t)x->sent_index | 0x80000000u) : 0;
    if (x->policy.auth_type != ORC_NULL_AUTHENTICATION) {
        authenticate_packet_hmac(x, b, L, index);
        int T = x->policy.auth_tag_len;
        b[L] = (uint8_t)(index >> 24); b[L + 1] = (uint8_t)(index >> 16);
        b[L + 2] = (uint8_t)(index >> 8); b[L + 3] = (uint8_t)index;
        L += 4;
        if (T > 0) { memcpy(b + L, x->tag_store, (size_t)T); L += T; }
    }
    x->sent_index = j_add(x->sent_index, 1);
    x->sent_index &= 0x7FFFFFFF;
    *len = (uint32_t)L;
    return ORC_OK;
}

/* reverseTransformPacket :315-374 */
static int srtcp_reverse(orc_ctx *x, uint8_t *b, uint32_t *len, int cap) {
    int L = (int)*len;
    int T = x->policy.auth_tag_len;
    int io = L - (4 + T); /* RawPacket.getSRTCPIndex :815-819 */
    if (io < 0) return ORC_ERR_MALFORMED;
    int32_t index_e = read_int(b, io);
    int decrypt = (index_e & (int32_t)0x80000000) == (int32_t)0x80000000;
    int32_t index = index_e & 0x7FFFFFFF;
    if (!srtcp_check_replay(x, index)) return ORC_DROP_REPLAY;
    if (x->policy.auth_type != ORC_NULL_AUTHENTICATION) {
        int o = L - T;
        if (!(o < 0 || T <= 0 || o + T > cap || (int)sizeof x->temp_store < T))
            memcpy(x->temp_store, b + o, (size_t)T);
        L -= T + 4;
        if (L < 0) L = 0;
        *len = (uint32_t)L;
        authenticate_packet_hmac(x, b, L, index_e);
        for (int i = 0; i < T; i++)
            if (x->temp_store[i] != x->tag_store[i]) return ORC_DROP_AUTH;
    }
    if (decrypt && is_ctr(x->policy.enc_type))
        if (srtcp_process_aescm(x, b, L, cap, index) == THROW) return ORC_ERR_MALFORMED;
    if (decrypt && is_f8(x->policy.enc_type))
        if (srtcp_process_aesf8(x, b, L, index) == THROW) return ORC_ERR_MALFORMED;
    srtcp_update(x, index);
    return ORC_OK;
}

/* ---------- transformer-level batch ------------------------------------ */
/* One packet through SRTPTransformer / SRTCPTransformer (.transform :211-219,
 * .reverseTransform :185-202; SRTCP :176-207). */
static int process_one(orc_transformer *t, int reverse, uint8_t *b, uint32_t *len, int cap,
                       uint32_t flags) {
    int L = (int)*len;
    if (L < 12 || L > cap) return ORC_DROP_INVALID; /* RawPacket.isInvalid :903-909 */
    if (t->kind == ORC_KIND_RTP) {
        if (reverse && (b[0] & 0xC0) != 0x80) return ORC_DROP_VERSION;
        uint32_t ssrc = (uint32_t)read_int(b, 8);
        orc_ctx *x = get_context(t, ssrc, reverse ? t->rev : t->fwd);
        if (!x) return ORC_DROP_NO_CONTEXT;
        if (!reverse) {
            int T = (x->policy.auth_type != ORC_NULL_AUTHENTICATION) ? x->policy.auth_tag_len : 0;
            if (L + T > cap) return ORC_ERR_CAPACITY;
            return srtp_transform(x, b, len, cap);
        }
        return srtp_reverse(x, b, len, cap, flags);
    } else {
        uint32_t ssrc = (uint32_t)read_int(b, 4);
        orc_ctx *x = get_context(t, ssrc, reverse ? t->rev : t->fwd);
        if (!x) return ORC_DROP_NO_CONTEXT;
        if (!reverse) {
            int T = (x->policy.auth_type != ORC_NULL_AUTHENTICATION) ? 4 + x->policy.auth_tag_len : 0;
            if (L + T > cap) return ORC_ERR_CAPACITY;
            return srtcp_transform(x, b, len, cap);
        }
        return srtcp_reverse(x, b, len, cap);
    }
}

/* SinglePacketTransformer.transform/reverseTransform(RawPacket[]) :121-216:
 * array order; a Throwable aborts the remaining elements of that call. */
int orc_process(orc_transformer *const *ts, int ts_stride, int reverse, uint8_t *seg,
                const uint32_t *off, uint32_t *len, const uint32_t *cap, const uint32_t *flags,
                int32_t *status, uint32_t n, int abort_on_error) {
    orc_transformer *aborted_small[64];
    uint32_t n_aborted = 0, aborted_cap = 64;
    orc_transformer **aborted = aborted_small;
    for (uint32_t i = 0; i < n; i++) {
        orc_transformer *t = ts[ts_stride ? i : 0];
        uint32_t fl = flags ? flags[i] : 0;
        if (fl & (uint32_t)ORC_FLAG_SKIP || !t) { status[i] = ORC_SKIPPED; continue; }
        int dead = 0;
        for (uint32_t k = 0; k < n_aborted; k++)
            if (aborted[k] == t) { dead = 1; break; }
        if (dead) { status[i] = ORC_NOT_PROCESSED; continue; }
        int st = process_one(t, reverse, seg + off[i], &len[i], (int)cap[i], fl);
        status[i] = st;
        if (st == ORC_ERR_MALFORMED && abort_on_error) {
            if (n_aborted == aborted_cap) {
                orc_transformer **na =
                    (orc_transformer **)malloc(sizeof(*na) * (size_t)aborted_cap * 2);
                memcpy(na, aborted, sizeof(*na) * n_aborted);
                if (aborted != aborted_small) free(aborted);
                aborted = na; aborted_cap *= 2;
            }
            aborted[n_aborted++] = t;
        }
    }
    if (aborted != aborted_small) free(aborted);
    return 0;
}

int orc_get_state(orc_transformer *t, uint32_t ssrc, orc_ctx_state *out) {
    orc_ctx *x = map_get(&t->map, ssrc);
    if (!x) return 0;
    out->roc = x->roc; out->s_l = x->s_l; out->seq_num_set = x->seq_num_set;
    out->guessed_roc = x->guessed_roc;
    out->sent_index = x->sent_index; out->received_index = x->received_index;
    out->replay_window = (uint64_t)x->replay_window;
    return 1;
}

uint32_t orc_num_contexts(orc_transformer *t) { return t->map.count; }

/* Context-state export / import (the engine's srtp_export_contexts /
 * srtp_set_context_state; the reference has no such API -- the state is the
 * private fields of SRTPCryptoContext :96-135 / SRTCPCryptoContext :54-59).
 * Export: up to max (ssrc, state) pairs in map order, returns the count held. */
uint32_t orc_export_contexts(orc_transformer *t, uint32_t *ssrcs, orc_ctx_state *states, uint32_t max) {
    uint32_t n = 0;
    for (uint32_t i = 0; i < t->map.cap; i++) {
        if (!t->map.vals[i]) continue;
        if (n < max) {
            ssrcs[n] = t->map.keys[i];
            orc_get_state(t, t->map.keys[i], &states[n]);
        }
        n++;
    }
    return n;
}

/* Import: create or replace the context for ssrc, keyed by the transformer's
 * forward or reverse factory (which must be open), with the given state.
 * Returns 0, or -1 when that factory is closed. */
int orc_set_context_state(orc_transformer *t, uint32_t ssrc, int forward, const orc_ctx_state *st) {
    orc_factory *f = forward ? t->fwd : t->rev;
    if (!f || f->closed) return -1;
    orc_ctx *x = make_context(t, ssrc, f);
    x->roc = st->roc; x->s_l = st->s_l; x->seq_num_set = st->seq_num_set;
    x->guessed_roc = st->guessed_roc;
    x->sent_index = st->sent_index; x->received_index = st->received_index;
    x->replay_window = (int64_t)st->replay_window;
    const uint32_t mask = t->map.cap - 1;
    for (uint32_t i = mix32(ssrc) & mask;; i = (i + 1) & mask) {
        if (!t->map.vals[i]) break;
        if (t->map.keys[i] == ssrc) {
            ctx_free(t->map.vals[i]);
            t->map.vals[i] = x;
            return 0;
        }
    }
    map_put(&t->map, ssrc, x);
    return 0;
}

/* Removes the context for ssrc (backward-shift deletion keeps every probe
 * path intact).  Returns 1 if there was one.  Test infrastructure: the
 * sharded-dispatch rehearsal (tests/test_dispatch_dist.py) rolls contexts
 * back to their state before a bundle, which may be "absent". */
int orc_remove_context(orc_transformer *t, uint32_t ssrc) {
    ctx_map *m = &t->map;
    const uint32_t mask = m->cap - 1;
    uint32_t i = mix32(ssrc) & mask;
    for (;; i = (i + 1) & mask) {
        if (!m->vals[i]) return 0;
        if (m->keys[i] == ssrc) break;
    }
    ctx_free(m->vals[i]);
    m->vals[i] = NULL;
    m->count--;
    for (uint32_t j = (i + 1) & mask; m->vals[j]; j = (j + 1) & mask) {
        const uint32_t h = mix32(m->keys[j]) & mask;
        /* entry j may move to the hole i unless its home h lies in (i, j] */
        const int stays = i <= j ? (h > i && h <= j) : (h > i || h <= j);
        if (stays) continue;
        m->keys[i] = m->keys[j];
        m->vals[i] = m->vals[j];
        m->vals[j] = NULL;
        i = j;
    }
    return 1;
}

/* RFC 5705 keying-material exporter (no context value) over the TLS PRF, via
 * OpenSSL's TLS1-PRF KDF: the checker for the engine's
 * srtp_tls_export_keying_material (what BouncyCastle's
 * TlsContext.exportKeyingMaterial does for DtlsPacketTransformer.java:614-617).
 * prf 0: TLS 1.0/1.1 (MD5-SHA1), 1: TLS 1.2 (SHA256).  Returns 0 on success. */
int orc_tls_export(int prf, const uint8_t *secret, int secret_len, const uint8_t cr[32],
                   const uint8_t sr[32], const char *label, uint8_t *out, int out_len) {
    EVP_KDF *kdf = EVP_KDF_fetch(NULL, "TLS1-PRF", NULL);
    if (!kdf) return -1;
    EVP_KDF_CTX *kc = EVP_KDF_CTX_new(kdf);
    EVP_KDF_free(kdf);
    if (!kc) return -1;
    size_t ll = strlen(label);
    uint8_t *seed = (uint8_t *)malloc(ll + 64);
    memcpy(seed, label, ll);
    memcpy(seed + ll, cr, 32);
    memcpy(seed + ll + 32, sr, 32);
    OSSL_PARAM ps[4];
    ps[0] = OSSL_PARAM_construct_utf8_string(OSSL_KDF_PARAM_DIGEST, prf ? (char *)"SHA256" : (char *)"MD5-SHA1", 0);
    ps[1] = OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_SECRET, (void *)secret, (size_t)secret_len);
    ps[2] = OSSL_PARAM_construct_octet_string(OSSL_KDF_PARAM_SEED, seed, ll + 64);
    ps[3] = OSSL_PARAM_construct_end();
    int rc = EVP_KDF_derive(kc, out, (size_t)out_len, ps) == 1 ? 0 : -1;
    EVP_KDF_CTX_free(kc);
    free(seed);
    return rc;
}
