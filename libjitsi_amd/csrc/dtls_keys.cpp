// dtls_keys.cpp -- DTLS-SRTP keying (control plane, host only).
//
// The reference turns a finished DTLS handshake into SRTP contexts in
// DtlsPacketTransformer.initializeSRTPTransformer
// (transform/dtls/DtlsPacketTransformer.java:549-690):
//   1. the negotiated protection profile fixes key / salt / tag lengths
//      (:574-612; the _32 profiles keep a 10-byte SRTCP tag);
//   2. 2 * (key + salt) bytes are exported from the TLS context with the
//      RFC 5705 label "EXTRACTOR-dtls_srtp" and no context value (:614-617);
//   3. the bytes split as client key | server key | client salt | server salt
//      (:618-638, RFC 5764 4.2);
//   4. a client factory (sender iff this side is the TLS client) and a server
//      factory are built, and the transformer's forward factory is this side's
//      own one, reverse the peer's (:639-680).
// Step 2 runs inside BouncyCastle's TlsContext.exportKeyingMaterial; here it is
// srtp_tls_export_keying_material over the TLS PRF of RFC 2246 5 (DTLS 1.0,
// which the reference negotiates: TlsClientImpl.java:148-155, TlsServerImpl.java
// :167-174 -- MD5 xor SHA-1) or RFC 5246 5 (DTLS 1.2, P_SHA256).  Steps 1, 3
// and 4 are srtp_dtls_profile_keys and srtp_dtls_transformer_create.
#include <string.h>

#include <vector>

#include "../../include/srtp_mi355x.h"
#include "host_crypto.h"

namespace {

inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
inline uint32_t rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// MD5 compression (RFC 1321 3.4) of one 64-byte block.
void md5_compress(uint32_t h[4], const uint8_t blk[64]) {
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    uint32_t m[16];
    for (int i = 0; i < 16; i++)
        m[i] = blk[4 * i] | (uint32_t)blk[4 * i + 1] << 8 | (uint32_t)blk[4 * i + 2] << 16 |
               (uint32_t)blk[4 * i + 3] << 24;
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g, r = i >> 4;
        if (r == 0) { f = (b & c) | (~b & d); g = i; }
        else if (r == 1) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (r == 2) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
        else { f = c ^ (b | ~d); g = (7 * i) & 15; }
        uint32_t t = d;
        d = c;
        c = b;
        b = b + rotl(a + f + K[i] + m[g], S[r * 4 + (i & 3)]);
        a = t;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}

// SHA-256 compression (FIPS 180-4 6.2.2) of one 64-byte block.
void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
    static const uint32_t K[64] = {
        0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4,
        0xab1c5ed5, 0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe,
        0x9bdc06a7, 0xc19bf174, 0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f,
        0x4a7484aa, 0x5cb0a9dc, 0x76f988da, 0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7,
        0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967, 0x27b70a85, 0x2e1b2138, 0x4d2c6dfc,
        0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85, 0xa2bfe8a1, 0xa81a664b,
        0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070, 0x19a4c116,
        0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
        0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7,
        0xc67178f2};
    uint32_t w[64];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 |
               (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = rotr(w[i - 15], 7) ^ rotr(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = rotr(w[i - 2], 17) ^ rotr(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = hh + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
        uint32_t t2 = (rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

enum HashKind { kMd5, kSha1, kSha256 };

// One-shot Merkle-Damgard hash over a byte string (64-byte blocks for all three).
std::vector<uint8_t> hash(HashKind k, const uint8_t *p, size_t n) {
    uint32_t h[8];
    int words;
    if (k == kMd5) {
        static const uint32_t iv[4] = {0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476};
        memcpy(h, iv, sizeof iv);
        words = 4;
    } else if (k == kSha1) {
        memcpy(h, srtp::kSha1Init, 20);
        words = 5;
    } else {
        static const uint32_t iv[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                       0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
        memcpy(h, iv, sizeof iv);
        words = 8;
    }
    auto compress = [&](const uint8_t *b) {
        if (k == kMd5) md5_compress(h, b);
        else if (k == kSha1) srtp::sha1_compress(h, b);
        else sha256_compress(h, b);
    };
    size_t full = n / 64;
    for (size_t i = 0; i < full; i++) compress(p + 64 * i);
    uint8_t tail[128] = {0};
    size_t r = n - 64 * full;
    memcpy(tail, p + 64 * full, r);
    tail[r] = 0x80;
    size_t tl = r + 9 <= 64 ? 64 : 128;
    uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++)  // MD5: little-endian length; SHA: big-endian
        tail[k == kMd5 ? tl - 8 + i : tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    compress(tail);
    if (tl == 128) compress(tail + 64);
    std::vector<uint8_t> out(4 * words);
    for (int i = 0; i < words; i++)
        for (int j = 0; j < 4; j++)
            out[4 * i + j] = (uint8_t)(k == kMd5 ? h[i] >> (8 * j) : h[i] >> (24 - 8 * j));
    return out;
}

std::vector<uint8_t> hmac(HashKind k, const uint8_t *key, size_t klen, const std::vector<uint8_t> &msg) {
    uint8_t kb[64] = {0};
    if (klen > 64) {
        std::vector<uint8_t> kh = hash(k, key, klen);
        memcpy(kb, kh.data(), kh.size());
    } else if (klen) {
        memcpy(kb, key, klen);
    }
    std::vector<uint8_t> in(64 + msg.size());
    for (int i = 0; i < 64; i++) in[i] = kb[i] ^ 0x36;
    if (!msg.empty()) memcpy(in.data() + 64, msg.data(), msg.size());
    std::vector<uint8_t> ih = hash(k, in.data(), in.size());
    std::vector<uint8_t> out(64 + ih.size());
    for (int i = 0; i < 64; i++) out[i] = kb[i] ^ 0x5c;
    memcpy(out.data() + 64, ih.data(), ih.size());
    return hash(k, out.data(), out.size());
}

// P_hash(secret, seed) of RFC 2246 5 / RFC 5246 5, XORed into out[0..n).
void p_hash_xor(HashKind k, const uint8_t *secret, size_t slen, const std::vector<uint8_t> &seed,
                uint8_t *out, size_t n) {
    std::vector<uint8_t> a = hmac(k, secret, slen, seed);  // A(1)
    size_t done = 0;
    while (done < n) {
        std::vector<uint8_t> m(a);
        m.insert(m.end(), seed.begin(), seed.end());
        std::vector<uint8_t> blk = hmac(k, secret, slen, m);
        for (size_t i = 0; i < blk.size() && done < n; i++) out[done++] ^= blk[i];
        a = hmac(k, secret, slen, a);
    }
}

struct Profile {
    int32_t id, enc_type, key_len, salt_len, rtp_tag, rtcp_tag;
};
// DtlsPacketTransformer.java:574-612 (ids: RFC 5764 4.1.2 / SRTPProtectionProfile)
const Profile kProfiles[] = {
    {SRTP_PROFILE_AES128_CM_HMAC_SHA1_80, SRTP_AESCM_ENCRYPTION, 16, 14, 10, 10},
    {SRTP_PROFILE_AES128_CM_HMAC_SHA1_32, SRTP_AESCM_ENCRYPTION, 16, 14, 4, 10},
    {SRTP_PROFILE_NULL_HMAC_SHA1_80, SRTP_NULL_ENCRYPTION, 0, 0, 10, 10},
    {SRTP_PROFILE_NULL_HMAC_SHA1_32, SRTP_NULL_ENCRYPTION, 0, 0, 4, 10},
};

} // namespace

extern "C" {

int srtp_tls_export_keying_material(int32_t prf, const uint8_t *master_secret, int32_t secret_len,
                                    const uint8_t client_random[32], const uint8_t server_random[32],
                                    const char *label, uint8_t *out, int32_t out_len) {
    if (!master_secret || secret_len <= 0 || !client_random || !server_random || !label || !out ||
        out_len < 0)
        return SRTP_EINVAL;
    if (prf != SRTP_TLS_PRF_TLS10 && prf != SRTP_TLS_PRF_SHA256) return SRTP_EINVAL;
    // seed = label || client_random || server_random (RFC 5705 4, no context)
    std::vector<uint8_t> seed(label, label + strlen(label));
    seed.insert(seed.end(), client_random, client_random + 32);
    seed.insert(seed.end(), server_random, server_random + 32);
    memset(out, 0, (size_t)out_len);
    if (prf == SRTP_TLS_PRF_SHA256) {
        p_hash_xor(kSha256, master_secret, (size_t)secret_len, seed, out, (size_t)out_len);
    } else {  // RFC 2246 5: halves S1, S2 (sharing the middle byte when odd)
        size_t half = ((size_t)secret_len + 1) / 2;
        p_hash_xor(kMd5, master_secret, half, seed, out, (size_t)out_len);
        p_hash_xor(kSha1, master_secret + secret_len - half, half, seed, out, (size_t)out_len);
    }
    return SRTP_OK;
}

int srtp_dtls_profile_keys(int32_t profile, const uint8_t *km, int32_t km_len, srtp_dtls_keys *out) {
    if (!out) return SRTP_EINVAL;
    const Profile *p = nullptr;
    for (const Profile &q : kProfiles)
        if (q.id == profile) p = &q;
    if (!p) return SRTP_EPOLICY;  // IllegalArgumentException("srtpProtectionProfile")
    memset(out, 0, sizeof *out);
    out->key_len = p->key_len;
    out->salt_len = p->salt_len;
    out->keying_material_len = 2 * (p->key_len + p->salt_len);
    srtp_policy pol = {p->enc_type, p->key_len, SRTP_HMACSHA1_AUTHENTICATION, 20, p->rtp_tag, p->salt_len};
    out->srtp = pol;
    pol.auth_tag_len = p->rtcp_tag;
    out->srtcp = pol;
    if (!km) return SRTP_OK;  // lengths and policies only
    if (km_len < out->keying_material_len) return SRTP_EINVAL;
    const uint8_t *q = km;  // client key | server key | client salt | server salt
    memcpy(out->client_key, q, p->key_len); q += p->key_len;
    memcpy(out->server_key, q, p->key_len); q += p->key_len;
    memcpy(out->client_salt, q, p->salt_len); q += p->salt_len;
    memcpy(out->server_salt, q, p->salt_len);
    return SRTP_OK;
}

int srtp_dtls_transformer_create(srtp_engine *e, int32_t profile, int32_t is_client, int32_t kind,
                                 const uint8_t *km, int32_t km_len, int32_t *out_transformer,
                                 int32_t out_factories[2]) {
    if (!e || !km || !out_transformer) return SRTP_EINVAL;
    if (kind != SRTP_KIND_RTP && kind != SRTP_KIND_RTCP) return SRTP_EINVAL;
    srtp_dtls_keys k;
    int rc = srtp_dtls_profile_keys(profile, km, km_len, &k);
    if (rc != SRTP_OK) return rc;
    // NULL-cipher profiles export no master key (0-byte key and salt, :594-609);
    // the reference then fails in key derivation (SRTPCryptoContext.deriveSrtpKeys
    // :398 on a null cipher).  Refused here, at creation.
    if (k.key_len == 0) return SRTP_EPOLICY;
    int32_t fc = -1, fs = -1, t = -1;
    rc = srtp_factory_create(e, is_client ? 1 : 0, k.client_key, k.key_len, k.client_salt,
                             k.salt_len, &k.srtp, &k.srtcp, &fc);
    if (rc == SRTP_OK)
        rc = srtp_factory_create(e, is_client ? 0 : 1, k.server_key, k.key_len, k.server_salt,
                                 k.salt_len, &k.srtp, &k.srtcp, &fs);
    if (rc == SRTP_OK)
        rc = is_client ? srtp_transformer_create(e, kind, fc, fs, &t)
                       : srtp_transformer_create(e, kind, fs, fc, &t);
    memset(&k, 0, sizeof k);
    if (rc != SRTP_OK) {
        if (fs >= 0) srtp_factory_close(e, fs);
        if (fc >= 0) srtp_factory_close(e, fc);
        return rc;
    }
    *out_transformer = t;
    if (out_factories) {
        out_factories[0] = fc;
        out_factories[1] = fs;
    }
    return SRTP_OK;
}

} // extern "C"
