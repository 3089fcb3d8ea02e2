/*
 * srtp_oracle.h -- CPU restatement of libjitsi's SRTP/SRTCP hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X engine
 * (libjitsi_amd).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product never links or calls it.
 *
 * It restates, with Java integer semantics (two's-complement i32/i64, JLS
 * 15.19 shift-distance masking, signed bytes), the reference files:
 *   srtp/SRTPCryptoContext.java:237-744   (auth, replay, IV, guessIndex, update)
 *   srtp/SRTCPCryptoContext.java:106-451  (SRTCP replay, IV, protect/unprotect)
 *   srtp/BaseSRTPCryptoContext.java:178-278 (key storage, authenticatePacketHMAC)
 *   srtp/SRTPCipherCTR.java:68-121        (AES-CM keystream + XOR)
 *   srtp/SRTPCipherF8.java:66-183         (AES-F8 IV' key, keystream chain)
 *   srtp/BaseSRTPCryptoContext.java:244-248, SRTPCryptoContext.java:421-428
 *                                         (SKEIN_AUTHENTICATION: Skein-512 MAC, skein.c)
 *   srtp/SRTPTransformer.java:100-219, srtp/SRTCPTransformer.java:92-207,
 *   srtp/SRTPContextFactory.java:50-68    (per-transformer SSRC context map)
 *   nm/RawPacket.java:203-220,463-614,723-839,885-909,988-999,1284-1292
 *   tf/SinglePacketTransformer.java:121-216 (array loop, rethrow aborts batch)
 * where srtp/ = src/org/jitsi/impl/neomedia/transform/srtp/ and
 * nm/ = src/org/jitsi/impl/neomedia/, tf/ = .../neomedia/transform/.
 *
 * Primitives (AES-128 block, HMAC-SHA1) come from OpenSSL 3 libcrypto, the
 * same library family the reference's JNI backend binds
 * (src/native/openssl/BlockCipher.c, HMAC.c).  Parity pinning: FIPS-197,
 * RFC 2202, RFC 3711 App. B.2/B.3 known-answer tests (the reference ships no
 * SRTP test vectors); see tests/test_oracle_kat.py.
 *
 * Packet model: packet i lives in seg[off[i] .. off[i]+cap[i]); this region is
 * the Java RawPacket buffer with offset 0 and buffer.length == cap[i].  len[i]
 * is RawPacket.length (updated in place).  A reallocating RawPacket.append /
 * grow is modelled as "fits in cap"; a packet whose cap is too small is
 * rejected up front with ORC_ERR_CAPACITY and leaves no trace.
 */
#ifndef SRTP_ORACLE_H
#define SRTP_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SRTPPolicy constants, srtp/SRTPPolicy.java:29-63 */
enum { ORC_NULL_ENCRYPTION = 0, ORC_AESCM_ENCRYPTION = 1, ORC_AESF8_ENCRYPTION = 2,
       ORC_TWOFISH_ENCRYPTION = 3, ORC_TWOFISHF8_ENCRYPTION = 4 };
enum { ORC_NULL_AUTHENTICATION = 0, ORC_HMACSHA1_AUTHENTICATION = 1,
       ORC_SKEIN_AUTHENTICATION = 2 };

/* Per-packet status (same numbering as include/srtp_mi355x.h). */
enum {
    ORC_OK = 0,
    ORC_DROP_REPLAY = 1,     /* checkReplay false -> null */
    ORC_DROP_AUTH = 2,       /* authenticatePacket false -> null */
    ORC_DROP_VERSION = 3,    /* SRTPTransformer.reverseTransform version check */
    ORC_DROP_NO_CONTEXT = 4, /* factory closed -> getContext null */
    ORC_ERR_CAPACITY = 5,    /* cap too small for the in-place append */
    ORC_ERR_MALFORMED = 6,   /* reference throws (AIOOBE / IOOBE) */
    ORC_DROP_INVALID = 7,    /* RawPacket.isInvalid (length < 12) */
    ORC_NOT_PROCESSED = 8,   /* after a throw: rest of the array aborted */
    ORC_SKIPPED = 9          /* null element / predicate mismatch */
};

/* Packet flags (javax.media.Buffer values used by SRTPCryptoContext:609-611) */
enum { ORC_FLAG_DISCARD = 0x2, ORC_FLAG_SILENCE = 0x4, ORC_FLAG_SKIP = (int)0x80000000u };

enum { ORC_KIND_RTP = 0, ORC_KIND_RTCP = 1 };
/* MODE_REF: the reference call structure (one 16-B AES-ECB call per keystream
 * block + tail block, HMAC re-keyed per packet).  MODE_TUNED: one
 * EVP_aes_128_ctr call per packet, pre-keyed HMAC context copied per packet. */
enum { ORC_MODE_REF = 0, ORC_MODE_TUNED = 1 };

typedef struct {
    int32_t enc_type, enc_key_len, auth_type, auth_key_len, auth_tag_len, salt_key_len;
} orc_policy;

typedef struct orc_factory orc_factory;
typedef struct orc_transformer orc_transformer;

/* SRTPContextFactory(sender, masterKey, masterSalt, srtpPolicy, srtcpPolicy).
 * Returns NULL if the policy is outside the restated profiles. */
orc_factory *orc_factory_new(int sender, const uint8_t *master_key, int key_len,
                             const uint8_t *master_salt, int salt_len,
                             const orc_policy *srtp, const orc_policy *srtcp, int mode);
void orc_factory_close(orc_factory *f);

/* new SRTPTransformer(fwd, rev) / new SRTCPTransformer(fwd, rev) */
orc_transformer *orc_transformer_new(int kind, orc_factory *fwd, orc_factory *rev);
/* setContextFactory / updateFactory: closes the replaced factory, keeps contexts */
void orc_transformer_set_factory(orc_transformer *t, orc_factory *f, int forward);
/* close(): closes both factories, drops all contexts */
void orc_transformer_close(orc_transformer *t);
void orc_transformer_free(orc_transformer *t);
/* SRTPCryptoContext.checkReplay property (SRTP only; SRTCP always checks). */
void orc_set_check_replay(int enabled);

/* transform(RawPacket[]) (reverse=0) / reverseTransform(RawPacket[]) (reverse=1).
 * ts[i] is packet i's transformer (a bundle may span transformers; abort on a
 * throw is scoped to that transformer's packets, like one transform() call per
 * transformer).  If ts_stride == 0 every packet uses ts[0]. */
int orc_process(orc_transformer *const *ts, int ts_stride, int reverse,
                uint8_t *seg, const uint32_t *off, uint32_t *len, const uint32_t *cap,
                const uint32_t *flags, int32_t *status, uint32_t n, int abort_on_error);

/* Context state snapshot for parity tests. Returns 0 if the SSRC has no context. */
typedef struct {
    int32_t roc, s_l, seq_num_set, guessed_roc;   /* SRTP */
    int32_t sent_index, received_index;           /* SRTCP */
    uint64_t replay_window;
} orc_ctx_state;
int orc_get_state(orc_transformer *t, uint32_t ssrc, orc_ctx_state *out);
uint32_t orc_num_contexts(orc_transformer *t);
/* Context-state export / import, as the engine's srtp_export_contexts /
 * srtp_set_context_state (no reference API; the state is SRTPCryptoContext's
 * private fields :96-135). */
uint32_t orc_export_contexts(orc_transformer *t, uint32_t *ssrcs, orc_ctx_state *states, uint32_t max);
int orc_set_context_state(orc_transformer *t, uint32_t ssrc, int forward, const orc_ctx_state *st);
/* Remove the context for ssrc (1 if there was one). */
int orc_remove_context(orc_transformer *t, uint32_t ssrc);

/* Primitive helpers exposed for the KAT tests. */
/* RFC 5705 exporter over the TLS PRF (OpenSSL TLS1-PRF KDF); prf 0 = TLS 1.0
 * MD5-SHA1, 1 = TLS 1.2 SHA256 (DtlsPacketTransformer.java:614-617). */
int orc_tls_export(int prf, const uint8_t *secret, int secret_len, const uint8_t cr[32],
                   const uint8_t sr[32], const char *label, uint8_t *out, int out_len);
void orc_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]);
void orc_hmac_sha1(const uint8_t *key, int key_len, const uint8_t *msg, size_t n, uint8_t out[20]);
/* RFC 3711 4.3 PRF exactly as SRTPCryptoContext.deriveSrtpKeys (labels 0/1/2)
 * or SRTCPCryptoContext.deriveSrtcpKeys (labels 3/4/5). */
/* AES-F8 (SRTPCipherF8.deriveForIV + process) over data[0..len) with IV iv. */
void orc_aes_f8(const uint8_t key[16], const uint8_t *salt, int salt_len, const uint8_t iv[16],
                uint8_t *data, int len);
void orc_derive_keys(const uint8_t mk[16], const uint8_t ms[14], int rtcp,
                     uint8_t enc[16], uint8_t auth[20], uint8_t salt[14]);
void orc_derive_keys_n(const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                       uint8_t *enc, uint8_t auth[20], uint8_t salt[14]);
/* Twofish policies: the PRF is Twofish keyed with the master key. */
void orc_derive_keys_twofish(const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                             uint8_t *enc, uint8_t auth[20], uint8_t salt[14]);
/* key derivation with the policy's auth key length (Skein: 32), PRF AES or Twofish */
void orc_derive_keys_auth(int twofish, const uint8_t *mk, int key_len, const uint8_t ms[14], int rtcp,
                          uint8_t *enc, uint8_t *auth, int auth_len, uint8_t salt[14]);
/* Skein-512 (skein.c, version 1.3) keyed with key[0..key_len) (key_len 0: plain
 * hash), out_bits output bits: the tag SkeinMac computes */
void orc_skein512_mac(const uint8_t *key, int key_len, int out_bits, const uint8_t *msg, size_t n,
                      uint8_t *out);
void orc_skein512_state0(const uint8_t *key, int key_len, int out_bits, uint64_t g0[8]);
/* one Twofish block (twofish.c), key_len 16 / 24 / 32 */
void orc_twofish_encrypt_block(const uint8_t *key, int key_len, const uint8_t in[16],
                               uint8_t out[16]);

/* CPU baseline timing (oracle_bench.c): packets protected AND unprotected by
 * `threads` pinned threads in about `seconds` (-1 on a rejected packet). */
int64_t orc_bench_round_trips(int mode, int threads, double seconds, int pkt_len, int ssrcs,
                              uint32_t seed, double *elapsed);

#ifdef __cplusplus
}
#endif
#endif
