/* skein.h -- Skein-512 hash and MAC for the oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The reference's SKEIN_AUTHENTICATION runs bccontrib's SkeinMac
 * (BaseSRTPCryptoContext.java:244-248, keyed in SRTPCryptoContext.java:421-428
 * and SRTCPCryptoContext.java:185-192 with ParametersForSkein(authKey,
 * Skein512, tagLength * 8)).  bccontrib is not in /root/reference, so this is a
 * restatement of the published algorithm: "The Skein Hash Function Family",
 * version 1.3 (Threefish-512, UBI chaining, Skein-MAC = key UBI, config UBI,
 * message UBI, output UBI).  Pinned by the paper's Skein-512-512 known
 * answers and by its precomputed Skein-512-512 IV (tests/test_skein.py). */
#ifndef ORC_SKEIN_H
#define ORC_SKEIN_H
#include <stddef.h>
#include <stdint.h>

/* one Threefish-512 block: key k[8], tweak t[2], little-endian words */
void sk_threefish512(const uint64_t k[8], const uint64_t t[2], const uint64_t in[8], uint64_t out[8]);

/* Streaming Skein-512 with an optional key (Skein-MAC when key_len > 0). */
typedef struct {
    uint64_t g0[8];      /* chaining value after the key and config UBIs */
    uint64_t h[8];       /* running chaining value */
    uint8_t buf[64];     /* pending message bytes (the last block is held back) */
    int nbuf;
    uint64_t pos;        /* message bytes processed (tweak position) */
    int first;
    int out_bits;
} sk_ctx;

/* Skein-512 with output length out_bits (1..512) keyed with key[0..key_len). */
void sk_init(sk_ctx *c, const uint8_t *key, int key_len, int out_bits);
/* restart the message from the precomputed g0 (doFinal resets the MAC) */
void sk_reset(sk_ctx *c);
void sk_update(sk_ctx *c, const uint8_t *msg, size_t n);
/* writes ceil(out_bits / 8) bytes, then resets */
void sk_final(sk_ctx *c, uint8_t *out);

#endif
