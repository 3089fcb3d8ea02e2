/* twofish.h -- Twofish for the oracle (TEST INFRASTRUCTURE ONLY). */
#ifndef ORC_TWOFISH_H
#define ORC_TWOFISH_H
#include <stdint.h>

typedef struct {
    uint32_t K[40];      /* expanded subkeys: whitening K0..K7, round keys K8..K39 */
    uint32_t T[4][256];  /* g(X) = T0[x0] ^ T1[x1] ^ T2[x2] ^ T3[x3] (S-boxes and MDS) */
} tf_key;

/* key_len 16, 24 or 32; returns 0, or -1 for another length */
int tf_set_key(tf_key *t, const uint8_t *key, int key_len);
void tf_encrypt(const tf_key *t, const uint8_t in[16], uint8_t out[16]);

#endif
