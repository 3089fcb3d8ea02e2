// host_crypto.h -- control-plane crypto on the host: AES-128 key schedule and
// single-block encrypt (for the RFC 3711 4.3 key derivation PRF) and the SHA-1
// compression function (for the HMAC ipad/opad midstates).  Runs once per
// factory; the per-packet path is on the GPU.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace srtp {

// Expanded AES-128 encryption key, 44 words.  Word i holds round-key bytes
// 4i..4i+3 in little-endian order (byte 4i in bits 0..7), the layout the
// gfx950 T-table rounds use.
void aes128_expand_le(const uint8_t key[16], uint32_t rk_le[44]);
// AES-128 (key_len 16) or AES-256 (32) key expansion in the same layout;
// returns the number of rounds (10 / 14), 4 * (nr + 1) words written.
int aes_expand_le(const uint8_t *key, int key_len, uint32_t rk_le[60]);
void aes_encrypt_block_nr(const uint32_t *rk_le, int nr, const uint8_t in[16], uint8_t out[16]);
void aes128_encrypt_block(const uint32_t rk_le[44], const uint8_t in[16], uint8_t out[16]);
// SHA-1 compression of one 64-byte block into state[5].
void sha1_compress(uint32_t state[5], const uint8_t block[64]);
extern const uint32_t kSha1Init[5];
// The AES forward T-table used by the device (LE layout: 2s | s<<8 | s<<16 | 3s<<24).
void aes_te0_le(uint32_t te0[256]);

// RFC 3711 4.3 key derivation exactly as SRTPCryptoContext.deriveSrtpKeys
// (labels 0,1,2; :393-447) or SRTCPCryptoContext.deriveSrtcpKeys (3,4,5;
// :158-211) with kdr == 0.
void derive_session_keys(const uint8_t master_key[16], const uint8_t master_salt[14], bool rtcp,
                         uint8_t enc[16], uint8_t auth[20], uint8_t salt[14]);
// The same with a 16- or 32-byte master key: the PRF is AES-128 / AES-256 and
// the session encryption key is key_len bytes (RFC 6188 4.1 for AES-256).
void derive_session_keys_n(const uint8_t *mk, int key_len, const uint8_t ms[14], bool rtcp,
                           uint8_t *enc, uint8_t auth[20], uint8_t salt[14]);
// With the Twofish PRF (twofish = true: the ZRTP Twofish policies key their
// TwofishEngine with the master key).
// auth_len: the policy's auth key length (20 for HMAC-SHA1, 32 for ZRTP's Skein).
void derive_session_keys_cipher(bool twofish, const uint8_t *mk, int key_len, const uint8_t ms[14],
                                bool rtcp, uint8_t *enc, uint8_t *auth, uint8_t salt[14],
                                int auth_len = 20);
// Twofish key schedule (key_len 16, 24 or 32): subkeys K[40] and the four g()
// tables (key-dependent S-boxes times the MDS columns); one block.
void twofish_schedule(const uint8_t *key, int key_len, uint32_t K[40], uint32_t T[4][256]);
void twofish_encrypt_block(const uint32_t K[40], const uint32_t T[4][256], const uint8_t in[16],
                           uint8_t out[16]);
// HMAC-SHA1 ipad/opad midstates for a 20-byte key.
void hmac_sha1_midstates(const uint8_t key[20], uint32_t ipad[5], uint32_t opad[5]);

// Skein-512 (version 1.3): UBI block types, and the key-schedule parity
// constant C240 of Threefish.
constexpr uint64_t kSkeinParity = 0x1BD11BDAA9FC1A22ull;
constexpr uint64_t kSkeinTypeKey = 0, kSkeinTypeCfg = 4, kSkeinTypeMsg = 48, kSkeinTypeOut = 63;
// The chaining value of a keyed Skein-512 with out_bits output bits after the
// key UBI (skipped for key_len 0) and the config UBI: SkeinMac's state before
// the first message byte.
void skein512_key_state(const uint8_t *key, int key_len, int out_bits, uint64_t g0[8]);
// Whole Skein-512 MAC (key_len 0: the plain hash), ceil(out_bits / 8) bytes.
void skein512_mac(const uint8_t *key, int key_len, int out_bits, const uint8_t *msg, size_t n,
                  uint8_t *out);

} // namespace srtp
