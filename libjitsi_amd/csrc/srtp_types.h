// srtp_types.h -- device-resident tables shared by the host engine and the
// gfx950 kernels.  Layouts are sized for HBM: one 256-B session-key record per
// (factory, RTP|RTCP), one 32-B state record per (transformer, SSRC) context.
#pragma once
#include <stdint.h>

namespace srtp {

constexpr int kAesRounds = 10;
constexpr uint64_t kEmptyKey = ~0ull;       // hash slot never used
constexpr uint64_t kTombKey = ~0ull - 1ull; // context removed (transformer close / abort)
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

// Session keys of one SRTPCryptoContext / SRTCPCryptoContext family.  Every
// context derived from one factory shares them (kdr == 0):
// SRTPCryptoContext.deriveSrtpKeys :393-447, SRTCPCryptoContext.deriveSrtcpKeys
// :158-211.  The HMAC key is stored as its two SHA-1 midstates (ipad/opad),
// so the per-packet MAC costs no key blocks.
struct alignas(256) KeySet {
    uint32_t rk[4 * (kAesRounds + 1)]; // AES-128 round keys (AES-128-CM), little-endian column words
    uint32_t ipad[5];                  // SHA-1 state after (authKey ^ 0x36..) block
    uint32_t opad[5];                  // SHA-1 state after (authKey ^ 0x5c..) block
    uint32_t salt[4];                  // session salt bytes 0..13 as LE words (14,15 = 0)
    int32_t enc_type;                  // SRTP_NULL_ENCRYPTION / SRTP_AESCM_ENCRYPTION
    int32_t auth_type;                 // SRTP_NULL_AUTHENTICATION / _HMACSHA1_ / _SKEIN_ (SkeinKeys)
    int32_t tag_len;                   // policy.getAuthTagLength()
    int32_t kind;                      // SRTP_KIND_RTP / SRTP_KIND_RTCP
    int32_t ext;                       // 1: packets run by k_ext (AES-F8, AES-256-CM, Twofish, Skein MAC)
    uint32_t pad;
};
static_assert(sizeof(KeySet) == 256, "KeySet is one 256-B record");

// Round keys of the key sets whose cipher k_ext runs, beside KeySet, indexed by
// key-set id: AES-F8's IV' key (SRTPCipherF8.deriveForIV :66-95: the session
// key ^ (session salt || 0x55 0x55); 10 rounds), or the AES-256-CM session
// key (14 rounds; RFC 6188).
struct alignas(64) ExtKeys {
    uint32_t rk[60]; // 4 * (nr + 1) round-key words, little-endian column words
    int32_t nr;      // 10 or 14
    uint32_t pad[3];
};
static_assert(sizeof(ExtKeys) == 256, "ExtKeys is 256 B");

// Twofish key material of a key set (ZRTP "2FS": TWOFISH_ENCRYPTION /
// TWOFISHF8_ENCRYPTION): subkeys and the four g() tables of the key schedule
// (key-dependent S-boxes times the MDS columns).  Two per key set -- [0] the
// session key, [1] the F8 IV' key -- in a table allocated with the first
// Twofish factory.
struct alignas(256) TwofishKeys {
    uint32_t K[40];
    uint32_t pad[24];
    uint32_t T[4][256];
};
static_assert(sizeof(TwofishKeys) == 4352, "TwofishKeys is 4352 B");

// Skein-512 MAC key of a key set (SKEIN_AUTHENTICATION, ZRTP "SK32"/"SK64":
// bccontrib's SkeinMac keyed with the 32-byte session auth key and an output
// of tag_len * 8 bits, SRTPCryptoContext.java:421-428): the chaining value
// after the key and config UBIs, so a packet's MAC starts at its message
// blocks.  Indexed by key-set id, allocated with the first Skein factory.
struct alignas(64) SkeinKeys {
    uint64_t g0[8];
};
static_assert(sizeof(SkeinKeys) == 64, "SkeinKeys is 64 B");

struct FactoryRec {      // SRTPContextFactory
    int32_t open;        // 0 after close(): getDefaultContext() == null
    int32_t ks_rtp;      // key set of its default SRTPCryptoContext
    int32_t ks_rtcp;     // key set of its default SRTCPCryptoContext
    int32_t sender;
};

struct TransformerRec {  // SRTPTransformer / SRTCPTransformer
    int32_t kind;
    int32_t fwd;         // forwardFactory id (-1 none)
    int32_t rev;         // reverseFactory id
    int32_t alive;
};

// Per-(transformer, SSRC) context state, the mutable part of
// SRTPCryptoContext (:130-164) / SRTCPCryptoContext (:54-59).
struct alignas(32) CtxState {
    uint32_t ks;     // key set (fixed at derivation; survives factory swaps, Q16)
    int32_t a;       // SRTP roc            | SRTCP sentIndex
    int32_t b;       // SRTP s_l            | SRTCP receivedIndex
    int32_t g;       // SRTP guessedROC (last value, kept for state parity)
    uint64_t window; // replayWindow (Java long)
    uint32_t flags;  // bit0: seqNumSet
    uint32_t birth;  // bundle serial in which the context was derived
};
static_assert(sizeof(CtxState) == 32, "CtxState is 32 B");

// One packet as seen by the per-context walk (sorted by context slot).
struct alignas(16) WalkRec {
    uint32_t p;      // packet index | kRecSkipDec
    uint32_t word;   // RTP: sequence number; RTCP unprotect: E|index word
    uint32_t lc;     // len (low 16) | min(cap, 65535) (high 16)
    int32_t h;       // RTP: header length or kHdrThrow; RTCP unprotect: tag length used for `word`
};
constexpr uint32_t kRecSkipDec = 0x80000000u; // FLAG_DISCARD|FLAG_SILENCE: no decrypt

// k_unprotect's per-packet summary (BundleArgs::spec), read by the walk's
// tag re-check and by k_unprotect_fix to decide a repair without the key set
constexpr uint32_t kSpecDid = 1u;  // decrypted in place under the ROC guess
constexpr uint32_t kSpecAes = 2u;  // AES-128-CM key set of the fused path (not k_ext's)
constexpr uint32_t kSpecRtp = 4u;  // SRTP (else SRTCP)
constexpr uint32_t kSpecSkip = 8u; // SRTP packet flagged DISCARD / SILENCE: not deciphered
constexpr uint32_t kRecIdxMask = 0x0FFFFFFFu;
constexpr int32_t kHdrThrow = (int32_t)0x80000000; // getHeaderLength would throw

constexpr uint32_t kLongRank = 1024; // k_unprotect: chain packets from this rank on get a rank-based ROC guess

// bundle control block (zeroed per bundle)
struct BundleCtl {
    uint32_t any_throw;   // some packet could make the reference throw -> two-pass walk
    uint32_t n_long;      // nonzero: the bundle has a context chain of >= kLongMin records
    uint32_t tile_ticket; // next walk tile of the chain pass
    uint32_t tiles_done;  // chain-pass tiles finished (the last one runs the stall fix-up)
    uint32_t n_stall;     // chain-pass tiles whose look-back gave up (their parts left to the fix-up)
    uint32_t len_classes; // bit c: some packet has c 64-B chunks (c = 31: 31 or more); the sort's first pass
    uint32_t small_ready; // k_small: 2 once the walk is done (workgroup 0 -> the others)
    uint32_t pad;
    uint32_t cls_cursor[32]; // the sort's first pass: reservations per length class
};

// BundleArgs::dbg bits (srtp_engine_set_debug): test hooks, 0 in production
constexpr uint32_t kDbgForceStall = 1u; // chain-pass tiles 1, 4, 7, ... give up their look-back at once

// Cumulative per-engine event counters (srtp_engine_stats), 64-bit, kept in
// kCountReplicas copies so that one bundle's wave-aggregated atomics spread
// over many addresses; the host sums the copies.
constexpr int kCountReplicas = 64;
constexpr int kCtrStatus = 0;        // [0, 16): final status counts (SRTP_STATUS_*)
constexpr int kStatusHole = 11;      // ... and at SRTP_NUM_STATUS: bundle-former holes (srtp_stats.holes)
constexpr int kCtrRocRecheck = 16;   // unprotect tags re-checked under a walk ROC != the speculation
constexpr int kCtrRepaired = 17;     // packets k_unprotect_fix re-ciphered
constexpr int kCtrOverflow = 18;     // packets refused a new context (table full)
constexpr int kCtrChainStall = 19;   // walk tiles that gave up waiting on a long chain's look-back
                                     // (their chain is then walked by the fix-up; never expected)
constexpr int kCtrLongWalked = 20;   // records walk_long walked one at a time (they broke the speculation)
constexpr int kCtrStride = 32;       // u64 words per replica (one 256-B line)

// internal walk statuses (beyond SRTP_STATUS_*)
constexpr int32_t kStPending = 100;

} // namespace srtp
