// srtp_kernels.hip -- gfx950 kernels of the SRTP/SRTCP engine.
//
// Bundle pipeline (one HIP stream, see engine.cpp):
//   k_parse    one lane per packet: RawPacket accessors, version check,
//              (transformer, SSRC) -> context slot in an HBM hash table
//              (SRTPTransformer.getContext :152-175, lazily derived contexts),
//              emits a 16-B walk record keyed by slot.
//   radix sort (own LSD, 8-bit digits) by slot, stable -> each context's
//              packets in array order.
//   k_unprotect [unprotect] one lane per packet: HMAC-SHA1 tag check and
//              speculative in-place AES-CM decryption under the ROC guessed from
//              the context state at bundle start; keeps the inner SHA-1 midstate
//              and ciphertext of the ROC-carrying block for re-checks.
//   k_walk     one lane per context segment: the serial integer state machine of
//              SRTPCryptoContext (guessIndex :457-475, checkReplay :279-323,
//              update :719-744) / SRTCPCryptoContext (:106-120, :435-451), in
//              array order, committing the context state in HBM (in-order
//              packets on a fast prefix).  The second launch walks chains of
//              >= 256 packets with every tile they cross at once (chain_part),
//              or is the "limit" pass reproducing SinglePacketTransformer's
//              abort-on-throw.
//   k_skein    [engines with Skein-MAC key sets] Skein-512 tag check / trailer.
//   k_ext      [engines with F8 / AES-256 / Twofish / Skein key sets] their
//              ciphers (and the F8 / AES-256 HMAC trailers).
//   k_protect  [protect] one lane per packet: fused AES-CM keystream + XOR +
//              HMAC-SHA1 (one read and one write of the packet bytes).
//   k_unprotect_fix [unprotect] statuses/lengths out; undoes/redoes the rare
//              packets whose speculation the walk overturned.
//
// AES uses four little-endian T-tables replicated 32x in LDS (128 KB) so that
// lane l only ever touches LDS bank (l & 31): conflict-free ds_read_b32 with a
// single v_perm_b32 per lookup address and v_bitop3 XORs.  Round keys, salt
// and HMAC midstates are wave-uniform SGPRs; SHA-1 runs per lane with
// v_alignbit rotates.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>


#include "../../include/srtp_mi355x.h"
#include "srtp_kernels.h"

namespace srtp {

__device__ uint32_t d_te0[256];

constexpr int kBlock = 256;

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
    return __builtin_amdgcn_alignbit(x, x, 32u - n);
}
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }
__device__ __forceinline__ uint32_t ld_be32(const uint8_t *p) {
    return (ld_u8(p) << 24) | (ld_u8(p + 1) << 16) | (ld_u8(p + 2) << 8) | ld_u8(p + 3);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

__device__ __forceinline__ int32_t java_ishl1(int32_t n) { return (int32_t)(1u << (n & 31)); }
__device__ __forceinline__ int64_t java_lshl(int64_t v, int64_t n) {
    return (int64_t)((uint64_t)v << (n & 63));
}

// ----------------------------------------------------------------- AES-128
// LDS image of the four AES T-tables T_r = rotl(T0, 8r), 32 lane copies each,
// 128 KB.  Byte address of entry x of table t for a lane with copy c = lane & 31:
//     (t >> 1) << 16 | x << 8 | (t & 1) << 7 | c << 2
// so a ds_read_b32 wave instruction hits bank c for every lane (conflict-free:
// lanes l and l+32 sit in different halves of the wave's LDS access), and the
// address is one v_perm_b32 of the state word and a per-lane base
// (byte 1 <- state byte k, bytes 0 and 2 <- base).
constexpr int kTeWords = 32768;  // 128 KB
constexpr int kTeCounters = 16;  // per-workgroup status counts, after the image (which stays at LDS 0)
constexpr int kAesBlock = 1024;  // threads per workgroup of the AES kernels (1 WG per CU)
constexpr int kMacBlock = 256;   // at most, the MacOnly instances' (small bundles)
// (tools/build_variant.sh builds the occupancy variants of
// profiles/r05/kernel_experiments.md with smaller workgroups: more VGPRs per
// lane, fewer waves per SIMD)
#ifndef SRTP_UNPROTECT_BLOCK
#define SRTP_UNPROTECT_BLOCK 1024
#endif
#ifndef SRTP_PROTECT_BLOCK
#define SRTP_PROTECT_BLOCK 1024
#endif
constexpr int kUnprotectBlock = SRTP_UNPROTECT_BLOCK; // k_unprotect's workgroup size
constexpr int kProtectBlock = SRTP_PROTECT_BLOCK;     // k_protect's

__device__ __forceinline__ void fill_te4(uint32_t *s_te) {
    // Entry e of te0 fills words (h << 14) | (e << 6) | l (h = 0, 1; l =
    // 0..63) of table t = 2h + (l >> 5), rotated left by 8t.  Wave w of W
    // takes entries w, w + W, ...: one te0 load per lane for up to 64 of
    // them, then per entry a broadcast (readlane) and two stores per lane to
    // consecutive words (no bank conflicts) -- one memory round trip per
    // workgroup instead of one per 8 words per thread.  blockDim.x is a
    // multiple of 64.
    const int W = (int)(blockDim.x >> 6), w = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63u);
    const uint32_t r = (uint32_t)(lane >> 5) << 3;
    for (int j0 = 0; w + j0 * W < 256; j0 += 64) {
        const int ej = w + (j0 + lane) * W;
        const uint32_t mine = ej < 256 ? d_te0[ej] : 0u;
        for (int k = 0; k < 64; k++) {
            const int e = w + (j0 + k) * W;
            if (e >= 256) break;
            const uint32_t v = __builtin_amdgcn_readlane(mine, k);
            s_te[(e << 6) | lane] = rotl(v, r);
            s_te[(1 << 14) | (e << 6) | lane] = rotl(v, r + 16u);
        }
    }
    __syncthreads();
    // The table is read only by inline asm (aes_rounds_asm.inc): let the
    // pointer escape so the LDS image and the stores above are kept.
    asm volatile("" ::"s"(s_te) : "memory");
}

struct TeBase {
    uint32_t b[4]; // per-lane byte base of table t (bytes 0 and 2 of the address)
};

__device__ __forceinline__ TeBase te_base() {
    TeBase tb;
    const uint32_t c4 = (threadIdx.x & 31u) << 2;
#pragma unroll
    for (int t = 0; t < 4; t++) tb.b[t] = (uint32_t)((t >> 1) << 16) | (uint32_t)((t & 1) << 7) | c4;
    return tb;
}

// entry (byte k of s) of table t
#define TL(s, k, t)                                                                     \
    (*reinterpret_cast<const uint32_t *>(                                               \
        lds + __builtin_amdgcn_perm((s), tb.b[t], 0x0c020000u | ((4u + (k)) << 8))))

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct RoundKeys {
    uint32_t k[44];
};

__device__ __forceinline__ void aes_encrypt2(const char *__restrict__ lds, const TeBase &tb,
                                             const RoundKeys &rk, uint32_t a[4], uint32_t b[4]);

// AES-CM state of one packet (SRTPCipherCTR.getCipherStream :68-92): keystream
// block j = AES(iv[0..13] || u16_be(j)), XORed over packet bytes [off, end).
struct Ctr {
    uint32_t iv[4];
    int off, end;
    uint32_t carry[4]; // keystream block preceding the current 64-B chunk
};

__device__ __forceinline__ void ctr_input(const uint32_t iv[4], int j, uint32_t out[4]) {
    out[0] = iv[0]; out[1] = iv[1]; out[2] = iv[2];
    out[3] = iv[3] | ((((uint32_t)j >> 8) & 0xffu) << 16) | (((uint32_t)j & 0xffu) << 24);
}

// XOR the keystream into the 16 LE words d[] of packet chunk c (bytes 64c ..
// 64c+63).  Payload word i uses keystream word i; the payload starts `off`
// bytes into the packet (a multiple of 4), so chunk word 4m+k takes keystream
// word 16c + 4m + k - off/4, i.e. blocks 4c - off/16 - 1 .. 4c - off/16 + 3.
// Computes four new blocks (two interleaved pairs, one AES code site).
__device__ __forceinline__ void ctr_chunk(const char *__restrict__ lds, const TeBase &tb,
                                          const RoundKeys &rk, Ctr &cs, int c, uint32_t d[16]) {
    const int hq = cs.off >> 4, s = (cs.off >> 2) & 3;
    const int j0 = 4 * c - hq;
    uint32_t K[16];
#pragma unroll 1
    for (int pr = 0; pr < 2; pr++) {
        uint32_t x[4], y[4];
        ctr_input(cs.iv, j0 + 2 * pr, x);
        ctr_input(cs.iv, j0 + 2 * pr + 1, y);
        aes_encrypt2(lds, tb, rk, x, y);
#pragma unroll
        for (int k = 0; k < 8; k++) K[k] = K[k + 8];
#pragma unroll
        for (int k = 0; k < 4; k++) { K[8 + k] = x[k]; K[12 + k] = y[k]; }
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
        // keystream word for chunk word i: concat(carry, K)[4 + i - s]
        const uint32_t a0 = K[i];
        const uint32_t a1 = i >= 1 ? K[i - 1] : cs.carry[3 + i];
        const uint32_t a2 = i >= 2 ? K[i - 2] : cs.carry[2 + i];
        const uint32_t a3 = i >= 3 ? K[i - 3] : cs.carry[1 + i];
        const uint32_t ksw = (s & 2) ? ((s & 1) ? a3 : a2) : ((s & 1) ? a1 : a0);
        const int pos = 64 * c + 4 * i;
        uint32_t m = 0u;
        if (pos >= cs.off && pos < cs.end) {
            const int rem = cs.end - pos;
            m = rem >= 4 ? 0xffffffffu : ((1u << (8 * rem)) - 1u);
        }
        d[i] ^= ksw & m;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) cs.carry[k] = K[12 + k];
}

// ----------------------------------------------------------------- SHA-1
// (xor3 is defined with the AES helpers below)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c);

// One block.  Each step in single gfx950 instructions: the schedule word
// xor3 + xor + rotate, f one v_bitop3 (Ch 0xCA, parity 0x96, Maj 0xE8),
// e + k + w and rotl(a, 5) + f + (e + k + w) one v_add3 each -- five VALU
// per round, where the plain expressions took about eight (a lone packet's
// MAC is this chain: the per-packet path's latency).
__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); k = 0x5A827999u; }
        else if (t < 40) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0x6ED9EBA1u; }
        else if (t < 60) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); k = 0x8F1BBCDCu; }
        else { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0xCA62C1D6u; }
        const uint32_t ekw = e + k + wt;
        const uint32_t tmp = rotl(a, 5) + f + ekw;
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// ------------------------------------------------------ progress priority
// The AES kernels run one workgroup of 16 waves per CU (the LDS image), all
// waves with the same work.  The SIMD arbiter favours older waves, so without
// help the waves of a SIMD finish one after another and the last ones run
// with nothing to hide their LDS latency.  SRTP_PRIO: each wave lowers its
// issue priority as it advances through its packets, so they stay abreast.
#ifndef SRTP_PRIO
#define SRTP_PRIO 1
#endif
__device__ __forceinline__ int wave_max_i(int x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = max(x, __shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ void progress_prio(int b, int nbw) {
#if SRTP_PRIO
    const int q = __builtin_amdgcn_readfirstlane((4 * b) / (nbw + 1));
    if (q <= 0) __builtin_amdgcn_s_setprio(3);
    else if (q == 1) __builtin_amdgcn_s_setprio(2);
    else if (q == 2) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
#else
    (void)b; (void)nbw;
#endif
}

// ------------------------------------------------- fused AES-CM + SHA-1 step
// One SHA-1 round t (compile-time after unrolling) on working state v[0..4].
template <int t>
__device__ __forceinline__ void sha1_round(uint32_t v[5], uint32_t w[16]) {
    uint32_t wt;
    if (t < 16) {
        wt = w[t];
    } else {
        wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
        w[t & 15] = wt;
    }
    const uint32_t b = v[1], c = v[2], d = v[3];
    uint32_t f, k;
    if (t < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
    else if (t < 40) { f = xor3(b, c, d); k = 0x6ED9EBA1u; }
    else if (t < 60) { f = (b & c) | (d & (b | c)); k = 0x8F1BBCDCu; }
    else { f = xor3(b, c, d); k = 0xCA62C1D6u; }
    const uint32_t tmp = rotl(v[0], 5) + f + v[4] + k + wt;
    v[4] = d; v[3] = c; v[2] = rotl(b, 30); v[1] = v[0]; v[0] = tmp;
}

template <int t0>
__device__ __forceinline__ void sha1_rounds4(uint32_t v[5], uint32_t w[16]) {
    sha1_round<t0>(v, w); sha1_round<t0 + 1>(v, w);
    sha1_round<t0 + 2>(v, w); sha1_round<t0 + 3>(v, w);
}

// One middle AES round (1..9) / the last round on two interleaved blocks:
// hand-scheduled asm (aes_rounds_asm.inc, generated by tools/gen_aes_asm.py),
// which needs the T-table image at LDS address 0 -- s_te is the only LDS
// object of the AES kernels.
// (tools/build_variant.sh may compile a candidate schedule in its place)
#ifndef SRTP_AES_ROUNDS
#define SRTP_AES_ROUNDS "aes_rounds_asm.inc"
#endif
#include SRTP_AES_ROUNDS

__device__ __forceinline__ void aes_round2(const char *__restrict__ lds, const TeBase &tb,
                                           const uint32_t *rkr, uint32_t a[4], uint32_t b[4]) {
    (void)lds;
    aes_round2_asm(a, b, tb.b, rkr);
}

__device__ __forceinline__ void aes_last2(const char *__restrict__ lds, const TeBase &tb,
                                          const uint32_t *rkr, uint32_t a[4], uint32_t b[4]) {
    (void)lds;
    aes_last2_asm(a, b, tb.b, rkr);
}

// FIPS-197 AES-128 on two independent blocks (interleaved for ILP), each held
// as four little-endian column words (byte r of word j = state row r, column
// j).  Output column j, row r comes from input column j+r (ShiftRows), looked
// up in T_r (MixColumns coefficients rotated by row).
__device__ __forceinline__ void aes_encrypt2(const char *__restrict__ lds, const TeBase &tb,
                                             const RoundKeys &rk, uint32_t a[4], uint32_t b[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) { a[j] ^= rk.k[j]; b[j] ^= rk.k[j]; }
#pragma unroll
    for (int r = 1; r < 10; r++) aes_round2(lds, tb, rk.k + 4 * r, a, b);
    aes_last2(lds, tb, rk.k + 40, a, b);
}

// ------------------------------------------- AES-CM rounds 1-2, precomputed
// Counter blocks of one packet differ only in IV bytes 14-15, and for block
// index j < 256 only in byte 15 (row 3 of column 3).  After AddRoundKey and
// round 1 that byte reaches output column 0 alone (through T3); in round 2
// that column reaches each output column through exactly one lookup.  So per
// packet: p0 = the constant part of round-1 column 0, r[0..3] = the constant
// parts of the round-2 columns (27 lookups once), and per block only
//     u0 = p0 ^ T3[j ^ kb];   s = (r0 ^ T0[u0.b0], r1 ^ T3[u0.b3],
//                                 r2 ^ T2[u0.b2], r3 ^ T1[u0.b1])
// -- 5 lookups instead of 32 for rounds 1-2 (133 instead of 160 per block).
struct CtrPre {
    uint32_t p0, r[4], kb;
};

__device__ __forceinline__ void ctr_precompute(const char *__restrict__ lds, const TeBase &tb,
                                               const uint32_t *rk, const uint32_t iv[4],
                                               CtrPre &cp) {
    // rk: round keys 0..2 (12 words)
    const uint32_t w0 = iv[0] ^ rk[0], w1 = iv[1] ^ rk[1], w2 = iv[2] ^ rk[2];
    const uint32_t w3 = iv[3] ^ rk[3]; // bytes 14-15 of iv are zero (counter slot)
    cp.kb = w3 >> 24;
    cp.p0 = xor3(TL(w0, 0, 0), TL(w1, 1, 1), TL(w2, 2, 2)) ^ rk[4];
    const uint32_t u1 = xor3(TL(w1, 0, 0), TL(w2, 1, 1), TL(w3, 2, 2)) ^ TL(w0, 3, 3) ^ rk[5];
    const uint32_t u2 = xor3(TL(w2, 0, 0), TL(w3, 1, 1), TL(w0, 2, 2)) ^ TL(w1, 3, 3) ^ rk[6];
    const uint32_t u3 = xor3(TL(w3, 0, 0), TL(w0, 1, 1), TL(w1, 2, 2)) ^ TL(w2, 3, 3) ^ rk[7];
    cp.r[0] = xor3(TL(u1, 1, 1), TL(u2, 2, 2), TL(u3, 3, 3)) ^ rk[8];
    cp.r[1] = xor3(TL(u1, 0, 0), TL(u2, 1, 1), TL(u3, 2, 2)) ^ rk[9];
    cp.r[2] = xor3(TL(u2, 0, 0), TL(u3, 1, 1), TL(u1, 3, 3)) ^ rk[10];
    cp.r[3] = xor3(TL(u3, 0, 0), TL(u1, 2, 2), TL(u2, 3, 3)) ^ rk[11];
}

// State after round 2 (round key 2 included) of counter blocks ja and jb
// (both < 256).
__device__ __forceinline__ void ctr_first2(const char *__restrict__ lds, const TeBase &tb,
                                           const CtrPre &cp, int ja, int jb, uint32_t a[4],
                                           uint32_t b[4]) {
    const uint32_t xa = (uint32_t)ja ^ cp.kb, xb = (uint32_t)jb ^ cp.kb;
    const uint32_t ua = cp.p0 ^ TL(xa, 0, 3), ub = cp.p0 ^ TL(xb, 0, 3);
    a[0] = cp.r[0] ^ TL(ua, 0, 0); b[0] = cp.r[0] ^ TL(ub, 0, 0);
    a[1] = cp.r[1] ^ TL(ua, 3, 3); b[1] = cp.r[1] ^ TL(ub, 3, 3);
    a[2] = cp.r[2] ^ TL(ua, 2, 2); b[2] = cp.r[2] ^ TL(ub, 2, 2);
    a[3] = cp.r[3] ^ TL(ua, 1, 1); b[3] = cp.r[3] ^ TL(ub, 1, 1);
}

// True when a counter block of this chunk step could reach index 256 (IV
// byte 14 no longer zero: the precompute does not apply), on any active lane.
__device__ __forceinline__ bool ctr_pre_exhausted(int j0) {
    return __ballot(j0 + 3 >= 256) != 0ull;
}

__device__ __forceinline__ void ctr_apply(Ctr &cs, int c, const uint32_t K[16], uint32_t d[16]);

// ctr_chunk with rounds 1-2 from the counter precompute when no active lane's
// blocks of chunk c reach index 256 (otherwise the full rounds).
__device__ __forceinline__ void ctr_chunk_pre(const char *__restrict__ lds, const TeBase &tb,
                                              const RoundKeys &rk, const CtrPre &cp, Ctr &cs, int c,
                                              uint32_t d[16]) {
    const int j0 = 4 * c - (cs.off >> 4);
    if (ctr_pre_exhausted(j0)) {
        ctr_chunk(lds, tb, rk, cs, c, d);
        return;
    }
    uint32_t K[16];
#pragma unroll 1
    for (int pr = 0; pr < 2; pr++) {
        uint32_t x[4], y[4];
        ctr_first2(lds, tb, cp, j0 + 2 * pr, j0 + 2 * pr + 1, x, y);
#pragma unroll
        for (int r = 3; r < 10; r++) aes_round2(lds, tb, rk.k + 4 * r, x, y);
        aes_last2(lds, tb, rk.k + 40, x, y);
#pragma unroll
        for (int k = 0; k < 8; k++) K[k] = K[k + 8];
#pragma unroll
        for (int k = 0; k < 4; k++) { K[8 + k] = x[k]; K[12 + k] = y[k]; }
    }
    ctr_apply(cs, c, K, d);
}

// Half P (0/1) of the interleaved chunk step: keystream blocks j0+2P, j0+2P+1
// into K8[8] and SHA-1 rounds 40P .. 40P+39 on v / w.  Rounds 1-2 come from
// the counter precompute (8 SHA-1 rounds beside them), then after each
// remaining AES round of the block pair come four SHA-1 rounds, so the VALU
// work of the hash fills the LDS latency of the table lookups.  Straight-line
// code, no branches.
template <int P>
__device__ __forceinline__ void ks_sha_half(const char *__restrict__ lds, const TeBase &tb,
                                            const RoundKeys &rk, const CtrPre &cp, int j0,
                                            uint32_t K8[8], uint32_t v[5], uint32_t w[16]) {
    uint32_t x[4], y[4];
    constexpr int t = 40 * P;
    ctr_first2(lds, tb, cp, j0 + 2 * P, j0 + 2 * P + 1, x, y);
    sha1_rounds4<t + 0>(v, w); sha1_rounds4<t + 4>(v, w);
    // rounds 3..10: SHA-1 rounds t+8 .. t+39 inside the round asm, at its LDS
    // wait points (aes_rounds_asm.inc)
    aes_round2_sha<t + 8>(x, y, tb.b, rk.k + 12, v, w);
    aes_round2_sha<t + 12>(x, y, tb.b, rk.k + 16, v, w);
    aes_round2_sha<t + 16>(x, y, tb.b, rk.k + 20, v, w);
    aes_round2_sha<t + 20>(x, y, tb.b, rk.k + 24, v, w);
    aes_round2_sha<t + 24>(x, y, tb.b, rk.k + 28, v, w);
    aes_round2_sha<t + 28>(x, y, tb.b, rk.k + 32, v, w);
    aes_round2_sha<t + 32>(x, y, tb.b, rk.k + 36, v, w);
    aes_last2_sha<t + 36>(x, y, tb.b, rk.k + 40, v, w);
#pragma unroll
    for (int k = 0; k < 4; k++) { K8[k] = x[k]; K8[4 + k] = y[k]; }
}

// ------------------------------------------------ per-lane key schedule
// A wave whose packets belong to several session-key sets (a bridge's many
// DTLS sessions in one bundle) runs every lane at once on its own keys rather
// than one pass per key set (for_each_keyset: k passes for k key sets).  The
// lane holds round keys 0-2 of its key set (loaded once per packet) and
// derives rounds 3..10 on the fly (FIPS-197 5.2), four S-box lookups from the
// LDS T-table image per round key: S(x) is byte 1 of T0[x], so byte j of the
// rotated word comes from the table whose rotation puts S there.  Per block
// pair that is 32 lookups and ~90 VALU more than the SGPR path's 266 lookups;
// a wave of k > 1 key sets costs ~1.15 passes instead of k.
__device__ __forceinline__ void key_next(const char *__restrict__ lds, const TeBase &tb, uint32_t k[4],
                                         uint32_t rcon) {
    const uint32_t w3 = k[3];
    // SubWord(RotWord(w3)) in little-endian column words: S[a1] | S[a2] << 8 |
    // S[a3] << 16 | S[a0] << 24, with a_j = byte j of w3
    const uint32_t t3 = TL(w3, 1, 3), t0 = TL(w3, 2, 0), t1 = TL(w3, 3, 1), t2 = TL(w3, 0, 2);
    const uint32_t lo = __builtin_amdgcn_perm(t0, t3, 0x0c0c0500u); // S[a1], S[a2]
    const uint32_t hi = __builtin_amdgcn_perm(t2, t1, 0x07020c0cu); // S[a3], S[a0]
    k[0] = xor3(k[0], lo | hi, rcon);
    k[1] ^= k[0];
    k[2] ^= k[1];
    k[3] ^= k[2];
}

constexpr uint32_t kRcon[11] = {0x00, 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};

// aes_encrypt2 with the lane's own key schedule from round key 0 (k0).
__device__ __forceinline__ void aes_encrypt2_v(const char *__restrict__ lds, const TeBase &tb,
                                               const uint32_t k0[4], uint32_t a[4], uint32_t b[4]) {
    uint32_t k[4] = {k0[0], k0[1], k0[2], k0[3]};
#pragma unroll
    for (int j = 0; j < 4; j++) { a[j] ^= k[j]; b[j] ^= k[j]; }
#pragma unroll
    for (int r = 1; r < 10; r++) {
        key_next(lds, tb, k, kRcon[r]);
        aes_round2_asm_v(a, b, tb.b, k);
    }
    key_next(lds, tb, k, kRcon[10]);
    aes_last2_asm_v(a, b, tb.b, k);
}

// ks_sha_half<P> with the lane's own round keys: k2 = round key 2 (rounds 1-2
// come from the counter precompute, made with the lane's keys 0-2).
template <int P>
__device__ __forceinline__ void ks_sha_half_v(const char *__restrict__ lds, const TeBase &tb,
                                              const uint32_t k2[4], const CtrPre &cp, int j0,
                                              uint32_t K8[8], uint32_t v[5], uint32_t w[16]) {
    uint32_t x[4], y[4];
    constexpr int t = 40 * P;
    ctr_first2(lds, tb, cp, j0 + 2 * P, j0 + 2 * P + 1, x, y);
    sha1_rounds4<t + 0>(v, w); sha1_rounds4<t + 4>(v, w);
    uint32_t k[4] = {k2[0], k2[1], k2[2], k2[3]};
    key_next(lds, tb, k, kRcon[3]); aes_round2_sha_v<t + 8>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[4]); aes_round2_sha_v<t + 12>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[5]); aes_round2_sha_v<t + 16>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[6]); aes_round2_sha_v<t + 20>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[7]); aes_round2_sha_v<t + 24>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[8]); aes_round2_sha_v<t + 28>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[9]); aes_round2_sha_v<t + 32>(x, y, tb.b, k, v, w);
    key_next(lds, tb, k, kRcon[10]); aes_last2_sha_v<t + 36>(x, y, tb.b, k, v, w);
#pragma unroll
    for (int q = 0; q < 4; q++) { K8[q] = x[q]; K8[4 + q] = y[q]; }
}

// The round keys a packet runs with.  LK = false: the wave-uniform key set's
// 44 words in SGPRs; LK = true: the lane's own round keys 0-2 (the rest are
// derived per block pair, above).
template <bool LK> struct PktKeys;
template <> struct PktKeys<false> {
    RoundKeys rk;
};
template <> struct PktKeys<true> {
    uint32_t r[12];
};

__device__ __forceinline__ void ctr_apply(Ctr &cs, int c, const uint32_t K[16], uint32_t d[16]);

__device__ __forceinline__ void ctr_chunk_v(const char *__restrict__ lds, const TeBase &tb,
                                            const uint32_t k0[4], Ctr &cs, int c, uint32_t d[16]) {
    const int j0 = 4 * c - (cs.off >> 4);
    uint32_t K[16];
#pragma unroll 1
    for (int pr = 0; pr < 2; pr++) {
        uint32_t x[4], y[4];
        ctr_input(cs.iv, j0 + 2 * pr, x);
        ctr_input(cs.iv, j0 + 2 * pr + 1, y);
        aes_encrypt2_v(lds, tb, k0, x, y);
#pragma unroll
        for (int k = 0; k < 8; k++) K[k] = K[k + 8];
#pragma unroll
        for (int k = 0; k < 4; k++) { K[8 + k] = x[k]; K[12 + k] = y[k]; }
    }
    ctr_apply(cs, c, K, d);
}

// The key-set-agnostic forms the packet functions call (pk_load: after
// load_round_keys_uniform below).
__device__ __forceinline__ const uint32_t *pk_words(const PktKeys<false> &pk) { return pk.rk.k; }
__device__ __forceinline__ const uint32_t *pk_words(const PktKeys<true> &pk) { return pk.r; }

template <int P>
__device__ __forceinline__ void pk_half(const char *__restrict__ lds, const TeBase &tb, const PktKeys<false> &pk,
                                        const CtrPre &cp, int j0, uint32_t K8[8], uint32_t v[5], uint32_t w[16]) {
    ks_sha_half<P>(lds, tb, pk.rk, cp, j0, K8, v, w);
}
template <int P>
__device__ __forceinline__ void pk_half(const char *__restrict__ lds, const TeBase &tb, const PktKeys<true> &pk,
                                        const CtrPre &cp, int j0, uint32_t K8[8], uint32_t v[5], uint32_t w[16]) {
    ks_sha_half_v<P>(lds, tb, pk.r + 8, cp, j0, K8, v, w);
}

__device__ __forceinline__ void pk_chunk(const char *__restrict__ lds, const TeBase &tb, const PktKeys<false> &pk,
                                         Ctr &cs, int c, uint32_t d[16]) {
    ctr_chunk(lds, tb, pk.rk, cs, c, d);
}
__device__ __forceinline__ void pk_chunk(const char *__restrict__ lds, const TeBase &tb, const PktKeys<true> &pk,
                                         Ctr &cs, int c, uint32_t d[16]) {
    ctr_chunk_v(lds, tb, pk.r, cs, c, d);
}

__device__ __forceinline__ void pk_chunk_pre(const char *__restrict__ lds, const TeBase &tb,
                                             const PktKeys<false> &pk, const CtrPre &cp, Ctr &cs, int c,
                                             uint32_t d[16]) {
    ctr_chunk_pre(lds, tb, pk.rk, cp, cs, c, d);
}
__device__ __forceinline__ void pk_chunk_pre(const char *__restrict__ lds, const TeBase &tb,
                                             const PktKeys<true> &pk, const CtrPre &cp, Ctr &cs, int c,
                                             uint32_t d[16]) {
    const int j0 = 4 * c - (cs.off >> 4);
    if (ctr_pre_exhausted(j0)) {
        ctr_chunk_v(lds, tb, pk.r, cs, c, d);
        return;
    }
    uint32_t K[16];
#pragma unroll 1
    for (int pr = 0; pr < 2; pr++) {
        uint32_t x[4], y[4];
        ctr_first2(lds, tb, cp, j0 + 2 * pr, j0 + 2 * pr + 1, x, y);
        uint32_t k[4] = {pk.r[8], pk.r[9], pk.r[10], pk.r[11]};
#pragma unroll
        for (int r = 3; r < 10; r++) {
            key_next(lds, tb, k, kRcon[r]);
            aes_round2_asm_v(x, y, tb.b, k);
        }
        key_next(lds, tb, k, kRcon[10]);
        aes_last2_asm_v(x, y, tb.b, k);
#pragma unroll
        for (int q = 0; q < 8; q++) K[q] = K[q + 8];
#pragma unroll
        for (int q = 0; q < 4; q++) { K[8 + q] = x[q]; K[12 + q] = y[q]; }
    }
    ctr_apply(cs, c, K, d);
}


// XOR keystream K (blocks 4c - off/16 .. +3, see ctr_chunk) into the chunk
// words d[] of chunk c, within [off, end); advances the carry.
__device__ __forceinline__ void ctr_apply(Ctr &cs, int c, const uint32_t K[16], uint32_t d[16]) {
    const int s = (cs.off >> 2) & 3;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t a0 = K[i];
        const uint32_t a1 = i >= 1 ? K[i - 1] : cs.carry[3 + i];
        const uint32_t a2 = i >= 2 ? K[i - 2] : cs.carry[2 + i];
        const uint32_t a3 = i >= 3 ? K[i - 3] : cs.carry[1 + i];
        const uint32_t ksw = (s & 2) ? ((s & 1) ? a3 : a2) : ((s & 1) ? a1 : a0);
        // branch-free byte mask of [off, end) over this word (off is a multiple
        // of 4): keeps the loop body one basic block
        const int pos = 64 * c + 4 * i;
        const int valid = min(max(cs.end - pos, 0), 4);
        uint32_t m = (uint32_t)((1ull << (8 * valid)) - 1ull);
        m = pos >= cs.off ? m : 0u;
        d[i] ^= ksw & m;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) cs.carry[k] = K[12 + k];
}

// ctr_apply for a chunk wholly inside the ciphered range (64c >= off and
// 64c + 64 <= end) with the keystream shift S = (off >> 2) & 3 known: one XOR
// per word, no byte masks or shift selects.
template <int S>
__device__ __forceinline__ void ctr_apply_full(Ctr &cs, const uint32_t K[16], uint32_t d[16]) {
#pragma unroll
    for (int i = 0; i < 16; i++) d[i] ^= (i >= S) ? K[i - S] : cs.carry[4 + i - S];
#pragma unroll
    for (int k = 0; k < 4; k++) cs.carry[k] = K[12 + k];
}

// ctr_apply with the unmasked form when the whole wave allows it (the steady
// state of the fused loops: headers of one length class, interior chunks).
__device__ __forceinline__ void ctr_apply_wave(Ctr &cs, int c, const uint32_t K[16], uint32_t d[16]) {
    const int s = (cs.off >> 2) & 3;
    const int su = (int)__builtin_amdgcn_readfirstlane(s);
    const bool odd = s != su || 64 * c < cs.off || 64 * c + 64 > cs.end;
    if (__ballot(odd) == 0ull) {
        if (su == 0) ctr_apply_full<0>(cs, K, d);
        else if (su == 1) ctr_apply_full<1>(cs, K, d);
        else if (su == 2) ctr_apply_full<2>(cs, K, d);
        else ctr_apply_full<3>(cs, K, d);
    } else {
        ctr_apply(cs, c, K, d);
    }
}

// Message word (big-endian) at byte position pos of the HMAC inner stream
// pkt[0..mac_len) || u32_be(suffix) || 0x80 || 0...  where d is the LE packet
// word at pos (ignored where pos >= mac_len).
__device__ __forceinline__ uint32_t tail_word(uint32_t d, int pos, int mac_len, uint32_t suffix) {
    int x = pos - mac_len;
    if (x <= -4) return bswap(d);
    if (x >= 5) return 0u;
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        int y = x + i;
        uint32_t byte;
        if (y < 0) byte = (d >> (8 * i)) & 0xffu;
        else if (y < 4) byte = (suffix >> (24 - 8 * y)) & 0xffu;
        else if (y == 4) byte = 0x80u;
        else byte = 0u;
        w |= byte << (24 - 8 * i);
    }
    return w;
}

// HMAC inner block b as SHA-1 message words.  d[16] holds the LE packet words
// at bytes 64b.. (only bytes below mac_len are used); blocks past the data see
// the ROC/index suffix, the 0x80 pad and the 64-bit length.
__device__ __forceinline__ void inner_words(uint32_t w[16], int b, int mac_len, uint32_t suffix) {
    const int nb_full = mac_len >> 6;
    const int nb_inner = ((mac_len + 12) >> 6) + 1;
    if (b < nb_full) {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = bswap(w[k]);
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = tail_word(w[k], 64 * b + 4 * k, mac_len, suffix);
        if (b == nb_inner - 1) {
            w[14] = 0u;
            w[15] = (uint32_t)(64 + mac_len + 4) * 8u;
        }
    }
}

// HMAC outer block: w = inner digest || padding, h = opad midstate.  UNIFORM:
// ks is the same for every active lane (the packet kernels, which loop over
// the wave's key sets), so the midstate is read into SGPRs; otherwise (k_walk's
// re-check, one context per lane) each lane reads its own key set's.
template <bool UNIFORM = true>
__device__ __forceinline__ void outer_words(uint32_t w[16], uint32_t h[5], const KeySet *ks) {
#pragma unroll
    for (int k = 0; k < 5; k++) {
        w[k] = h[k];
        h[k] = UNIFORM ? (uint32_t)__builtin_amdgcn_readfirstlane((int)ks->opad[k]) : ks->opad[k];
    }
    w[5] = 0x80000000u;
#pragma unroll
    for (int k = 6; k < 15; k++) w[k] = 0u;
    w[15] = (64 + 20) * 8;
}

// The first T (<= 12) bytes of the big-endian digest h, as stored / compared
// at p (byte accesses: tags sit at arbitrary alignment).  Fully unrolled so h
// stays in registers.
__device__ __forceinline__ bool tag_matches(const uint32_t h[5], const uint8_t *p, int T) {
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        uint32_t got = 0u, mask = 0u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int idx = 4 * k + i;
            if (idx < T) {
                got |= ld_u8(p + idx) << (24 - 8 * i);
                mask |= 0xffu << (24 - 8 * i);
            }
        }
        ok &= ((got ^ h[k]) & mask) == 0u;
    }
    return ok;
}

// Word i (0..7, lane-varying) of w[8] by selects: no dynamic register index.
__device__ __forceinline__ uint32_t pick8(const uint32_t w[8], int i) {
    const bool o = i & 1;
    const uint32_t a0 = o ? w[1] : w[0], a1 = o ? w[3] : w[2], a2 = o ? w[5] : w[4], a3 = o ? w[7] : w[6];
    const uint32_t b0 = (i & 2) ? a1 : a0, b1 = (i & 2) ? a3 : a2;
    return (i & 4) ? b1 : b0;
}

// tag_matches for the tag at byte `at` of a packet whose region starts 16-B
// aligned (k_unprotect, once per packet after the MAC): the aligned 16-B
// piece(s) holding the compared bytes in one or two vector loads instead of a
// byte load per tag byte.  The second piece is loaded only when a compared
// byte lies in it, so both lie inside the packet's region.
__device__ __forceinline__ bool tag_matches_at(const uint32_t h[5], const uint8_t *pkt, int at, int T) {
    if (at < 0) return tag_matches(h, pkt + at, T);
    const int Tc = min(T, 12), sh = at & 15;
    const uint4 *q = reinterpret_cast<const uint4 *>(pkt + (at - sh));
    const uint4 v0 = q[0];
    const uint4 v1 = sh + Tc > 16 ? q[1] : make_uint4(0u, 0u, 0u, 0u);
    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const int s4 = sh >> 2, sb = sh & 3;
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        // the little-endian word at byte sh + 4k, as the digest's big-endian word k
        const uint32_t le = __builtin_amdgcn_alignbyte(pick8(w, s4 + k + 1), pick8(w, s4 + k), (uint32_t)sb);
        const int nb = min(max(Tc - 4 * k, 0), 4);
        const uint32_t mask = nb ? 0xffffffffu << (8 * (4 - nb)) : 0u;
        ok &= ((bswap(le) ^ h[k]) & mask) == 0u;
    }
    return ok;
}

// The trailer (SRTCP: the E|index word, then the tag's first min(T, 12)
// bytes) at a 4-byte-aligned address: a store per word and one short / byte
// store for the tag's last bytes -- three stores for an 80-bit tag instead of
// ten byte stores (k_protect: 7 us per 2^18-packet bundle).
__device__ __forceinline__ void trailer_write_aligned(uint32_t *q, bool rtcp, uint32_t suffix,
                                                      const uint32_t h[5], int T) {
    if (rtcp) *q++ = bswap(suffix);
    const int Tc = min(T, 12), nw = Tc >> 2, rem = Tc & 3;
#pragma unroll
    for (int k = 0; k < 3; k++)
        if (k < nw) q[k] = bswap(h[k]);
    if (rem) {
        const uint32_t hw = bswap(nw == 0 ? h[0] : nw == 1 ? h[1] : h[2]);
        uint8_t *tp = reinterpret_cast<uint8_t *>(q + nw);
        if (rem >= 2) *reinterpret_cast<uint16_t *>(tp) = (uint16_t)hw;
        if (rem == 3) tp[2] = (uint8_t)(hw >> 16);
        if (rem == 1) tp[0] = (uint8_t)hw;
    }
}

__device__ __forceinline__ void tag_write(const uint32_t h[5], uint8_t *p, int T) {
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (4 * k + i < T) p[4 * k + i] = (uint8_t)(h[k] >> (24 - 8 * i));
}

// ------------------------------------------------------- RawPacket helpers
// getHeaderLength (RawPacket.java:602-614) with the signed extension length
// (:544-556); kHdrThrow when reading the extension length leaves the buffer.
__device__ __forceinline__ int32_t rtp_header_len(const uint8_t *pkt, uint32_t b0, int cap) {
    int cc = (int)(b0 & 0x0fu);
    int h = 12 + 4 * cc;
    if (b0 & 0x10u) {
        int idx = 12 + cc * 4 + 2;
        if (idx + 1 >= cap) return kHdrThrow;
        int ext = ((int)(int8_t)ld_u8(pkt + idx) * 256) | (int)ld_u8(pkt + idx + 1);
        h += 4 + ext * 4;
    }
    return h;
}

// SRTPCipherCTR.process would throw on region [h, h+plen) (SRTPCipherCTR.java:99-120)
__device__ __forceinline__ bool ctr_would_throw(int32_t h, int plen) {
    if (h == kHdrThrow) return true;
    if (plen < 0) return (plen % 16) != 0;
    return plen > 0 && h < 0;
}

// The cipher of policy `enc` would throw on region [h, h+plen): AES-CM as
// above; AES-F8 (SRTPCipherF8.process :97-128) only when the header length
// throws or a block is XORed at a negative offset (a negative length ciphers
// nothing and a non-negative offset stays inside the packet).
__device__ __forceinline__ bool enc_would_throw(int enc, int32_t h, int plen) {
    if (enc == SRTP_AESCM_ENCRYPTION || enc == SRTP_TWOFISH_ENCRYPTION) return ctr_would_throw(h, plen);
    if (enc == SRTP_AESF8_ENCRYPTION || enc == SRTP_TWOFISHF8_ENCRYPTION)
        return h == kHdrThrow || (plen > 0 && h < 0);
    return false;
}

// Packet p's {g0, auth_ok} (BundleArgs::gok): one 8-B load.
__device__ __forceinline__ uint2 gok_of(const BundleArgs &a, uint32_t p) {
    return reinterpret_cast<const uint2 *>(a.gok)[p];
}

__device__ __forceinline__ int32_t packet_tid(const BundleArgs &a, uint32_t p) {
    return a.tids ? a.tids[p] : a.tid;
}

// Index of a final status in the engine's status counters: a bundle former's
// hole (SKIPPED, no transformer: srtp_aggregator_* seals unclaimed entries so)
// is counted apart from the packets the caller skipped (srtp_stats.holes).
__device__ __forceinline__ uint32_t status_counter(const BundleArgs &a, uint32_t p, int32_t st) {
    if (st == SRTP_STATUS_SKIPPED && packet_tid(a, p) < 0) return kStatusHole;
    return (uint32_t)st & 15u;
}

// ------------------------------------------------------- context hash table
// Linear probing over (transformer << 32 | SSRC) keys.  A key absent from the
// table is inserted into the first tombstone of its probe path (slots freed by
// transformer close or abort rollback), else into the empty slot that ended
// the path; a lost race for that slot re-probes.  Two lanes inserting the same
// key see the same path, so the loser finds the winner's key.
__device__ uint32_t ctx_lookup_insert(const BundleArgs &a, uint64_t key, bool may_create,
                                      uint32_t ks_new, bool *created) {
    *created = false;
    const uint32_t mask = a.ctx_mask;
    const uint32_t h0 = (uint32_t)mix64(key) & mask;
    for (int attempt = 0; attempt < 64; attempt++) {
        uint32_t h = h0, tomb = kNoSlot, target = kNoSlot;
        for (uint32_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
            const uint64_t cur =
                __hip_atomic_load(&a.ctx_keys[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == key) return h;
            if (cur == kTombKey) {
                if (tomb == kNoSlot) tomb = h;
                continue;
            }
            if (cur == kEmptyKey) {
                target = tomb != kNoSlot ? tomb : h;
                break;
            }
        }
        if (target == kNoSlot) target = tomb; // whole table probed: only tombstones free
        if (!may_create || target == kNoSlot) return kNoSlot;
        const uint64_t expect = target == tomb ? kTombKey : kEmptyKey;
        const unsigned long long prev = atomicCAS((unsigned long long *)&a.ctx_keys[target],
                                                  (unsigned long long)expect,
                                                  (unsigned long long)key);
        if (prev == expect) {
            CtxState s;
            s.ks = ks_new; s.a = 0; s.b = 0; s.g = 0; s.window = 0; s.flags = 0;
            s.birth = a.serial;
            a.ctx[target] = s;
            *created = true;
            return target;
        }
        if (prev == key) return target;
        // another key took the slot: probe again
    }
    return kNoSlot;
}

// ============================================================== k_parse
// Returns the packet's sort key: its context slot, or ctx_mask + 1 when the
// packet is not walked (skipped, invalid, dropped before the state machine).
__device__ __forceinline__ uint32_t parse_one(const BundleArgs &a, uint32_t p) {
    uint32_t invalid_key = a.ctx_mask + 1u;
    // the per-packet words first, all in flight together; then the transformer
    // record and the header (when the packet has a valid region) together
    const uint32_t L = a.len[p];
    const uint32_t fl = a.flags ? a.flags[p] : 0u;
    const int32_t tid = packet_tid(a, p);
    const uint32_t C = a.cap[p];
    const uint32_t o = a.off[p];
    a.sk_in[p] = invalid_key;
    a.p_slot[p] = kNoSlot;
    a.w_len[p] = L;
    if ((fl & SRTP_PKT_FLAG_SKIP) || tid < 0 || (uint32_t)tid >= a.n_transformers) {
        a.w_status[p] = SRTP_STATUS_SKIPPED;
        return invalid_key;
    }
    const bool bad_len = L < 12 || L > C || C > 65535u; // RawPacket.isInvalid :903-909
    const uint8_t *pkt = a.seg + o;
    uint4 hdr = make_uint4(0, 0, 0, 0);
    if (!bad_len) hdr = *reinterpret_cast<const uint4 *>(pkt);
    const TransformerRec tr = a.transformers[tid];
    if (!tr.alive) {
        a.w_status[p] = SRTP_STATUS_SKIPPED;
        return invalid_key;
    }
    if (bad_len) {
        a.w_status[p] = SRTP_STATUS_DROP_INVALID;
        return invalid_key;
    }
    uint32_t b0 = hdr.x & 0xffu;
    uint32_t ssrc;
    if (tr.kind == SRTP_KIND_RTP) {
        // SRTPTransformer.reverseTransform: RTP version 2 only (:189-190)
        if (a.reverse && (b0 & 0xC0u) != 0x80u) {
            a.w_status[p] = SRTP_STATUS_DROP_VERSION;
            return invalid_key;
        }
        ssrc = bswap(hdr.z);  // RawPacket.getSSRC :839
    } else {
        ssrc = bswap(hdr.y);  // RawPacket.getRTCPSSRC :770
    }
    int32_t f = a.reverse ? tr.rev : tr.fwd;
    bool may_create = f >= 0 && a.factories[f].open;
    uint32_t ks_new = 0;
    if (may_create) ks_new = (uint32_t)(tr.kind == SRTP_KIND_RTP ? a.factories[f].ks_rtp
                                                                 : a.factories[f].ks_rtcp);
    uint64_t key = ((uint64_t)(uint32_t)tid << 32) | ssrc;
    bool created;
    // Lanes that share the first active lane's key take its lookup: a bundle
    // dominated by one stream would otherwise send every lane's atomic load
    // to the same table word (one SSRC: parse 67 us instead of 19).
    const unsigned long long act = __ballot(1);
    const int leader = __ffsll((long long)act) - 1;
    const uint32_t klo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, leader);
    const uint32_t khi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), leader);
    const bool same = key == (((uint64_t)khi << 32) | klo);
    uint32_t slot = kNoSlot;
    if (!same || (int)(threadIdx.x & 63u) == leader) slot = ctx_lookup_insert(a, key, may_create, ks_new, &created);
    if (same) slot = (uint32_t)__builtin_amdgcn_readlane((int)slot, leader);
    if (slot == kNoSlot) {
        if (may_create) atomicAdd(&a.counters[kCtrOverflow], 1ull); // table full
        a.w_status[p] = SRTP_STATUS_DROP_NO_CONTEXT;
        return invalid_key;
    }
    a.p_slot[p] = slot;
    WalkRec rec;
    rec.p = p;
    rec.lc = L | (C << 16);
    bool maybe_throw = false;
    if (tr.kind == SRTP_KIND_RTP) {
        rec.word = bswap(hdr.x) & 0xffffu; // RawPacket.getSequenceNumber :804
        if (a.reverse) { // a packet far from its context's s_l (see BundleArgs::far)
            const int32_t sl = a.ctx[slot].b, dist = (int32_t)rec.word - sl;
            if (!(a.ctx[slot].flags & 1u) || dist >= 16384 || dist <= -16384) a.far[slot] = a.serial + 1u;
        }
        rec.h = rtp_header_len(pkt, b0, (int)C);
        if (a.reverse && (fl & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE))) rec.p |= kRecSkipDec;
        // conservative: a throw is possible for some tag length 0..20
        maybe_throw = rec.h == kHdrThrow || rec.h < 0 || (int)L - 20 - rec.h < 0;
    } else if (a.reverse) {
        // E|index word at length - (4 + tag) (RawPacket.getSRTCPIndex :815-819)
        int T;
        if (may_create) T = a.keysets[ks_new].tag_len;
        else T = a.keysets[a.ctx[slot].ks].tag_len; // existing context (no insert possible)
        int io = (int)L - 4 - T;
        rec.word = io >= 0 ? ld_be32(pkt + io) : 0u;
        rec.h = T;
        maybe_throw = (int)L - 4 - 20 - 8 < 0;
    } else {
        rec.word = 0u;
        rec.h = 0;
    }
    if (maybe_throw) atomicOr(&a.ctl->any_throw, 1u);
    a.sk_in[p] = slot;
    a.sv_in[p] = rec;
    a.w_status[p] = kStPending;
    return slot;
}

// One lane per packet; the block also counts the first sort digit of its
// packets' keys into their 2048-record tile (the radix sort's first pass).
#ifndef SRTP_PARSE_BLOCK
#define SRTP_PARSE_BLOCK 256
#endif
constexpr int kParseBlock = SRTP_PARSE_BLOCK; // divides the sort's 2048-record tile
// Length class of a packet for the crypto kernels' lane order: its number of
// 64-B chunks (31: 31 or more).  One lane walks one packet chunk by chunk, so a
// wave lasts as long as its longest packet; grouping packets by class keeps the
// lanes of a wave busy on mixed-size bundles (k_lenperm).
__device__ __forceinline__ uint32_t len_class(uint32_t L) { return min((L + 63u) >> 6, 31u); }
constexpr uint32_t kClsWords = 33; // per tile: 32 class counts + the class mask
// The radix sort's tile (see "radix sort" below): 512 threads x kSortItems records.
#ifndef SRTP_SORT_ITEMS
#define SRTP_SORT_ITEMS 4
#endif
constexpr int kSortThreads = 512, kSortItems = SRTP_SORT_ITEMS, kSortTile = kSortThreads * kSortItems;
static_assert(kSortTile % kParseBlock == 0 && kParseBlock >= 256, "k_parse tiles");
uint32_t sort_tile_records() { return (uint32_t)kSortTile; }

// HB: the first digit's histogram bins (256, or 2^kSortWideMaxBits for the
// wide sort, which uses 2^a.sort_bits of them).
template <int HB>
__global__ __launch_bounds__(kParseBlock) void k_parse(BundleArgs a) {
    __shared__ uint32_t s_hist[HB], s_cls[32];
    const uint32_t bins = HB == 256 ? 256u : 1u << a.sort_bits;
    for (uint32_t d = threadIdx.x; d < bins; d += kParseBlock) s_hist[d] = 0u;
    if (threadIdx.x < 32) s_cls[threadIdx.x] = 0u;
    __syncthreads();
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    // reset the next bundle's control block (the previous bundle, which used
    // it, completed before this kernel started)
    if (p == 0) *a.ctl_next = BundleCtl{};
    if (a.abort_on_error)
        for (uint32_t i = p; i < a.n_transformers; i += gridDim.x * blockDim.x)
            a.e_min_next[i] = 0x7f7f7f7f;
    if (p < a.n) {
        // one LDS atomic per distinct class of the wave (a fixed-size bundle
        // would otherwise send all 256 lanes to one word)
        const uint32_t cls = len_class(a.len[p]);
        const unsigned long long act = __ballot(1);
        const int leader = __ffsll((long long)act) - 1;
        const uint32_t lc = (uint32_t)__builtin_amdgcn_readlane((int)cls, leader);
        const unsigned long long same = __ballot(cls == lc);
        if (cls != lc) atomicAdd(&s_cls[cls], 1u);
        else if ((int)(threadIdx.x & 63u) == leader) atomicAdd(&s_cls[cls], (uint32_t)__popcll(same));
        atomicAdd(&s_hist[parse_one(a, p) & (bins - 1u)], 1u);
    }
    __syncthreads();
    const uint32_t tile = (blockIdx.x * blockDim.x) / (uint32_t)kSortTile; // a multiple of kParseBlock
    for (uint32_t d = threadIdx.x; d < bins; d += kParseBlock)
        if (s_hist[d]) atomicAdd(&a.sort_counts[tile * bins + d], s_hist[d]);
    if (threadIdx.x < 32) { // per sort tile: at most kSortTile / kParseBlock parse blocks share a word
        const uint32_t c = s_cls[threadIdx.x];
        if (c) atomicAdd(&a.cls_tile[tile * kClsWords + threadIdx.x], c);
        const unsigned long long m = __ballot(c != 0u);
        if (threadIdx.x == 0 && (uint32_t)m) atomicOr(&a.cls_tile[tile * kClsWords + 32], (uint32_t)m);
    }
}

// Lane order of the crypto kernels (k_protect, k_unprotect): with packets of
// more than one length class in the bundle, lord[] lists the packets grouped
// by class, the longest class first, so that the lanes of a wave walk packets
// of about the same length.  The radix sort's first scatter pass writes it
// (k_sort_scatter, SortPass::lord); within a class the order is whatever its
// tiles' reservations give, since the crypto kernels treat every packet on its
// own.  A bundle of one class (the fixed-size case) keeps lane = packet.
#ifndef SRTP_LEN_ORDER
#define SRTP_LEN_ORDER 1
#endif

// The packet lane i of a crypto kernel takes (i < a.n).
__device__ __forceinline__ uint32_t lane_packet(const BundleArgs &a, uint32_t i) {
    if (SRTP_LEN_ORDER && __popc(a.ctl->len_classes & ~1u) > 1) return a.lord[i];
    return i;
}

// ============================================================== radix sort
// Stable LSD radix sort of the walk records by context slot, 8-bit digits,
// reduce-then-scan per digit: the digit counts of every 2048-record tile
// (k_parse for the first digit, the previous pass's scatter for the next),
// and one scatter kernel per digit that turns them into its tile's scatter
// bases and ranks the tile's digits stably in LDS.  Two launches for a
// two-digit sort and no memsets: pass q re-zeroes pass q-1's counts, k_walk
// the last pass's.

static inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

size_t sort_temp_bytes(uint32_t n_max) {
    const size_t tiles = (n_max + kSortTile - 1) / kSortTile;
    const size_t wide = align256(tiles << kSortWideMaxBits << 2);
    return align256((size_t)n_max * 4) + align256((size_t)n_max * sizeof(WalkRec)) +
           kSortMaxPass * align256(tiles * 256 * 4) + 3 * wide + align256((size_t)4 << kSortWideMaxBits);
}

SortScratch sort_scratch(void *temp, uint32_t n_max) {
    SortScratch ss;
    char *p = reinterpret_cast<char *>(temp);
    ss.max_tiles = (n_max + kSortTile - 1) / kSortTile;
    const size_t cb = align256((size_t)ss.max_tiles * 256 * 4);
    ss.keys_tmp = reinterpret_cast<uint32_t *>(p); p += align256((size_t)n_max * 4);
    ss.vals_tmp = reinterpret_cast<WalkRec *>(p); p += align256((size_t)n_max * sizeof(WalkRec));
    for (int q = 0; q < kSortMaxPass; q++) { ss.counts[q] = reinterpret_cast<uint32_t *>(p); p += cb; }
    const size_t wide = align256((size_t)ss.max_tiles << kSortWideMaxBits << 2);
    ss.wcounts[0] = reinterpret_cast<uint32_t *>(p); p += wide;
    ss.wcounts[1] = reinterpret_cast<uint32_t *>(p); p += wide;
    ss.wprefix = reinterpret_cast<uint32_t *>(p); p += wide;
    ss.wtotal = reinterpret_cast<uint32_t *>(p);
    return ss;
}

struct SortPass {
    const uint32_t *sk;
    const WalkRec *sv;
    uint32_t *dk;
    WalkRec *dv;
    uint32_t n, shift, tiles;
    const uint32_t *counts;   // this pass's [tiles][256] digit counts
    uint32_t *next_counts;    // next pass's [tiles][256] counts, or null on the last pass
    uint32_t *zero;           // the previous pass's counts (this tile's row is re-zeroed), or null
    uint32_t *spos;           // last unprotect pass: spos[packet] = its sorted position, or null
    uint32_t walk_max;        // largest key of a walked record (the context table's mask)
    // first pass only (else null): the crypto kernels' lane order by length
    // class (see lane_packet); its input records are in packet order
    uint32_t *lord;
    const uint32_t *len;
    BundleCtl *ctl;
    const uint32_t *cls_tile;
};

// The crypto kernels' lane order (first sort pass): this tile's packets by
// length class, at the class bases (longest first) plus a reserved range --
// when the bundle has more than one class (k_parse's per-tile masks).  s_cb
// (32 words) and s_run (97) are LDS the caller no longer needs.
__device__ __forceinline__ void write_lord(uint32_t n, uint32_t tiles, uint32_t tile, uint32_t base,
                                           const uint32_t *len, BundleCtl *ctl, const uint32_t *cls_tile,
                                           uint32_t *lord, uint32_t *s_cb, uint32_t *s_run) {
    const int t = threadIdx.x;
    uint32_t *s_cc = s_run, *s_co = s_run + 32, *s_tot = s_run + 64;
    if (t < 64) {
        uint32_t m = 0u;
        for (uint32_t u = (uint32_t)t; u < tiles; u += 64u) m |= cls_tile[u * kClsWords + 32];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m |= (uint32_t)__shfl_xor((int)m, o);
        if (t == 0) {
            s_run[96] = m;
            if (tile == 0u) ctl->len_classes = m; // read by the crypto kernels' lane_packet
        }
    }
    __syncthreads();
    // one class: lane = packet.  Class 0 (length 0: a bundle former's holes,
    // null elements) runs no crypto and does not count.
    if (__popc(s_run[96] & ~1u) <= 1) return;
    if (t < 32) {
        uint32_t tot = 0u;
        for (uint32_t u = 0u; u < tiles; u++) tot += cls_tile[u * kClsWords + t];
        s_tot[t] = tot;
        s_cc[t] = 0u;
    }
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0u;
        for (int c = 31; c >= 0; c--) {
            s_cb[c] = acc;
            acc += s_tot[c];
        }
    }
    __syncthreads();
    uint32_t cls[kSortItems], rk[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < n) {
            cls[r] = len_class(len[i]);
            rk[r] = atomicAdd(&s_cc[cls[r]], 1u);
        }
    }
    __syncthreads();
    if (t < 32 && s_cc[t]) s_co[t] = atomicAdd(&ctl->cls_cursor[t], s_cc[t]);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < n) lord[s_cb[cls[r]] + s_co[cls[r]] + rk[r]] = i;
    }
}

#ifndef SRTP_SORT_COUNT_LOADS
#define SRTP_SORT_COUNT_LOADS 64
#endif
constexpr int kSortCountLoads = SRTP_SORT_COUNT_LOADS;
static_assert(kSortThreads == 512, "two threads per digit read the count table");
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(SortPass sp) {
    __shared__ uint32_t s_base[256], s_run[256], s_wcnt[kSortThreads / 64][256];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t tile = blockIdx.x, base = tile * kSortTile;
    {
        // scatter base of digit d in this tile = (records with a smaller digit)
        // + (records with digit d in earlier tiles).  Every tile re-reads the
        // whole [tiles][256] count table (128 KB at 2^18 records, L2-resident),
        // which costs less than a separate scan launch.  Thread (g, d) sums
        // digit d over every other tile, kSortCountLoads loads in flight (one
        // round up to 2 x kSortCountLoads tiles: 2^18 records at 64).
        const int d = t & 255, g = t >> 8;
        uint32_t before = 0u, total = 0u;
        for (uint32_t u0 = (uint32_t)g; u0 < sp.tiles; u0 += 2u * kSortCountLoads) {
            uint32_t c[kSortCountLoads];
#pragma unroll
            for (int k = 0; k < kSortCountLoads; k++) {
                const uint32_t u = u0 + 2u * k;
                c[k] = u < sp.tiles ? sp.counts[u * 256u + d] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kSortCountLoads; k++) {
                total += c[k];
                before += u0 + 2u * k < tile ? c[k] : 0u;
            }
        }
        s_wcnt[g][d] = total;
        s_wcnt[2 + g][d] = before;
        if (sp.zero && g == 0) sp.zero[tile * 256u + d] = 0u;
        __syncthreads();
        uint32_t x = 0u;
        if (g == 0) { x = s_wcnt[0][d] + s_wcnt[1][d]; s_run[d] = x; }
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) { // inclusive scan of the digit totals
            const uint32_t y = (g == 0 && d >= o) ? s_run[d - o] : 0u;
            __syncthreads();
            if (g == 0) s_run[d] += y;
            __syncthreads();
        }
        if (g == 0) s_base[d] = s_run[d] - x + s_wcnt[2][d] + s_wcnt[3][d];
        __syncthreads();
        if (t < 256) {
            s_run[t] = 0u;
#pragma unroll
            for (int k = 0; k < kSortThreads / 64; k++) s_wcnt[k][t] = 0u;
        }
    }
    uint32_t key[kSortItems], loc[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < sp.n) key[r] = sp.sk[i];
    }
    __syncthreads();
    // stable local ranks: items in order r-major, t-minor (= index order)
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const bool valid = base + r * kSortThreads + t < sp.n;
        const uint32_t d = valid ? (key[r] >> sp.shift) & 255u : 0u;
        unsigned long long m = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const unsigned long long b = __ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? b : ~b;
        }
        const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        if (valid && below == 0u) s_wcnt[w][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pre = s_run[d];
            for (int k = 0; k < w; k++) pre += s_wcnt[k][d];
            loc[r] = pre + below;
        }
        __syncthreads();
        if (t < 256) {
            uint32_t add = 0u;
#pragma unroll
            for (int k = 0; k < kSortThreads / 64; k++) { add += s_wcnt[k][t]; s_wcnt[k][t] = 0u; }
            s_run[t] += add;
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < sp.n) {
            const uint32_t pos = s_base[(key[r] >> sp.shift) & 255u] + loc[r];
            sp.dk[pos] = key[r];
            const WalkRec rec = sp.sv[i]; // read here, not held across the ranking (a held copy went to scratch)
            sp.dv[pos] = rec;
            // only walked records carry a packet index: k_parse leaves the
            // record of a skipped / invalid packet unwritten (stale scratch,
            // whose index may lie anywhere)
            if (sp.spos && key[r] <= sp.walk_max) sp.spos[rec.p & kRecIdxMask] = pos;
            if (sp.next_counts)
                atomicAdd(&sp.next_counts[(pos / kSortTile) * 256 + ((key[r] >> (sp.shift + 8)) & 255u)], 1u);
        }
    }
    if (SRTP_LEN_ORDER && sp.lord) {
        __syncthreads(); // s_base / s_run / s_wcnt are free again
        write_lord(sp.n, sp.tiles, tile, base, sp.len, sp.ctl, sp.cls_tile, sp.lord, s_base, s_run);
    }
}

// The next pass's digit counts per tile of this pass's output: one workgroup
// per 2048-record tile, an LDS histogram, 256 plain stores (every bin, so the
// table needs no zeroing).  Cheaper than one global atomic per record in the
// scatter (sort 0.045 -> 0.035 ms per bundle without them).
__global__ __launch_bounds__(kSortThreads) void k_sort_count(const uint32_t *keys, uint32_t n, uint32_t shift,
                                                             uint32_t *counts) {
    __shared__ uint32_t s_h[256];
    const uint32_t t = threadIdx.x, base = blockIdx.x * kSortTile;
    if (t < 256) s_h[t] = 0u;
    __syncthreads();
    uint32_t k[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        k[r] = i < n ? keys[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kSortItems; r++)
        if (base + r * kSortThreads + t < n) atomicAdd(&s_h[(k[r] >> shift) & 255u], 1u);
    __syncthreads();
    if (t < 256) counts[blockIdx.x * 256u + t] = s_h[t];
}

// ------------------------------------------------- the two-pass wide sort
// Keys of 17-22 bits (context tables of 2^16-2^21 slots: 40k-1.3M streams)
// in two passes of 9-11-bit digits instead of three of 8.  A digit's scatter
// base can no longer come from each tile re-reading the whole count table
// (2^11 digits x every tile), so a small kernel turns the counts into per-tile
// prefixes and digit totals once per pass (k_sort_prefix); the scatter scans
// the totals itself.

// counts [tiles][B] -> prefix[t][d] = records with digit d in tiles < t, and
// total[d]; counts are zeroed behind (pass 0's table is k_parse's, which
// accumulates with atomics).  Grid B / 64, 1024 threads: 64 digits x 16
// groups of tiles, each thread's loads issued 8 at a time (a thread walking
// its tiles one dependent load after another made this launch the wide
// sort's longest).
constexpr int kPrefixGroups = 16, kPrefixUnroll = 8;
__global__ __launch_bounds__(64 * kPrefixGroups) void k_sort_prefix(uint32_t *counts, uint32_t tiles, uint32_t B,
                                                                   uint32_t *prefix, uint32_t *total) {
    __shared__ uint32_t s_sum[kPrefixGroups][64];
    const uint32_t dl = threadIdx.x & 63u, g = threadIdx.x >> 6, d = blockIdx.x * 64u + dl;
    const uint32_t t0 = tiles * g / kPrefixGroups, t1 = tiles * (g + 1u) / kPrefixGroups;
    uint32_t sum = 0u;
    for (uint32_t u0 = t0; u0 < t1; u0 += kPrefixUnroll) {
        uint32_t c[kPrefixUnroll];
#pragma unroll
        for (int k = 0; k < kPrefixUnroll; k++) c[k] = u0 + k < t1 ? counts[(u0 + k) * B + d] : 0u;
#pragma unroll
        for (int k = 0; k < kPrefixUnroll; k++) sum += c[k];
    }
    s_sum[g][dl] = sum;
    __syncthreads();
    uint32_t run = 0u;
    for (uint32_t k = 0; k < g; k++) run += s_sum[k][dl];
    if (g == kPrefixGroups - 1) total[d] = run + sum;
    for (uint32_t u0 = t0; u0 < t1; u0 += kPrefixUnroll) {
        uint32_t c[kPrefixUnroll];
#pragma unroll
        for (int k = 0; k < kPrefixUnroll; k++) c[k] = u0 + k < t1 ? counts[(u0 + k) * B + d] : 0u;
#pragma unroll
        for (int k = 0; k < kPrefixUnroll; k++) {
            if (u0 + k < t1) {
                prefix[(u0 + k) * B + d] = run;
                counts[(u0 + k) * B + d] = 0u;
                run += c[k];
            }
        }
    }
}

// k_sort_count with B (<= 2^kSortWideMaxBits) bins: every bin stored.
__global__ __launch_bounds__(kSortThreads) void k_sort_count_wide(const uint32_t *keys, uint32_t n, uint32_t shift,
                                                                  uint32_t B, uint32_t *counts) {
    __shared__ uint32_t s_h[1 << kSortWideMaxBits];
    const uint32_t t = threadIdx.x, base = blockIdx.x * kSortTile;
    for (uint32_t d = t; d < B; d += kSortThreads) s_h[d] = 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < n) atomicAdd(&s_h[(keys[i] >> shift) & (B - 1u)], 1u);
    }
    __syncthreads();
    for (uint32_t d = t; d < B; d += kSortThreads) counts[blockIdx.x * B + d] = s_h[d];
}

struct SortPassWide {
    const uint32_t *sk;
    const WalkRec *sv;
    uint32_t *dk;
    WalkRec *dv;
    uint32_t n, shift, bits, tiles;
    const uint32_t *prefix, *total;
    uint32_t *spos;
    uint32_t walk_max;
    uint32_t *lord;
    const uint32_t *len;
    BundleCtl *ctl;
    const uint32_t *cls_tile;
};

// One wide scatter pass: k_sort_scatter's stable tile ranking with B = 2^bits
// digits (bits ballots per item), bases from k_sort_prefix.
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter_wide(SortPassWide sp) {
    constexpr int HB = 1 << kSortWideMaxBits, W = kSortThreads / 64;
    __shared__ uint32_t s_base[HB], s_run[HB], s_wcnt[W][HB];
    __shared__ uint32_t s_part[W];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t tile = blockIdx.x, base = tile * kSortTile;
    const uint32_t B = 1u << sp.bits, per = B / kSortThreads; // 1, 2 or 4 digits per thread
    {
        // digit offsets: exclusive scan of the totals (thread t owns digits
        // [t * per, t * per + per)), plus this tile's prefix
        uint32_t loc[4], sum = 0u;
        for (uint32_t k = 0; k < per; k++) {
            loc[k] = sp.total[t * per + k];
            sum += loc[k];
        }
        uint32_t x = sum; // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) s_part[w] = x;
        for (uint32_t d = t; d < B; d += kSortThreads) {
            s_run[d] = 0u;
            for (int k = 0; k < W; k++) s_wcnt[k][d] = 0u;
        }
        __syncthreads();
        uint32_t off = x - sum;
        for (int k = 0; k < w; k++) off += s_part[k];
        for (uint32_t k = 0; k < per; k++) {
            const uint32_t d = t * per + k;
            s_base[d] = off + sp.prefix[tile * B + d];
            off += loc[k];
        }
    }
    uint32_t key[kSortItems], loc[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < sp.n) key[r] = sp.sk[i];
    }
    __syncthreads();
    // stable local ranks: items in order r-major, t-minor (= index order)
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const bool valid = base + r * kSortThreads + t < sp.n;
        const uint32_t d = valid ? (key[r] >> sp.shift) & (B - 1u) : 0u;
        unsigned long long m = __ballot(valid);
        for (uint32_t bit = 0; bit < sp.bits; bit++) {
            const unsigned long long b = __ballot((d >> bit) & 1u);
            m &= ((d >> bit) & 1u) ? b : ~b;
        }
        const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
        const uint32_t cnt = (uint32_t)__popcll(m);
        const bool leader = valid && below == 0u;
        if (leader) s_wcnt[w][d] = cnt;
        __syncthreads();
        if (valid) {
            uint32_t pre = s_run[d];
            for (int k = 0; k < w; k++) pre += s_wcnt[k][d];
            loc[r] = pre + below;
        }
        __syncthreads();
        // each wave's leader moves its digit's count into the running totals
        // and clears its own entry (the next item's ranks read both after the
        // next barrier)
        if (leader) {
            atomicAdd(&s_run[d], cnt);
            s_wcnt[w][d] = 0u;
        }
    }
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = base + r * kSortThreads + t;
        if (i < sp.n) {
            const uint32_t pos = s_base[(key[r] >> sp.shift) & (B - 1u)] + loc[r];
            sp.dk[pos] = key[r];
            const WalkRec rec = sp.sv[i];
            sp.dv[pos] = rec;
            if (sp.spos && key[r] <= sp.walk_max) sp.spos[rec.p & kRecIdxMask] = pos;
        }
    }
    if (SRTP_LEN_ORDER && sp.lord) { // as k_sort_scatter (first pass only)
        __syncthreads();
        write_lord(sp.n, sp.tiles, tile, base, sp.len, sp.ctl, sp.cls_tile, sp.lord, s_base, s_run);
    }
}

hipError_t launch_sort_wide(const BundleArgs &a, const SortScratch &ss, hipStream_t s) {
    const uint32_t tiles = (a.n + kSortTile - 1) / kSortTile;
    const uint32_t bits = (uint32_t)a.sort_bits, B = 1u << bits;
    for (int q = 0; q < 2; q++) {
        if (q == 1)
            hipLaunchKernelGGL(k_sort_count_wide, dim3(tiles), dim3(kSortThreads), 0, s, (const uint32_t *)ss.keys_tmp,
                               a.n, bits, B, ss.wcounts[1]);
        hipLaunchKernelGGL(k_sort_prefix, dim3(B / 64u), dim3(64 * kPrefixGroups), 0, s, q == 0 ? a.sort_counts : ss.wcounts[1],
                           tiles, B, ss.wprefix, ss.wtotal);
        SortPassWide sp;
        sp.sk = q == 0 ? a.sk_in : ss.keys_tmp;
        sp.sv = q == 0 ? a.sv_in : ss.vals_tmp;
        sp.dk = q == 0 ? ss.keys_tmp : a.sk_out;
        sp.dv = q == 0 ? ss.vals_tmp : a.sv_out;
        sp.n = a.n;
        sp.shift = bits * (uint32_t)q;
        sp.bits = bits;
        sp.tiles = tiles;
        sp.prefix = ss.wprefix;
        sp.total = ss.wtotal;
        sp.spos = q == 1 && a.reverse ? a.spos : nullptr;
        sp.walk_max = a.ctx_mask;
        sp.lord = q == 0 ? a.lord : nullptr;
        sp.len = a.len;
        sp.ctl = a.ctl;
        sp.cls_tile = a.cls_tile;
        hipLaunchKernelGGL(k_sort_scatter_wide, dim3(tiles), dim3(kSortThreads), 0, s, sp);
    }
    return hipGetLastError();
}

// ------------------------------------------------ one-tile bundles
// A bundle of at most one sort tile (the per-packet path's small bundles: a
// few to a few hundred packets) is sorted by one workgroup in LDS, every
// 8-bit digit in turn -- one launch, where the multi-pass sort takes a
// scatter launch per digit plus count / prefix launches (five for the wide
// sort), each costing more than the sorting at this size.  Same output: the
// records stable by key, spos as the last pass writes it, lord as the first.
// It zeroes the tile's first-digit counts that k_parse accumulated (the walk
// clears the other tables as after a multi-pass sort).
// The one-tile sort of the records whose keys key_in[r] (record r *
// kSortThreads + threadIdx.x) the calling workgroup holds (k_sort_tile loads
// them).
__device__ __forceinline__ void sort_tile_body(const BundleArgs &a, uint32_t key_bits,
                                               const uint32_t key_in[kSortItems]) {
    constexpr int W = kSortThreads / 64;
    __shared__ uint32_t s_key[2][kSortTile];
    __shared__ uint16_t s_idx[2][kSortTile];
    __shared__ uint32_t s_base[256], s_run[256], s_wcnt[W][256];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const uint32_t n = a.n;
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = r * kSortThreads + t;
        if (i < n) {
            s_key[0][i] = key_in[r];
            s_idx[0][i] = (uint16_t)i;
        }
    }
    const int passes = (int)((key_bits + 7u) / 8u);
    for (int q = 0; q < passes; q++) {
        const int cur = q & 1;
        const uint32_t shift = 8u * (uint32_t)q;
        if (t < 256) {
            s_run[t] = 0u;
#pragma unroll
            for (int k = 0; k < W; k++) s_wcnt[k][t] = 0u;
        }
        __syncthreads();
        uint32_t key[kSortItems], loc[kSortItems];
        uint16_t idx[kSortItems];
#pragma unroll
        for (int r = 0; r < kSortItems; r++) {
            const uint32_t i = r * kSortThreads + t;
            key[r] = i < n ? s_key[cur][i] : 0u;
            idx[r] = i < n ? s_idx[cur][i] : (uint16_t)0;
        }
        // stable ranks within each digit, items in index order (k_sort_scatter's);
        // rows past the last record are skipped (block-uniform)
#pragma unroll
        for (int r = 0; r < kSortItems; r++) {
            if (r * kSortThreads >= (int)n) break;
            const bool valid = r * kSortThreads + t < (int)n;
            const uint32_t d = valid ? (key[r] >> shift) & 255u : 0u;
            unsigned long long m = __ballot(valid);
#pragma unroll
            for (int bit = 0; bit < 8; bit++) {
                const unsigned long long b = __ballot((d >> bit) & 1u);
                m &= ((d >> bit) & 1u) ? b : ~b;
            }
            const uint32_t below = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            if (valid && below == 0u) s_wcnt[w][d] = (uint32_t)__popcll(m);
            __syncthreads();
            if (valid) {
                uint32_t pre = s_run[d];
                for (int k = 0; k < w; k++) pre += s_wcnt[k][d];
                loc[r] = pre + below;
            }
            __syncthreads();
            if (t < 256) {
                uint32_t add = 0u;
#pragma unroll
                for (int k = 0; k < W; k++) { add += s_wcnt[k][t]; s_wcnt[k][t] = 0u; }
                s_run[t] += add;
            }
            __syncthreads();
        }
        // digit bases: exclusive scan of the digit totals (4 waves x 64 digits)
        if (t < 256) {
            const uint32_t c = s_run[t];
            uint32_t x = c;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, o);
                if (lane >= o) x += y;
            }
            if (lane == 63) s_wcnt[0][w] = x;
            s_base[t] = x - c;
        }
        __syncthreads();
        if (t < 256) {
            uint32_t off = 0u;
            for (int k = 0; k < w; k++) off += s_wcnt[0][k];
            s_base[t] += off;
        }
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kSortItems; r++) {
            if (r * kSortThreads + t < (int)n) {
                const uint32_t np = s_base[(key[r] >> shift) & 255u] + loc[r];
                s_key[cur ^ 1][np] = key[r];
                s_idx[cur ^ 1][np] = idx[r];
            }
        }
        __syncthreads();
    }
    const int fin = passes & 1;
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t pos = r * kSortThreads + t;
        if (pos < n) {
            const uint32_t key = s_key[fin][pos];
            const WalkRec rec = a.sv_in[s_idx[fin][pos]];
            a.sk_out[pos] = key;
            a.sv_out[pos] = rec;
            if (a.reverse && key <= a.ctx_mask) a.spos[rec.p & kRecIdxMask] = pos;
        }
    }
    if (SRTP_LEN_ORDER) {
        __syncthreads();
        write_lord(n, 1u, 0u, 0u, a.len, a.ctl, a.cls_tile, a.lord, s_base, s_run);
    }
}

__global__ __launch_bounds__(kSortThreads) void k_sort_tile(BundleArgs a, uint32_t key_bits, uint32_t bins) {
    const int t = threadIdx.x;
    for (uint32_t d = (uint32_t)t; d < bins; d += kSortThreads) a.sort_counts[d] = 0u;
    uint32_t key[kSortItems];
#pragma unroll
    for (int r = 0; r < kSortItems; r++) {
        const uint32_t i = r * kSortThreads + t;
        key[r] = i < a.n ? a.sk_in[i] : 0u;
    }
    sort_tile_body(a, key_bits, key);
}

hipError_t launch_sort_tile(const BundleArgs &a, hipStream_t s) {
    const uint32_t key_bits = (uint32_t)a.sort_key_bits;
    const uint32_t bins = 1u << a.sort_bits; // k_parse's first-digit counts
    hipLaunchKernelGGL(k_sort_tile, dim3(1), dim3(kSortThreads), 0, s, a, key_bits, bins);
    return hipGetLastError();
}

// Keys of 17-19 bits: an 8-bit pass (its bases from k_parse's counts, as the
// 8-bit sort's first pass: no prefix launch), then one wide pass of the
// remaining 9-11 bits -- four launches where two wide passes take five.
hipError_t launch_sort_hybrid(const BundleArgs &a, const SortScratch &ss, hipStream_t s) {
    const uint32_t tiles = (a.n + kSortTile - 1) / kSortTile;
    SortPass sp;
    sp.sk = a.sk_in;
    sp.sv = a.sv_in;
    sp.dk = ss.keys_tmp;
    sp.dv = ss.vals_tmp;
    sp.n = a.n;
    sp.shift = 0u;
    sp.tiles = tiles;
    sp.counts = a.sort_counts; // k_parse's; the walk re-zeroes them (sort_zero)
    sp.next_counts = nullptr;
    sp.zero = nullptr;
    sp.spos = nullptr;
    sp.walk_max = a.ctx_mask;
    sp.lord = a.lord;
    sp.len = a.len;
    sp.ctl = a.ctl;
    sp.cls_tile = a.cls_tile;
    hipLaunchKernelGGL(k_sort_scatter, dim3(tiles), dim3(kSortThreads), 0, s, sp);
    const uint32_t bits = (uint32_t)a.sort_hi_bits, B = 1u << bits;
    hipLaunchKernelGGL(k_sort_count_wide, dim3(tiles), dim3(kSortThreads), 0, s, (const uint32_t *)ss.keys_tmp,
                       a.n, 8u, B, ss.wcounts[1]);
    hipLaunchKernelGGL(k_sort_prefix, dim3(B / 64u), dim3(64 * kPrefixGroups), 0, s, ss.wcounts[1], tiles, B,
                       ss.wprefix, ss.wtotal);
    SortPassWide sw;
    sw.sk = ss.keys_tmp;
    sw.sv = ss.vals_tmp;
    sw.dk = a.sk_out;
    sw.dv = a.sv_out;
    sw.n = a.n;
    sw.shift = 8u;
    sw.bits = bits;
    sw.tiles = tiles;
    sw.prefix = ss.wprefix;
    sw.total = ss.wtotal;
    sw.spos = a.reverse ? a.spos : nullptr;
    sw.walk_max = a.ctx_mask;
    sw.lord = nullptr;
    sw.len = a.len;
    sw.ctl = a.ctl;
    sw.cls_tile = a.cls_tile;
    hipLaunchKernelGGL(k_sort_scatter_wide, dim3(tiles), dim3(kSortThreads), 0, s, sw);
    return hipGetLastError();
}

hipError_t launch_sort(const BundleArgs &a, const SortScratch &ss, hipStream_t s) {
    if (a.sort_hi_bits) return launch_sort_hybrid(a, ss, s);
    if (a.sort_bits > 8) return launch_sort_wide(a, ss, s);
    const uint32_t tiles = (a.n + kSortTile - 1) / kSortTile;
    const int P = a.sort_passes;
    for (int q = 0; q < P; q++) {
        SortPass sp;
        // ping-pong: in -> tmp -> (out | in) -> (out | tmp) -> out
        const bool last = q == P - 1;
        sp.sk = q == 0 ? a.sk_in : (q & 1) ? ss.keys_tmp : a.sk_in;
        sp.sv = q == 0 ? a.sv_in : (q & 1) ? ss.vals_tmp : a.sv_in;
        sp.dk = last ? a.sk_out : (q & 1) ? a.sk_in : ss.keys_tmp;
        sp.dv = last ? a.sv_out : (q & 1) ? a.sv_in : ss.vals_tmp;
        sp.n = a.n;
        sp.shift = 8u * (uint32_t)q;
        sp.tiles = tiles;
        sp.counts = ss.counts[q];
        sp.next_counts = nullptr; // k_sort_count below
        // pass q re-zeroes pass q-1's counts (read by all of pass q-1); the last
        // pass's are re-zeroed by the walk (BundleArgs::sort_zero)
        sp.zero = q ? ss.counts[q - 1] : nullptr;
        sp.spos = last && a.reverse ? a.spos : nullptr;
        sp.walk_max = a.ctx_mask;
        sp.lord = q == 0 ? a.lord : nullptr;
        sp.len = a.len;
        sp.ctl = a.ctl;
        sp.cls_tile = a.cls_tile;
        hipLaunchKernelGGL(k_sort_scatter, dim3(tiles), dim3(kSortThreads), 0, s, sp);
        if (!last)
            hipLaunchKernelGGL(k_sort_count, dim3(tiles), dim3(kSortThreads), 0, s, (const uint32_t *)sp.dk,
                               a.n, sp.shift + 8u, ss.counts[q + 1]);
    }
    return hipGetLastError();
}

// Runs body(ks) once per distinct session-key set among this wave's lanes with
// `todo` set; ks is wave-uniform, so round keys, salt and HMAC midstates are
// scalar loads held in SGPRs (one iteration when the wave shares one key set,
// the common case: every context of a factory shares its session keys, Q2).
template <class F>
__device__ __forceinline__ void for_each_keyset(bool todo, uint32_t ks_id, F &&body) {
    while (true) {
        const unsigned long long m = __ballot(todo);
        if (m == 0ull) break;
        const int lane = __ffsll((long long)m) - 1;
        const uint32_t ks_u = (uint32_t)__builtin_amdgcn_readlane((int)ks_id, lane);
        if (todo && ks_id == ks_u) {
            body(ks_u);
            todo = false;
        }
    }
}

// True when the wave's lanes with `todo` set hold more than one key set.
__device__ __forceinline__ bool wave_mixes_keysets(bool todo, uint32_t ks_id) {
    const unsigned long long m = __ballot(todo);
    if (m == 0ull) return false;
    const uint32_t first = (uint32_t)__builtin_amdgcn_readlane((int)ks_id, __ffsll((long long)m) - 1);
    return __ballot(todo && ks_id != first) != 0ull;
}

__device__ __forceinline__ uint32_t sgpr(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}

// Round keys of a wave-uniform key set into SGPRs (a vector load of one line,
// then v_readfirstlane: the kernel also stores to global memory, so the
// compiler would not use the scalar cache for them).
__device__ __forceinline__ void load_round_keys_uniform(const KeySet *__restrict__ ks,
                                                        RoundKeys &rk) {
    const uint4 *p = reinterpret_cast<const uint4 *>(ks->rk);
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const uint4 v = p[i];
        rk.k[4 * i] = sgpr(v.x); rk.k[4 * i + 1] = sgpr(v.y);
        rk.k[4 * i + 2] = sgpr(v.z); rk.k[4 * i + 3] = sgpr(v.w);
    }
}

template <bool LK>
__device__ __forceinline__ void pk_load(const KeySet *__restrict__ ks, PktKeys<LK> &pk);
template <>
__device__ __forceinline__ void pk_load<false>(const KeySet *__restrict__ ks, PktKeys<false> &pk) {
    load_round_keys_uniform(ks, pk.rk);
}
template <>
__device__ __forceinline__ void pk_load<true>(const KeySet *__restrict__ ks, PktKeys<true> &pk) {
    const uint4 *q = reinterpret_cast<const uint4 *>(ks->rk);
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const uint4 v = q[i];
        pk.r[4 * i] = v.x; pk.r[4 * i + 1] = v.y; pk.r[4 * i + 2] = v.z; pk.r[4 * i + 3] = v.w;
    }
}
// A key-set field: wave-uniform (SGPR) or the lane's own.
template <bool LK> __device__ __forceinline__ uint32_t kf(uint32_t x) { return LK ? x : sgpr(x); }

// Re-check one SRTP tag under another ROC from the verify pass's midstate
// (only the block(s) carrying the ROC are re-hashed).
struct ReverifyArgs { // by value: keeps the kernel arguments out of scratch
    const uint8_t *pkt;
    const uint32_t *mid;   // 5 words
    const uint32_t *tailc; // 16 words, or null when the packet still holds ciphertext
};

__device__ __forceinline__ bool reverify_rtp(ReverifyArgs r, const KeySet *ks, int L, int32_t g) {
    const int T = ks->tag_len;
    int mac_len = L - T;
    if (mac_len < 0) mac_len = 0;
    const uint8_t *pkt = r.pkt;
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = r.mid[k];
    const int nb_full = mac_len >> 6;
    const int nb_inner = ((mac_len + 12) >> 6) + 1;
    for (int b = nb_full; b <= nb_inner; b++) {
        uint32_t w[16];
        const uint4 *src = (r.tailc && b == nb_full) // packet holds plaintext: saved ciphertext
                               ? reinterpret_cast<const uint4 *>(r.tailc)
                               : reinterpret_cast<const uint4 *>(pkt + 64 * b);
#pragma unroll
        for (int m = 0; m < 4; m++) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (64 * b + 16 * m < mac_len) v = src[m];
            w[4 * m] = v.x; w[4 * m + 1] = v.y; w[4 * m + 2] = v.z; w[4 * m + 3] = v.w;
        }
        if (b < nb_inner) {
            inner_words(w, b, mac_len, (uint32_t)g);
        } else {
            outer_words<false>(w, h, ks); // ks varies across the walk's lanes
        }
        sha1_compress(h, w);
    }
    return tag_matches(h, pkt + mac_len, T);
}

// ============================================================== Skein-512 MAC
// SRTPPolicy.SKEIN_AUTHENTICATION (ZRTP "SK32"/"SK64"): bccontrib's SkeinMac,
// keyed with the session auth key and an output of tag_len * 8 bits
// (SRTPCryptoContext.java:421-428, SRTCPCryptoContext.java:185-192), fed the
// same bytes as authenticatePacketHMAC (BaseSRTPCryptoContext.java:269-278):
// the packet, then the ROC (SRTP) or the E|index word (SRTCP) big-endian.
// Skein 1.3: each 64-B message block is one Threefish-512 encryption keyed
// with the chaining value (UBI); the key and config blocks are folded into
// SkeinKeys.g0 on the host.  Threefish is 64-bit add / rotate / xor, so it
// runs on the VALU (two 32-bit ops each), one packet per lane.
constexpr uint64_t kSkeinParity = 0x1BD11BDAA9FC1A22ull;
constexpr uint64_t kSkeinMsg = 48ull << 56, kSkeinOut = 63ull << 56;
constexpr uint64_t kSkeinFirst = 1ull << 62, kSkeinFinal = 1ull << 63;

__device__ __forceinline__ constexpr int skein_rot(int d, int j) {
    // Skein 1.3 Table 4: Threefish-512 rotation constants R(d mod 8, j)
    constexpr int R[8][4] = {{46, 36, 19, 37}, {33, 27, 14, 42}, {17, 49, 36, 39}, {44, 9, 54, 56},
                             {39, 30, 34, 24}, {13, 50, 10, 17}, {25, 29, 39, 43}, {8, 35, 56, 22}};
    return R[d & 7][j];
}

template <int N>
__device__ __forceinline__ uint64_t rotl64(uint64_t x) {
    return (x << N) | (x >> (64 - N));
}

// Four rounds d0..d0+3 (MIX on word pairs, then the permutation {2,1,4,7,6,5,0,3}).
template <int D0>
__device__ __forceinline__ void threefish_rounds4(uint64_t v[8]) {
#define SK_MIX(d)                                                                  \
    v[0] += v[1]; v[1] = rotl64<skein_rot(d, 0)>(v[1]) ^ v[0];                     \
    v[2] += v[3]; v[3] = rotl64<skein_rot(d, 1)>(v[3]) ^ v[2];                     \
    v[4] += v[5]; v[5] = rotl64<skein_rot(d, 2)>(v[5]) ^ v[4];                     \
    v[6] += v[7]; v[7] = rotl64<skein_rot(d, 3)>(v[7]) ^ v[6];                     \
    { const uint64_t w0 = v[0], w3 = v[3];                                         \
      v[0] = v[2]; v[2] = v[4]; v[4] = v[6]; v[6] = w0; v[3] = v[7]; v[7] = w3; }
    SK_MIX(D0) SK_MIX(D0 + 1) SK_MIX(D0 + 2) SK_MIX(D0 + 3)
#undef SK_MIX
}

template <int S>
__device__ __forceinline__ void threefish_subkey(uint64_t v[8], const uint64_t k[9], const uint64_t t[3]) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] += k[(S + i) % 9];
    v[5] += t[S % 3];
    v[6] += t[(S + 1) % 3];
    v[7] += (uint64_t)S;
}

template <int S>
__device__ __forceinline__ void threefish_from(uint64_t v[8], const uint64_t k[9], const uint64_t t[3]) {
    if constexpr (S < 18) {
        threefish_subkey<S>(v, k, t);
        threefish_rounds4<4 * S>(v);
        threefish_from<S + 1>(v, k, t);
    } else {
        threefish_subkey<18>(v, k, t);
    }
}

// One UBI step: h = Threefish-512(key h, tweak {t0, t1}, m) ^ m (72 rounds).
__device__ __forceinline__ void skein_ubi_block(uint64_t h[8], const uint64_t m[8], uint64_t t0, uint64_t t1) {
    uint64_t k[9], v[8];
    const uint64_t t[3] = {t0, t1, t0 ^ t1};
    k[8] = kSkeinParity;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        k[i] = h[i];
        k[8] ^= h[i];
        v[i] = m[i];
    }
    threefish_from<0>(v, k, t);
#pragma unroll
    for (int i = 0; i < 8; i++) h[i] = v[i] ^ m[i];
}

// Message block b of pkt[0, L) || suffix (4 bytes big-endian), zero-padded,
// as Skein's little-endian 64-bit words.  Reads 16-B units below L only (the
// packet region is 16-B aligned and padded, so a unit may run past L).
__device__ __forceinline__ void skein_msg_block(const uint8_t *pkt, int b, int L, uint32_t suffix_le,
                                                uint64_t m[8]) {
    const uint4 *qp = reinterpret_cast<const uint4 *>(pkt + 64 * b);
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (64 * b + 16 * q < L) v = qp[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int wp = 64 * b + 4 * k; // stream position of the word's byte 0
        const int rem = L - wp;        // packet bytes in this word
        uint32_t d = w[k] & (rem >= 4 ? ~0u : (rem <= 0 ? 0u : (1u << (8 * rem)) - 1u));
        const int o = wp - L;          // suffix byte i sits at stream position L + i
        if (o > -4 && o < 4) d |= o >= 0 ? (suffix_le >> (8 * o)) : (suffix_le << (8 * -o));
        w[k] = d;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// Skein-MAC of pkt[0, L) || suffix under the key set's g0; returns the first
// 12 output bytes as big-endian words (the layout tag_matches / tag_write use).
// UNIFORM: g0 is the wave's key set (scalar registers); else per lane.
template <bool UNIFORM>
__device__ __forceinline__ void skein_mac(const SkeinKeys *sk, const uint8_t *pkt, int L, uint32_t suffix,
                                          uint32_t tag[5]) {
    uint64_t h[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint64_t g = sk->g0[i];
        h[i] = UNIFORM ? ((uint64_t)sgpr((uint32_t)(g >> 32)) << 32) | sgpr((uint32_t)g) : g;
    }
    const int n = L + 4;
    const int nb = (n + 63) >> 6;
    const uint32_t sle = bswap(suffix);
    // nb message blocks, then Output(G, No) = UBI(G, ToBytes(0, 8), Tout) --
    // one block for No <= 512 -- through the same Threefish code
    for (int b = 0; b <= nb; b++) {
        uint64_t m[8];
        uint64_t t0, t1;
        if (b < nb) {
            skein_msg_block(pkt, b, L, sle, m);
            t0 = (uint64_t)min(64 * (b + 1), n);
            t1 = kSkeinMsg | (b == 0 ? kSkeinFirst : 0ull) | (b == nb - 1 ? kSkeinFinal : 0ull);
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) m[i] = 0ull;
            t0 = 8;
            t1 = kSkeinOut | kSkeinFirst | kSkeinFinal;
        }
        skein_ubi_block(h, m, t0, t1);
    }
    tag[0] = bswap((uint32_t)h[0]);
    tag[1] = bswap((uint32_t)(h[0] >> 32));
    tag[2] = bswap((uint32_t)h[1]);
    tag[3] = tag[4] = 0u;
}

// The walk's re-check of a Skein-tagged SRTP packet under another ROC: the
// whole MAC again (Skein packets are not deciphered before the walk, so the
// packet still holds its ciphertext).  Only the walk instances launched for
// engines with Skein key sets contain it.
__device__ __forceinline__ bool skein_reverify(const SkeinKeys *sk, const uint8_t *pkt, int L, int T, uint32_t roc) {
    int mac_len = L - T;
    if (mac_len < 0) mac_len = 0;
    uint32_t tag[5];
    skein_mac<false>(sk, pkt, mac_len, roc, tag);
    return tag_matches(tag, pkt + mac_len, T);
}

// The walk's tag re-check under ROC g, by the key set's MAC (SK: the engine
// has Skein key sets).
template <bool SK>
__device__ __forceinline__ bool reverify_tag(const BundleArgs &a, ReverifyArgs rv, const KeySet *ks, int L,
                                             int32_t g) {
    if (SK && ks->auth_type == SRTP_SKEIN_AUTHENTICATION)
        return skein_reverify(a.skkeys + (ks - a.keysets), rv.pkt, L, ks->tag_len, (uint32_t)g);
    return reverify_rtp(rv, ks, L, g);
}

// ============================================================== k_walk
// One lane per context: the serial state machine over the context's packets in
// array order (records sorted by context slot, stable).
struct WalkCtx {
    int enc, auth, T, kind;
    bool check_replay, reverse;
};

// Processes one packet; returns false when the rest of the context's packets
// are aborted (a throw with abort_on_error).
template <bool SK>
__device__ __forceinline__ bool walk_one(const BundleArgs &a, const KeySet *ks, const WalkCtx &c,
                                         CtxState &st, const WalkRec &rec, uint32_t g0,
                                         uint32_t auth_ok, bool dry, int32_t tid) {
    const uint32_t p = rec.p & kRecIdxMask;
    const int L = (int)(rec.lc & 0xffffu), C = (int)(rec.lc >> 16);
    const int T = c.T;
    bool threw = false;
    if (c.kind == SRTP_KIND_RTP) {
        const int seq = (int)rec.word;
        if (!c.reverse) {
            const int Tt = (c.auth != SRTP_NULL_AUTHENTICATION) ? T : 0;
            if (L + Tt > C) { a.w_status[p] = SRTP_STATUS_ERR_CAPACITY; return true; }
        }
        if (!(st.flags & 1u)) { st.flags |= 1u; st.b = seq; } // seqNumSet (:587-591, :662-666)
        // guessIndex :457-475
        int32_t g;
        if (st.b < 32768) g = (seq - st.b > 32768) ? (int32_t)((uint32_t)st.a - 1u) : st.a;
        else g = (st.b - 32768 > seq) ? (int32_t)((uint32_t)st.a + 1u) : st.a;
        st.g = g;
        const int64_t gi = java_lshl((int64_t)g, 16) | seq;
        const int64_t local = java_lshl((int64_t)st.a, 16) | st.b;
        const int64_t delta = gi - local;
        // checkReplay :279-323
        if (c.check_replay && delta <= 0) {
            if (-delta > 64 || (((uint64_t)st.window >> ((-delta) & 63)) & 1u)) {
                a.w_status[p] = SRTP_STATUS_DROP_REPLAY;
                return true;
            }
        }
        int newL = L;
        if (c.reverse) {
            if (c.auth != SRTP_NULL_AUTHENTICATION) {
                newL = L - T > 0 ? L - T : 0;
                a.w_len[p] = (uint32_t)newL;
                bool ok;
                if ((uint32_t)g == g0) {
                    ok = (auth_ok & 1u) != 0;
                } else if ((auth_ok & 4u) && (uint32_t)g == g0 - 1u) {
                    ok = (auth_ok & 2u) != 0; // checked by the verify pass too
                } else {
                    ReverifyArgs rv;
                    rv.pkt = a.seg + a.off[p];
                    rv.mid = a.mid + 5 * (size_t)p;
                    rv.tailc = (a.spec[p] & kSpecDid) ? a.tailc + 16 * (size_t)p : nullptr;
                    ok = reverify_tag<SK>(a, rv, ks, L, g);
                    atomicAdd(&a.counters[kCtrRocRecheck], 1ull);
                }
                if (!ok) { a.w_status[p] = SRTP_STATUS_DROP_AUTH; return true; }
            }
            if (!(rec.p & kRecSkipDec)) threw = enc_would_throw(c.enc, rec.h, newL - rec.h);
        } else {
            threw = enc_would_throw(c.enc, rec.h, L - rec.h);
            if (!threw && c.auth != SRTP_NULL_AUTHENTICATION) newL = L + T;
        }
        if (!threw) {
            a.w_cw[p] = (uint32_t)g;
            a.w_len[p] = (uint32_t)newL;
            // update :719-744
            if (delta > 0) st.window = (uint64_t)java_lshl((int64_t)st.window, delta) | 1ull;
            else st.window |= (uint64_t)(int64_t)java_ishl1((int32_t)(-delta));
            if (g == st.a) {
                if (seq > st.b) st.b = seq & 0xffff;
            } else if (g == (int32_t)((uint32_t)st.a + 1u)) {
                st.b = seq & 0xffff;
                st.a = g;
            }
        }
    } else if (!c.reverse) {
        // SRTCPCryptoContext.transformPacket :391-427
        const int trailer = (c.auth != SRTP_NULL_AUTHENTICATION) ? 4 + T : 0;
        if (L + trailer > C) { a.w_status[p] = SRTP_STATUS_ERR_CAPACITY; return true; }
        a.w_cw[p] = (uint32_t)st.a;
        a.w_len[p] = (uint32_t)(L + trailer);
        st.a = (int32_t)(((uint32_t)st.a + 1u) & 0x7FFFFFFFu);
    } else {
        // SRTCPCryptoContext.reverseTransformPacket :315-374
        const int io = L - 4 - T;
        if (io < 0) {
            threw = true;
        } else {
            uint32_t word = rec.word;
            if (rec.h != T) word = ld_be32(a.seg + a.off[p] + io);
            const int32_t index = (int32_t)(word & 0x7FFFFFFFu);
            const bool decrypt = (word & 0x80000000u) != 0;
            const int64_t delta = (int64_t)(int32_t)((uint32_t)index - (uint32_t)st.b);
            // SRTCP checkReplay (:106-120) is not config-gated
            if (delta <= 0 && (-delta > 64 || (((uint64_t)st.window >> ((-delta) & 63)) & 1u))) {
                a.w_status[p] = SRTP_STATUS_DROP_REPLAY;
                return true;
            }
            int newL = L;
            if (c.auth != SRTP_NULL_AUTHENTICATION) {
                newL = L - T - 4 > 0 ? L - T - 4 : 0;
                a.w_len[p] = (uint32_t)newL;
                if (!(auth_ok & 1u)) { a.w_status[p] = SRTP_STATUS_DROP_AUTH; return true; }
            }
            if (decrypt && (c.enc == SRTP_AESCM_ENCRYPTION || c.enc == SRTP_TWOFISH_ENCRYPTION) &&
                newL - 8 < 0)
                threw = true;
            if (!threw) {
                a.w_cw[p] = word;
                // update :435-451 (reversed delta)
                const int32_t d2 = (int32_t)((uint32_t)st.b - (uint32_t)index);
                if (d2 > 0) st.window = (uint64_t)java_lshl((int64_t)st.window, d2) | 1ull;
                else st.window |= (uint64_t)(int64_t)java_ishl1(d2);
                st.b = index;
            }
        }
    }
    if (threw) {
        a.w_status[p] = SRTP_STATUS_ERR_MALFORMED;
        if (a.abort_on_error) {
            if (dry) atomicMin(&a.e_min[tid], (int32_t)p);
            return false; // the rest of this transformer's array is aborted
        }
        return true;
    }
    a.w_status[p] = SRTP_STATUS_OK;
    return true;
}

// ----------------------------------------------------- wave-parallel walk
// The rest of a long chain (see chain_part below), from the record where the
// tiles' speculation broke, is walked by a whole wave, 256 records per step,
// by speculating that every packet is the context's new highest index -- the
// steady state of an in-order stream.  Under that assumption each packet's
// guessed ROC (guessIndex, SRTPCryptoContext.java:457-475) depends only on
// the previous packet's sequence number: roc_k = roc + sum of the wrap steps
// d_j in {-1, 0, +1} of the packets before it, a prefix sum.  A packet keeps
// the speculation when it is that new maximum (delta > 0: checkReplay
// accepts, update :719-744 makes it s_l, and with d = +1 the new ROC), it
// authenticates under its ROC (unprotect: the verify pass's result when its
// guess was the same, else the midstate re-check), fits its capacity and does
// not throw.  Every packet before the first one that breaks it is committed
// in parallel; the replay window after them is the old window shifted by the
// Java-masked distances (delta & 63, :730) of all of them, OR one bit per
// packet at the masked distance of the packets after it (suffix sums).  The
// breaking packet goes through walk_one, exactly as the serial walk, and the
// speculation resumes after it.  SRTCP chains are walked serially.
#ifndef SRTP_LONG_PER
#define SRTP_LONG_PER 4
#endif
constexpr int kLongPer = SRTP_LONG_PER;          // records per lane per step
constexpr int kLongStep = 64 * kLongPer;         // records per wave step

__device__ __forceinline__ int32_t wave_excl_scan(int32_t x) {
    const int lane = (int)(threadIdx.x & 63u);
    int32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    return inc - x;
}

__device__ __forceinline__ uint64_t wave_or64(uint64_t x) {
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o, 64);
        hi |= (uint32_t)__shfl_xor((int)hi, o, 64);
    }
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void bcast_state(CtxState &st) {
    st.a = __builtin_amdgcn_readfirstlane(st.a);
    st.b = __builtin_amdgcn_readfirstlane(st.b);
    st.g = __builtin_amdgcn_readfirstlane(st.g);
    st.flags = (uint32_t)__builtin_amdgcn_readfirstlane((int)st.flags);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)st.window);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(st.window >> 32));
    st.window = ((uint64_t)hi << 32) | lo;
}

// The walk is one wave (k_walk's workgroup; k_small's wave 0): a barrier
// between its LDS phases only has to order the wave's own memory operations
// (what __syncthreads does, without s_barrier, so that k_small's other waves
// need not take part).
__device__ __forceinline__ void walk_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// LDS of the second k_walk pass when it walks long chains (the first pass's
// staging arrays, unused then): one step's records and per-record results.
struct LongLds {
    WalkRec *rec;     // [kLongStep] the step's records, block order
    uint32_t *roc;    // [kLongStep] guessed ROC under the speculation
    uint32_t *g0;     // [kLongStep] unprotect: the verify pass's ROC
    uint32_t *ok;     // [kLongStep] unprotect: the verify pass's auth bits
    uint32_t *info;   // [kLongStep] bit 0: keeps the speculation; bits 1..: delta & 63
};
// A window already staged in LDS (k_walk's first pass): records [base, base +
// win) of the sorted arrays, read in place instead of staged again.
struct LongWin {
    const WalkRec *rec;
    const uint32_t *key, *g0, *ok;
    uint32_t base, win;
};

template <bool REV, bool SK>
__device__ __forceinline__ void walk_long(const BundleArgs &a, uint32_t i0, const LongLds &sm, const CtxState &st_in,
                                          const LongWin *pw = nullptr) {
    const int lane = (int)(threadIdx.x & 63u);
    const uint32_t key = pw ? pw->key[i0 - pw->base] : a.sk_out[i0];
    const uint32_t slot = key;
    CtxState st = st_in;
    const KeySet *ks = a.keysets + st.ks;
    WalkCtx c;
    c.enc = ks->enc_type; c.auth = ks->auth_type; c.T = ks->tag_len; c.kind = ks->kind;
    c.check_replay = a.check_replay != 0;
    c.reverse = REV;
    const int32_t tid = (int32_t)(a.ctx_keys[slot] >> 32);
    const bool mac = c.auth != SRTP_NULL_AUTHENTICATION;
    uint32_t i = i0;
    uint32_t walked = 0u;
    for (;;) {
        const WalkRec *R = sm.rec;     // the step's records, block order
        const uint32_t *G0 = sm.g0, *OK = sm.ok;
        int nvalid;
        if (pw) { // already staged: the records sit in the window at i - pw->base
            const uint32_t jb = i - pw->base;
            int nv = 0;
#pragma unroll
            for (int k = 0; k < kLongPer; k++) {
                const uint32_t t = jb + (uint32_t)(lane + 64 * k);
                nv += (t < pw->win && pw->key[t] == key) ? 1 : 0;
            }
            nvalid = (int)__reduce_add_sync(~0ull, (unsigned)nv);
            R = pw->rec + jb; G0 = pw->g0 + jb; OK = pw->ok + jb;
        } else {
            // stage the step's records (coalesced), count the chain's
            int nv = 0;
#pragma unroll
            for (int k = 0; k < kLongPer; k++) {
                const int j = lane + 64 * k;
                const uint32_t idx = i + (uint32_t)j;
                const bool v = idx < a.n && a.sk_out[idx] == key;
                uint4 r = make_uint4(0u, 0u, 0u, 0u); // the WalkRec as one 16-B word
                if (v) r = reinterpret_cast<const uint4 *>(a.sv_out)[idx];
                reinterpret_cast<uint4 *>(sm.rec)[j] = r;
                if (REV) {
                    const uint32_t p = r.x & kRecIdxMask;
                    const uint2 go = v ? gok_of(a, p) : make_uint2(0u, 0u);
                    sm.g0[j] = go.x;
                    sm.ok[j] = go.y;
                }
                nv += v ? 1 : 0;
            }
            nvalid = (int)__reduce_add_sync(~0ull, (unsigned)nv); // a prefix of the step
            walk_sync();
        }
        if (nvalid == 0) break;
        int f = 0; // block position of the first packet that breaks the speculation
        if (c.kind == SRTP_KIND_RTP && (st.flags & 1u)) {
            // lane l owns block positions [4l, 4l + 4): wrap steps, their sum
            const int p0 = lane * kLongPer;
            int32_t lsum = 0;
#pragma unroll 1
            for (int r = 0; r < kLongPer; r++) {
                const int pos = p0 + r;
                if (pos >= nvalid) break;
                const int32_t seq = (int32_t)(R[pos].word & 0xffffu);
                const int32_t sl = pos ? (int32_t)(R[pos - 1].word & 0xffffu) : st.b;
                int32_t d;
                if (sl < 32768) d = (seq - sl > 32768) ? -1 : 0;
                else d = (sl - 32768 > seq) ? 1 : 0;
                lsum += d;
            }
            uint32_t roc = (uint32_t)st.a + (uint32_t)wave_excl_scan(lsum); // ROC before the lane
            int first_bad = kLongPer;
#pragma unroll 1
            for (int r = 0; r < kLongPer; r++) {
                const int pos = p0 + r;
                if (pos >= nvalid) { first_bad = min(first_bad, r); break; }
                const WalkRec rec = R[pos];
                const int32_t seq = (int32_t)(rec.word & 0xffffu);
                const int32_t sl = pos ? (int32_t)(R[pos - 1].word & 0xffffu) : st.b;
                const uint32_t roc_prev = roc;
                int32_t d;
                if (sl < 32768) d = (seq - sl > 32768) ? -1 : 0;
                else d = (sl - 32768 > seq) ? 1 : 0;
                roc += (uint32_t)d;
                const int64_t delta = (java_lshl((int64_t)(int32_t)roc, 16) | (int64_t)seq) -
                                      (java_lshl((int64_t)(int32_t)roc_prev, 16) | (int64_t)sl);
                const int L = (int)(rec.lc & 0xffffu), C = (int)(rec.lc >> 16);
                bool g = delta > 0;
                if (REV) {
                    const int newL = mac ? (L - c.T > 0 ? L - c.T : 0) : L;
                    if (!(rec.p & kRecSkipDec)) g = g && !enc_would_throw(c.enc, rec.h, newL - rec.h);
                    if (g && mac) { // the tag under this ROC
                        const uint32_t g0 = G0[pos], okb = OK[pos];
                        if (roc == g0) {
                            g = (okb & 1u) != 0u;
                        } else if ((okb & 4u) && roc == g0 - 1u) {
                            g = (okb & 2u) != 0u;
                        } else {
                            const uint32_t p = rec.p & kRecIdxMask;
                            ReverifyArgs rv;
                            rv.pkt = a.seg + a.off[p];
                            rv.mid = a.mid + 5 * (size_t)p;
                            rv.tailc = (a.spec[p] & kSpecDid) ? a.tailc + 16 * (size_t)p : nullptr;
                            g = reverify_tag<SK>(a, rv, ks, L, (int32_t)roc);
                        }
                    }
                } else {
                    g = g && L + (mac ? c.T : 0) <= C && !enc_would_throw(c.enc, rec.h, L - rec.h);
                }
                sm.roc[pos] = roc;
                sm.info[pos] = (g ? 1u : 0u) | ((uint32_t)((uint64_t)delta & 63u) << 1);
                if (!g) { first_bad = r; break; }
            }
            const unsigned long long bad_lanes = __ballot(first_bad < kLongPer);
            f = nvalid;
            if (bad_lanes) {
                const int bl = __ffsll((long long)bad_lanes) - 1;
                f = min(f, bl * kLongPer + __builtin_amdgcn_readlane(first_bad, bl));
            }
            // commit block positions [0, f)
            int32_t dsum = 0;
            uint32_t recheck = 0u;
#pragma unroll 1
            for (int r = 0; r < kLongPer; r++) {
                const int pos = p0 + r;
                if (pos >= f) break;
                const WalkRec rec = R[pos];
                const uint32_t p = rec.p & kRecIdxMask;
                const int L = (int)(rec.lc & 0xffffu);
                const uint32_t rr = sm.roc[pos];
                a.w_cw[p] = rr;
                a.w_len[p] = (uint32_t)(REV ? (mac ? (L - c.T > 0 ? L - c.T : 0) : L) : L + (mac ? c.T : 0));
                a.w_status[p] = SRTP_STATUS_OK;
                if (REV && mac) {
                    const uint32_t g0 = G0[pos], okb = OK[pos];
                    if (rr != g0 && !((okb & 4u) && rr == g0 - 1u)) recheck++;
                }
                dsum += (int32_t)(sm.info[pos] >> 1);
            }
            if (f > 0) {
                // masked shift distances after each committed packet (suffix sums)
                const int32_t total = (int32_t)__reduce_add_sync(~0ull, (unsigned)dsum);
                int32_t after = total - wave_excl_scan(dsum);
                uint64_t bits = 0ull;
#pragma unroll 1
                for (int r = 0; r < kLongPer; r++) {
                    const int pos = p0 + r;
                    if (pos >= f) break;
                    after -= (int32_t)(sm.info[pos] >> 1);
                    if (after < 64) bits |= 1ull << after;
                }
                bits = wave_or64(bits);
                st.window = (total < 64 ? st.window << total : 0ull) | bits;
                st.a = (int32_t)sm.roc[f - 1];
                st.b = (int32_t)(R[f - 1].word & 0xffffu);
                st.g = st.a;
                const uint32_t rc = (uint32_t)__reduce_add_sync(~0ull, recheck);
                if (lane == 0 && rc) atomicAdd(&a.counters[kCtrRocRecheck], (unsigned long long)rc);
            }
        }
        walked += (uint32_t)(f < nvalid ? (c.kind == SRTP_KIND_RTP ? 1 : nvalid - f) : 0);
        if (f < nvalid) { // the breaking packet (or every SRTCP packet): exactly as the serial walk
            const int stop = c.kind == SRTP_KIND_RTP ? f + 1 : nvalid;
            if (lane == 0) {
                for (int k = f; k < stop; k++) {
                    const WalkRec r = R[k];
                    uint32_t g0 = 0u, ok = 0u;
                    if (REV) { g0 = G0[k]; ok = OK[k]; }
                    (void)walk_one<SK>(a, ks, c, st, r, g0, ok, false, tid);
                }
            }
            bcast_state(st);
            i += (uint32_t)stop;
        } else {
            i += (uint32_t)nvalid;
        }
        walk_sync(); // the step's LDS is reused by the next
        if (nvalid < kLongStep && f >= nvalid) break;
    }
    if (lane == 0) {
        a.ctx[slot] = st;
        atomicAdd(&a.counters[kCtrLongWalked], (unsigned long long)walked);
    }
}

// k_walk's geometry (see k_walk): one wave per workgroup, a span of kWalkSpan
// sorted records ("tile") plus a look-ahead of kWalkAhead staged in LDS.
constexpr int kWalkBlock = 64;
#ifndef SRTP_WALK_PER
#define SRTP_WALK_PER 4
#endif
constexpr int kWalkPer = SRTP_WALK_PER; // records per lane of a span
constexpr int kWalkSpan = kWalkBlock * kWalkPer;
constexpr int kWalkAhead = 256;
constexpr int kWalkWin = kWalkSpan + kWalkAhead;
// A chain of kMedMin records or more (and shorter than kLongMin) is walked by
// the whole wave (walk_long) after the lanes' one-lane walks: a lane pays a
// few hundred cycles per record, the wave's speculation a few per record.
#ifndef SRTP_MED_MIN
#define SRTP_MED_MIN 32
#endif
constexpr uint32_t kMedMin = SRTP_MED_MIN;
constexpr int kMedMax = kWalkSpan / SRTP_MED_MIN + 1; // chains of kMedMin+ starting in a span
static_assert(kMedMax <= 64, "one medium chain start per lane");

// ------------------------------------------------ chains across walk tiles
// A context chain of kWalkSpan or more records (a heavy SSRC in a skewed
// bundle, or one stream carrying the whole bundle) is walked by every first-
// pass tile it crosses at once, under walk_long's speculation.  Each tile
// evaluates its part of the chain locally: the wrap steps d from consecutive
// sequence numbers (guessIndex :457-475 with s_l = the previous packet),
// delta = d * 2^16 + seq - prev (no ROC in it), the window shifts delta & 63
// (update :719-744), and the checks that keep the speculation (a new highest
// index, no throw, the capacity, the verify pass's tag result under a ROC that
// must equal g0 - (the d's so far), one ROC "x" the part must start from).
// A part's effect on the state (ROC steps, window shift and bits, last s_l)
// composes with its neighbours' like a scan operator.  Tiles take their
// indices from a ticket counter, publish the effect of the part that runs on
// into the next tile -- first as an aggregate, then as the exact state after
// it -- and look back over the tiles before them for the state their part
// starts from (decoupled look-back, 64 tiles per step, one per lane).  Then a
// tile commits its records up to the first that breaks the speculation; the
// chain's first break hands the rest of the chain, from that record on, to
// the second pass's walk_long (exactly as the serial walk), and the tiles
// after it commit nothing.  Published words are 8-byte {value, bundle epoch}
// granules written and read with agent-scope atomics: each is valid on its
// own, so neither side needs a fence.
constexpr int kChainPer = kWalkSpan / kWalkBlock;  // records per lane of a part (4)
static_assert(kLongMin == (uint32_t)kWalkSpan, "a long chain reaches the end of the tile it starts in");

struct ChainAgg {
    int32_t dsum;     // ROC steps
    uint32_t x;       // ROC the part must start from (hasx)
    uint32_t tshift;  // window shift, capped at 64
    uint64_t bits;    // window bits set by the part's packets
    int32_t s_l;      // sequence number of the last packet
    bool hasx, broken;
};
struct ChainState {
    uint32_t roc;
    int32_t s_l;
    uint64_t window;
    bool broken;      // the speculation broke before (the rest is walk_long's)
    bool stalled = false; // the look-back gave up: the part is left to the stall fix-up
};

__device__ __forceinline__ ChainState chain_apply(ChainState p, const ChainAgg &g) {
    if (p.broken || g.broken || (g.hasx && p.roc != g.x) ||
        (int64_t)(int32_t)p.roc + g.dsum > (int64_t)0x7fffffff) {
        p.broken = true;
        return p;
    }
    p.roc += (uint32_t)g.dsum;
    p.s_l = g.s_l;
    p.window = (g.tshift < 64u ? p.window << g.tshift : 0ull) | g.bits;
    return p;
}

// g1, then g2
__device__ __forceinline__ ChainAgg chain_compose(const ChainAgg &g1, const ChainAgg &g2) {
    ChainAgg o;
    o.broken = g1.broken || g2.broken ||
               (g1.hasx && g2.hasx && g2.x - (uint32_t)g1.dsum != g1.x);
    o.dsum = g1.dsum + g2.dsum;
    o.hasx = g1.hasx || g2.hasx;
    o.x = g1.hasx ? g1.x : g2.x - (uint32_t)g1.dsum;
    o.tshift = min(g1.tshift + g2.tshift, 64u);
    o.bits = (g2.tshift < 64u ? g1.bits << g2.tshift : 0ull) | g2.bits;
    o.s_l = g2.s_l;
    return o;
}

constexpr int kLinkWords = 10; // per tile: [0, 5) aggregate, [5, 9) state
__device__ __forceinline__ void gran_put(uint64_t *p, uint32_t epoch, uint32_t v) {
    __hip_atomic_store(p, ((uint64_t)v << 32) | epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool gran_get(const uint64_t *p, uint32_t epoch, uint32_t &v) {
    const uint64_t g = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v = (uint32_t)(g >> 32);
    return (uint32_t)g == epoch;
}

// Lanes 0..4 (aggregate) or 0..3 (state) store one granule each.
__device__ __forceinline__ void chain_publish_agg(const BundleArgs &a, uint32_t tile, uint32_t epoch,
                                                  const ChainAgg &g) {
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t v = (uint32_t)g.dsum;
    if (lane == 1) v = g.x;
    if (lane == 2) v = g.tshift | (g.hasx ? 0x80u : 0u) | (g.broken ? 0x100u : 0u) | ((uint32_t)g.s_l << 16);
    if (lane == 3) v = (uint32_t)g.bits;
    if (lane == 4) v = (uint32_t)(g.bits >> 32);
    if (lane < 5) gran_put(a.tile_link + (size_t)tile * kLinkWords + lane, epoch, v);
}
__device__ __forceinline__ void chain_publish_state(const BundleArgs &a, uint32_t tile, uint32_t epoch,
                                                    const ChainState &s) {
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t v = s.roc;
    if (lane == 1) v = ((uint32_t)s.s_l & 0xffffu) | (s.broken ? 0x10000u : 0u);
    if (lane == 2) v = (uint32_t)s.window;
    if (lane == 3) v = (uint32_t)(s.window >> 32);
    if (lane < 4) gran_put(a.tile_link + (size_t)tile * kLinkWords + 5 + lane, epoch, v);
}

// The exact state before tile `tile`'s first record, for a chain that runs
// into it from the tiles before (each of them published its part).
__device__ __forceinline__ ChainState chain_lookback(const BundleArgs &a, uint32_t tile, uint32_t epoch) {
    const int lane = (int)(threadIdx.x & 63u);
    ChainAgg acc = {};     // the composed parts of the tiles after the current window
    bool have_acc = false;
    if ((a.dbg & kDbgForceStall) && tile % 3u == 1u) { // test hook: give up at once
        if (lane == 0) atomicAdd(&a.counters[kCtrChainStall], 1ull);
        ChainState bad = {};
        bad.broken = bad.stalled = true;
        return bad;
    }
    int32_t k0 = (int32_t)tile - 1;
    for (;;) {
        const int32_t k = k0 - lane;
        const uint64_t *gl = a.tile_link + (size_t)(k < 0 ? 0 : k) * kLinkWords;
        uint32_t v[9];
        bool isP = false, done = k < 0;
        for (uint32_t spin = 0;; spin++) {
            if (!done) {
                bool pr = true;
#pragma unroll
                for (int i = 5; i < 9; i++) pr &= gran_get(gl + i, epoch, v[i]);
                if (pr) {
                    isP = done = true;
                } else {
                    bool ar = true;
#pragma unroll
                    for (int i = 0; i < 5; i++) ar &= gran_get(gl + i, epoch, v[i]);
                    done = ar;
                }
            }
            const unsigned long long pm = __ballot(isP), dm = __ballot(done);
            const int fp = pm ? __ffsll((long long)pm) - 1 : 64;
            const unsigned long long need = fp >= 63 ? ~0ull : ((2ull << fp) - 1ull);
            if ((dm & need) == need) break;
            if (spin > (1u << 24)) { // never expected: give up, the chain pass's last tile walks the part
                if (lane == 0) atomicAdd(&a.counters[kCtrChainStall], 1ull);
                ChainState bad = {};
                bad.broken = bad.stalled = true;
                return bad;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        const unsigned long long pm = __ballot(isP);
        const int fp = pm ? __ffsll((long long)pm) - 1 : 64;
        // aggregates of lanes fp-1 (earliest tile) .. 0 (the latest), composed
        // by a wave reduction: lane l takes in lanes (l, l + 2o) at step o
        const bool have_win = fp > 0;
        ChainAgg win = {};
        if (have_win) {
            bool gv = lane < fp;
            ChainAgg g = {};
            if (gv) {
                g.dsum = (int32_t)v[0];
                g.x = v[1];
                g.tshift = v[2] & 0x7fu;
                g.hasx = (v[2] & 0x80u) != 0u;
                g.broken = (v[2] & 0x100u) != 0u;
                g.s_l = (int32_t)(v[2] >> 16);
                g.bits = (uint64_t)v[3] | ((uint64_t)v[4] << 32);
            }
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t w = g.tshift | (g.hasx ? 0x80u : 0u) | (g.broken ? 0x100u : 0u) |
                                   (gv ? 0x200u : 0u) | ((uint32_t)g.s_l << 16);
                ChainAgg e;
                e.dsum = __shfl_down(g.dsum, o, 64);
                e.x = (uint32_t)__shfl_down((int)g.x, o, 64);
                const uint32_t ew = (uint32_t)__shfl_down((int)w, o, 64);
                const uint32_t elo = (uint32_t)__shfl_down((int)(uint32_t)g.bits, o, 64);
                const uint32_t ehi = (uint32_t)__shfl_down((int)(uint32_t)(g.bits >> 32), o, 64);
                e.tshift = ew & 0x7fu;
                e.hasx = (ew & 0x80u) != 0u;
                e.broken = (ew & 0x100u) != 0u;
                e.s_l = (int32_t)(ew >> 16);
                e.bits = (uint64_t)elo | ((uint64_t)ehi << 32);
                if (lane + o < 64 && (ew & 0x200u)) { // lanes (l, l + 2o): earlier tiles
                    g = gv ? chain_compose(e, g) : e;
                    gv = true;
                }
            }
            win.dsum = __builtin_amdgcn_readfirstlane(g.dsum);
            win.x = (uint32_t)__builtin_amdgcn_readfirstlane((int)g.x);
            const uint32_t w0 = (uint32_t)__builtin_amdgcn_readfirstlane(
                (int)(g.tshift | (g.hasx ? 0x80u : 0u) | (g.broken ? 0x100u : 0u) | ((uint32_t)g.s_l << 16)));
            win.tshift = w0 & 0x7fu;
            win.hasx = (w0 & 0x80u) != 0u;
            win.broken = (w0 & 0x100u) != 0u;
            win.s_l = (int32_t)(w0 >> 16);
            win.bits = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g.bits) |
                       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(g.bits >> 32)) << 32);
        }
        if (have_win) {
            acc = have_acc ? chain_compose(win, acc) : win;
            have_acc = true;
        }
        if (fp < 64) {
            ChainState st;
            st.roc = (uint32_t)__builtin_amdgcn_readlane((int)v[5], fp);
            const uint32_t w6 = (uint32_t)__builtin_amdgcn_readlane((int)v[6], fp);
            st.s_l = (int32_t)(w6 & 0xffffu);
            st.broken = (w6 & 0x10000u) != 0u;
            st.window = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)v[7], fp) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)v[8], fp) << 32);
            return have_acc ? chain_apply(st, acc) : st;
        }
        k0 -= 64;
    }
}

// Window shift and bits of the part's first f records (each lane's masked
// distances m[]), as walk_long's commit computes them.
__device__ __forceinline__ void chain_window(const uint32_t m[kChainPer], int f, uint32_t &tshift,
                                             uint64_t &bits) {
    const int lane = (int)(threadIdx.x & 63u);
    int32_t msum = 0;
#pragma unroll
    for (int r = 0; r < kChainPer; r++)
        if (lane * kChainPer + r < f) msum += (int32_t)m[r];
    const int32_t total = (int32_t)__reduce_add_sync(~0ull, (unsigned)msum);
    int32_t after = total - wave_excl_scan(msum);
    uint64_t b = 0ull;
#pragma unroll
    for (int r = 0; r < kChainPer; r++) {
        if (lane * kChainPer + r < f) {
            after -= (int32_t)m[r];
            if (after < 64) b |= 1ull << after;
        }
    }
    bits = wave_or64(b);
    tshift = (uint32_t)min(total, 64);
}

// One part of a long chain in this tile: records [j0, j0 + n) of the LDS
// window (n <= kWalkSpan).  head: the chain starts here (state from the
// context); else its state comes from the look-back.  out: the chain runs on
// into the next tile (this tile publishes for it).
// Where walk_long takes over a chain whose speculation broke in this tile.
struct ChainFix {
    uint32_t i0;      // sorted index of the first record it walks (kNoSlot: none)
    CtxState st;      // the context state before that record
};

template <bool REV>
__device__ __forceinline__ ChainFix chain_part(const BundleArgs &a, uint32_t tile, uint32_t epoch, uint32_t base, uint32_t j0,
                               int n, bool head, bool out, int32_t prev_seq_in, const WalkRec *s_rec,
                               const uint32_t *s_g0, const uint32_t *s_ok) {
    ChainFix fix;
    fix.i0 = kNoSlot;
    const int lane = (int)(threadIdx.x & 63u);
    const uint32_t slot = a.sk_out[base + j0];
    const CtxState st0 = a.ctx[slot];
    const KeySet *ks = a.keysets + st0.ks;
    WalkCtx c;
    c.enc = ks->enc_type; c.auth = ks->auth_type; c.T = ks->tag_len; c.kind = ks->kind;
    const bool mac = c.auth != SRTP_NULL_AUTHENTICATION;
    const int32_t prev_seq = head ? st0.b : prev_seq_in;
    // ---- local evaluation
    int32_t dpre[kChainPer];
    uint32_t m[kChainPer], xr[kChainPer];
    int32_t seqv[kChainPer];
    bool lok[kChainPer];
    int32_t lsum = 0;
#pragma unroll
    for (int r = 0; r < kChainPer; r++) {
        const int pos = lane * kChainPer + r;
        dpre[r] = 0; m[r] = 0u; xr[r] = 0u; seqv[r] = 0; lok[r] = false;
        if (pos >= n) continue;
        const WalkRec rec = s_rec[j0 + pos];
        const int32_t seq = (int32_t)(rec.word & 0xffffu);
        const int32_t sl = pos ? (int32_t)(s_rec[j0 + pos - 1].word & 0xffffu) : prev_seq;
        int32_t d;
        if (sl < 32768) d = (seq - sl > 32768) ? -1 : 0;
        else d = (sl - 32768 > seq) ? 1 : 0;
        const int64_t delta = (int64_t)d * 65536 + seq - sl;
        const int L = (int)(rec.lc & 0xffffu), C = (int)(rec.lc >> 16);
        bool ok = delta > 0;
        if (REV) {
            const int newL = mac ? (L - c.T > 0 ? L - c.T : 0) : L;
            if (!(rec.p & kRecSkipDec)) ok = ok && !enc_would_throw(c.enc, rec.h, newL - rec.h);
            if (mac) ok = ok && (s_ok[j0 + pos] & 1u) != 0u;
        } else {
            ok = ok && L + (mac ? c.T : 0) <= C && !enc_would_throw(c.enc, rec.h, L - rec.h);
        }
        lok[r] = ok;
        lsum += d;
        dpre[r] = lsum;
        m[r] = (uint32_t)((uint64_t)delta & 63u);
        seqv[r] = seq;
    }
    const int32_t dex = wave_excl_scan(lsum);
#pragma unroll
    for (int r = 0; r < kChainPer; r++) {
        dpre[r] += dex;
        if (REV && mac && lane * kChainPer + r < n) xr[r] = s_g0[j0 + lane * kChainPer + r] - (uint32_t)dpre[r];
    }
    const bool hasx = REV && mac && n > 0;
    const uint32_t x0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)xr[0]); // position 0's
    int fb = kChainPer;
#pragma unroll
    for (int r = kChainPer - 1; r >= 0; r--)
        if (lane * kChainPer + r < n && (!lok[r] || (hasx && xr[r] != x0))) fb = r;
    int first_bad = n;
    {
        const unsigned long long bl = __ballot(fb < kChainPer);
        if (bl) {
            const int l = __ffsll((long long)bl) - 1;
            first_bad = l * kChainPer + __builtin_amdgcn_readlane(fb, l);
        }
    }
    auto at = [&](const int32_t v[kChainPer], int pos) -> int32_t { // position pos's value (uniform)
        int32_t x = 0;
#pragma unroll
        for (int r = 0; r < kChainPer; r++)
            if (pos % kChainPer == r) x = __builtin_amdgcn_readlane(v[r], pos / kChainPer);
        return x;
    };
    if (out && !head) { // this tile's aggregate, before waiting on the tiles before it
        ChainAgg g;
        chain_window(m, first_bad, g.tshift, g.bits);
        g.dsum = first_bad ? at(dpre, first_bad - 1) : 0;
        g.s_l = first_bad ? at(seqv, first_bad - 1) : 0;
        g.x = x0;
        g.hasx = hasx;
        g.broken = first_bad < n;
        chain_publish_agg(a, tile, epoch, g);
    }
    // ---- the state the part starts from
    ChainState in;
    uint32_t g_in;
    if (head) {
        in.roc = (uint32_t)st0.a; in.s_l = st0.b; in.window = st0.window;
        in.broken = c.kind != SRTP_KIND_RTP || !(st0.flags & 1u);
        in.stalled = false;
        g_in = (uint32_t)st0.g;
    } else {
        in = chain_lookback(a, tile, epoch);
        g_in = in.roc;
    }
    if (in.broken) { // an earlier tile handed the chain over (or SRTCP / first packet)
        if (head) { // the whole chain goes to walk_long from its start
            fix.i0 = base + j0;
            fix.st = st0;
        }
        if (in.stalled && lane == 0) { // the fix-up walks the chain from this part on
            gran_put(a.tile_link + (size_t)tile * kLinkWords + 9, epoch, base + j0);
            atomicAdd(&a.ctl->n_stall, 1u);
        }
        if (out) chain_publish_state(a, tile, epoch, in);
        return fix;
    }
    int f = first_bad;
    if (hasx && in.roc != x0) f = 0;
    if (n > 0 && (int64_t)(int32_t)in.roc + at(dpre, n - 1) > (int64_t)0x7fffffff) f = 0;
    // ---- commit the records before f
#pragma unroll
    for (int r = 0; r < kChainPer; r++) {
        const int pos = lane * kChainPer + r;
        if (pos < f) {
            const WalkRec rec = s_rec[j0 + pos];
            const uint32_t p = rec.p & kRecIdxMask;
            const int L = (int)(rec.lc & 0xffffu);
            a.w_cw[p] = in.roc + (uint32_t)dpre[r];
            a.w_len[p] = (uint32_t)(REV ? (mac ? (L - c.T > 0 ? L - c.T : 0) : L) : L + (mac ? c.T : 0));
            a.w_status[p] = SRTP_STATUS_OK;
        }
    }
    ChainState st = in;
    uint32_t g_out = g_in;
    if (f > 0) {
        uint32_t tsh;
        uint64_t bits;
        chain_window(m, f, tsh, bits);
        st.roc = in.roc + (uint32_t)at(dpre, f - 1);
        st.s_l = at(seqv, f - 1);
        st.window = (tsh < 64u ? in.window << tsh : 0ull) | bits;
        g_out = st.roc;
    }
    CtxState cs = st0;
    cs.a = (int32_t)st.roc; cs.b = st.s_l; cs.g = (int32_t)g_out; cs.window = st.window;
    if (f < n) { // the speculation breaks at record f: walk_long walks the rest
        fix.i0 = base + j0 + (uint32_t)f;
        fix.st = cs;
        st.broken = true;
        if (out) chain_publish_state(a, tile, epoch, st);
        return fix;
    }
    if (out) chain_publish_state(a, tile, epoch, st);
    else if (lane == 0) a.ctx[slot] = cs; // the chain ends in this tile
    return fix;
}

// The stall fix-up (run by the chain pass's last tile to finish, when some
// tile's look-back gave up): the next tile from t on that left its part of a
// chain unwalked (link word 9 = the part's first sorted record), with the
// exact state the tile before it published -- every tile has finished, so it
// is there.  walk_long then walks the chain from that record to its end,
// exactly as after a speculation break; the tiles after the stalled one saw a
// broken state and committed nothing.  A part whose predecessor's state is
// itself broken is skipped: an earlier break or stall already hands that
// chain's rest to walk_long.
__device__ __forceinline__ ChainFix chain_stall_next(const BundleArgs &a, uint32_t epoch, uint32_t &t) {
    ChainFix f;
    f.i0 = kNoSlot;
    for (; t < gridDim.x; t++) {
        uint32_t i0 = 0u;
        const bool st = gran_get(a.tile_link + (size_t)t * kLinkWords + 9, epoch, i0);
        if (!__builtin_amdgcn_readfirstlane((int)st)) continue;
        uint32_t v[4];
        bool pr = true;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            pr &= gran_get(a.tile_link + (size_t)(t - 1u) * kLinkWords + 5 + i, epoch, v[i]);
            v[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)v[i]);
        }
        // not published would be a bug: the part stays unwalked (ERR_INTERNAL)
        if (!__builtin_amdgcn_readfirstlane((int)pr) || (v[1] & 0x10000u)) continue;
        i0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)i0);
        f.st = a.ctx[a.sk_out[i0]];
        f.st.a = (int32_t)v[0];
        f.st.b = (int32_t)(v[1] & 0xffffu);
        f.st.g = f.st.a;
        f.st.window = (uint64_t)v[2] | ((uint64_t)v[3] << 32);
        f.i0 = i0;
        t++;
        return f;
    }
    return f;
}

// One wave per workgroup owns the context segments that START among kWalkSpan
// consecutive sorted records, and stages those records plus a look-ahead of
// kWalkAhead more in LDS with one coalesced pass (plus, for unprotect, the
// verify pass's g0/auth_ok of each record, gathered in parallel); it compacts
// the segment starts and lane l walks the l-th segment: the per-context chain
// reads LDS (tens of cycles per record) instead of dependent HBM round trips.
// Only a segment longer than the look-ahead reads its tail from global memory.

// PASS 0: the first launch; PASS 1: the second (abort-on-throw's limit pass,
// or the long chains) -- separate instances, so that the first pass's
// registers do not pay for chain_part.
// The walk's LDS (k_walk's own; k_small's behind its T-table image).
template <bool REV>
struct WalkShared {
    WalkRec rec[kWalkWin];
    uint32_t key[kWalkWin];
    uint32_t g0[REV ? kWalkWin : 1];
    uint32_t ok[REV ? kWalkWin : 1];
    uint32_t start[kWalkSpan > kLongStep ? kWalkSpan : kLongStep];
    uint32_t pkey[kWalkSpan]; // keys of the tile before (long-chain test); medium chains: ROCs
    uint32_t med[kMedMax];
    uint32_t nstart, tile, nmed;
};
static_assert(kLongStep <= kWalkWin, "walk_long stages a step in the first pass's arrays");
static_assert(kLongStep <= kWalkSpan, "a medium chain's walk_long step keeps its ROCs in s_pkey");

// Tile `blk` of `nblk` (k_walk: blockIdx.x of gridDim.x), by one wave.
template <bool REV, bool SK, int PASS>
__device__ __forceinline__ void walk_tile(const BundleArgs &a, WalkShared<REV> &sh, uint32_t blk, uint32_t nblk) {
    constexpr int limit_pass = PASS;
    WalkRec *const s_rec = sh.rec;
    uint32_t *const s_key = sh.key;
    uint32_t *const s_g0 = sh.g0;
    uint32_t *const s_ok = sh.ok;
    uint32_t *const s_start = sh.start;
    uint32_t &s_nstart = sh.nstart;
    uint32_t *const s_pkey = sh.pkey;
    uint32_t &s_tile = sh.tile;
    uint32_t *const s_med = sh.med;
    uint32_t &s_nmed = sh.nmed;
    const bool two_pass = a.abort_on_error && a.ctl->any_throw;
    // Long chains (kWalkSpan records or more) are walked by the tiles they
    // cross (chain_part) in the second launch, unless abort-on-throw needs the
    // serial two-pass walk; the first pass only flags that there are some.
    const bool chains = !two_pass;
    const bool chain_pass = limit_pass && !two_pass;
    if (chain_pass && a.ctl->n_long == 0u) return; // no long chain in this bundle
    if (!limit_pass) { // the sort's last digit counts and k_parse's class counts, zero again for the next bundle
        for (uint32_t i = blk * kWalkBlock + threadIdx.x; i < a.sort_zero_words; i += nblk * kWalkBlock)
            a.sort_zero[i] = 0u;
        for (uint32_t i = blk * kWalkBlock + threadIdx.x; i < a.sort_zero_words / 256u * kClsWords;
             i += nblk * kWalkBlock)
            a.cls_tile[i] = 0u;
    }
    // The chain pass takes its tile from a ticket counter: a tile that waits on
    // the tiles before it for a long chain's state only waits on tiles already
    // running.
    uint32_t tile = blk;
    if (chain_pass) {
        if (threadIdx.x == 0) s_tile = atomicAdd(&a.ctl->tile_ticket, 1u);
        walk_sync();
        tile = s_tile;
    }
    const uint32_t base = tile * kWalkSpan;
    if (base >= a.n) return;
    const uint32_t span = min((uint32_t)kWalkSpan, a.n - base);
    const uint32_t win = min((uint32_t)kWalkWin, a.n - base);
    if (threadIdx.x == 0) { s_nstart = 0; s_nmed = 0; }
    if (chain_pass && base) {
#pragma unroll
        for (int k = 0; k < kWalkPer; k++) {
            const uint32_t j = threadIdx.x + k * kWalkBlock;
            s_pkey[j] = a.sk_out[base - kWalkSpan + j];
        }
    }
#pragma unroll
    for (int k = 0; k < kWalkWin / kWalkBlock; k++) {
        const uint32_t j = threadIdx.x + k * kWalkBlock;
        if (j < win) {
            const WalkRec r = a.sv_out[base + j];
            const uint32_t key = a.sk_out[base + j];
            s_rec[j] = r;
            s_key[j] = key;
            // only walked records carry a packet index: k_parse leaves the
            // record of a skipped / invalid packet unwritten (stale scratch)
            if (REV && key <= a.ctx_mask) {
                const uint32_t p = r.p & kRecIdxMask;
                const uint2 go = gok_of(a, p); // one 8-B gather: {g0, auth_ok}
                s_g0[j] = go.x;
                s_ok[j] = go.y;
            }
        }
    }
    walk_sync();
    const uint32_t prev_key = base ? a.sk_out[base - 1] : ~0u;
    // A chain of kWalkSpan records or more (it reaches the end of the tile it
    // starts in): record j's chain, starting at j, is that long iff the record
    // kLongMin - 1 places on carries its key.
    auto long_from = [&](uint32_t j, uint32_t key) -> bool {
        const uint32_t jl = j + kLongMin - 1u;
        const uint32_t kl = jl < win ? s_key[jl] : (base + jl < a.n ? a.sk_out[base + jl] : ~0u);
        return kl == key;
    };
    if constexpr (PASS == 1) if (chain_pass) {
        const uint32_t epoch = a.serial + 1u;
        // the part at the tile start that continues a chain from the tile before
        const uint32_t key0 = s_key[0];
        bool in_long = false;
        if (base && key0 == prev_key && key0 <= a.ctx_mask) {
            if (s_pkey[0] == key0) {
                in_long = true; // already kWalkSpan + 1 records
            } else {            // it starts at s in the tile before: long iff s + 255 has its key
                uint32_t sj = kWalkSpan;
#pragma unroll
                for (int k = 0; k < kWalkPer; k++) {
                    const uint32_t j = threadIdx.x * kWalkPer + k;
                    if (s_pkey[j] == key0 && (j == 0 || s_pkey[j - 1] != key0)) sj = j;
                }
                sj = (uint32_t)__reduce_min_sync(~0ull, sj);
                in_long = sj > 0 && sj < (uint32_t)kWalkSpan && s_key[sj - 1] == key0;
            }
        }
        // the run holding the tile's last record, and where it starts in the tile
        const uint32_t keyl = s_key[span - 1];
        uint32_t runs = span; // first position of keyl's run in the tile
#pragma unroll
        for (int k = 0; k < kWalkPer; k++) {
            const uint32_t j = threadIdx.x * kWalkPer + k;
            if (j < span && s_key[j] == keyl && (j == 0 || s_key[j - 1] != keyl)) runs = j;
        }
        runs = (uint32_t)__reduce_min_sync(~0ull, runs);
        const bool next_same = base + span < a.n &&
                               (span < win ? s_key[span] : a.sk_out[base + span]) == keyl;
        ChainFix fix_in, fix_head;
        fix_in.i0 = fix_head.i0 = kNoSlot;
        // a long chain that starts in this tile (it holds the tile's last record),
        // first: its state for the tiles after needs no look-back
        const bool head_long = keyl <= a.ctx_mask && !(in_long && runs == 0u) &&
                               !(runs == 0u && base && keyl == prev_key) && long_from(runs, keyl);
        if (head_long)
            fix_head = chain_part<REV>(a, tile, epoch, base, runs, (int)(span - runs), true, next_same, 0,
                                       s_rec, REV ? s_g0 : s_start, REV ? s_ok : s_start);
        // the part of a chain from the tiles before
        uint32_t e_in = 0u; // its end
        if (in_long) {
            uint32_t e = span;
#pragma unroll
            for (int k = 0; k < kWalkPer; k++) {
                const uint32_t j = threadIdx.x * kWalkPer + k;
                if (j < span && s_key[j] != key0) e = min(e, j);
            }
            e_in = (uint32_t)__reduce_min_sync(~0ull, e);
            int32_t prev_seq = 0;
            if (threadIdx.x == 0) prev_seq = (int32_t)(a.sv_out[base - 1].word & 0xffffu);
            prev_seq = __builtin_amdgcn_readfirstlane(prev_seq);
            fix_in = chain_part<REV>(a, tile, epoch, base, 0u, (int)e_in, false, e_in == span && next_same,
                                     prev_seq, s_rec, REV ? s_g0 : s_start, REV ? s_ok : s_start);
        }
        // walk_long takes over where a chain's speculation broke (the staged
        // window is no longer needed: its LDS is walk_long's)
        LongLds sm;
        sm.rec = s_rec;
        sm.roc = s_key;
        sm.g0 = REV ? s_g0 : s_start;
        sm.ok = REV ? s_ok : s_start;
        sm.info = s_start;
        // One walk_long call site for the tile's two hand-overs and, in the
        // last tile to finish, the stall fix-up's parts (chain_stall_next).
        uint32_t t_fix = 1u;
        bool fixup = false;
#pragma unroll 1
        for (int q = 0;; q++) {
            ChainFix f;
            if (q == 0) {
                f = fix_in;
            } else if (q == 1) {
                f = fix_head;
            } else {
                if (q == 2) { // every tile counts itself done; the last one runs the fix-up
                    uint32_t last = 0u;
                    if (threadIdx.x == 0) {
                        __threadfence();
                        last = atomicAdd(&a.ctl->tiles_done, 1u) == nblk - 1u ? 1u : 0u;
                        if (last) {
                            __threadfence();
                            last = __hip_atomic_load(&a.ctl->n_stall, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) != 0u ? 1u : 0u;
                        }
                    }
                    fixup = __builtin_amdgcn_readfirstlane((int)last) != 0;
                }
                if (!fixup) break;
                f = chain_stall_next(a, epoch, t_fix);
                if (f.i0 == kNoSlot) break;
            }
            if (f.i0 != kNoSlot) walk_long<REV, SK>(a, f.i0, sm, f.st);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < kWalkPer; k++) {
        const uint32_t j = threadIdx.x + k * kWalkBlock;
        if (j < span) {
            const uint32_t key = s_key[j];
            if (key <= a.ctx_mask && (j ? s_key[j - 1] : prev_key) != key)
                s_start[atomicAdd(&s_nstart, 1u)] = j;
        }
    }
    walk_sync();
    const uint32_t nstart = s_nstart;
    const bool dry = two_pass && !limit_pass;
#pragma unroll 1
    for (uint32_t q = threadIdx.x; q < nstart; q += kWalkBlock) {
        const uint32_t j = s_start[q];
        const uint32_t key = s_key[j];
        const uint32_t slot = key;
        // long chains are the chain pass's, unless abort-on-throw needs the serial walk
        if (chains && long_from(j, key)) {
            atomicOr(&a.ctl->n_long, 1u);
            continue;
        }
        // medium chains: the whole wave walks them after the lanes' own
        if (chains && j + kMedMin - 1u < win && s_key[j + kMedMin - 1u] == key) {
            s_med[atomicAdd(&s_nmed, 1u)] = j;
            continue;
        }
        CtxState st = a.ctx[slot];
        const KeySet *ks = a.keysets + st.ks;
        WalkCtx c;
        c.enc = ks->enc_type; c.auth = ks->auth_type; c.T = ks->tag_len; c.kind = ks->kind;
        c.check_replay = a.check_replay != 0;
        c.reverse = REV;
        const int32_t tid = (int32_t)(a.ctx_keys[slot] >> 32);
        const int32_t E = limit_pass ? a.e_min[tid] : 0x7fffffff;
        const uint32_t first_p = s_rec[j].p & kRecIdxMask;
        // One record of the chain; false ends it.
        auto step = [&](const WalkRec &r, uint32_t g0, uint32_t ok) -> bool {
            if (limit_pass && (int32_t)(r.p & kRecIdxMask) > E) return false;
            return walk_one<SK>(a, ks, c, st, r, g0, ok, dry, tid);
        };
        // The staged window, from LDS only: no global load in this loop, so
        // nothing waits on vmcnt -- which would also wait for walk_one's
        // status stores of earlier records.
        uint32_t jj = j;
        // Fast prefix (SRTP with seqNumSet, outside the abort-on-throw passes):
        // while each packet is the context's new highest index -- the steady
        // state of an in-order stream -- the state machine reduces to guessIndex,
        // a window shift and s_l/ROC advancing, with no replay drop; the packet
        // keeps that path when its tag checked out under the verify pass's ROC
        // and it neither throws nor (protect) overflows its capacity (the rules
        // of walk_long's speculation).  Such records cost a few instructions
        // here instead of walk_one's branches; the first record that leaves
        // the path, and every record after it, goes through walk_one.
        if (!two_pass && c.kind == SRTP_KIND_RTP && (st.flags & 1u)) {
            const bool mac = c.auth != SRTP_NULL_AUTHENTICATION;
            for (; jj < win; jj++) {
                if (s_key[jj] != key) break;
                const WalkRec rec = s_rec[jj];
                const int32_t seq = (int32_t)(rec.word & 0xffffu);
                const int32_t sl = st.b;
                int32_t d; // guessIndex :457-475
                if (sl < 32768) d = (seq - sl > 32768) ? -1 : 0;
                else d = (sl - 32768 > seq) ? 1 : 0;
                const uint32_t g = (uint32_t)st.a + (uint32_t)d;
                const int64_t delta = (java_lshl((int64_t)(int32_t)g, 16) | (int64_t)seq) -
                                      (java_lshl((int64_t)st.a, 16) | (int64_t)sl);
                const int L = (int)(rec.lc & 0xffffu), C = (int)(rec.lc >> 16);
                bool keep = delta > 0;
                int newL;
                if (REV) {
                    newL = mac ? (L - c.T > 0 ? L - c.T : 0) : L;
                    if (!(rec.p & kRecSkipDec)) keep = keep && !enc_would_throw(c.enc, rec.h, newL - rec.h);
                    if (mac) {
                        const uint32_t g0 = s_g0[jj], okb = s_ok[jj];
                        keep = keep && (g == g0 ? (okb & 1u) != 0u
                                                : (okb & 4u) != 0u && g == g0 - 1u && (okb & 2u) != 0u);
                    }
                } else {
                    newL = L + (mac ? c.T : 0);
                    keep = keep && newL <= C && !enc_would_throw(c.enc, rec.h, L - rec.h);
                }
                if (!keep) break;
                const uint32_t p = rec.p & kRecIdxMask;
                a.w_cw[p] = g;
                a.w_len[p] = (uint32_t)newL;
                a.w_status[p] = SRTP_STATUS_OK;
                // update :719-744 for delta > 0: the window shifts by delta & 63
                st.window = (uint64_t)java_lshl((int64_t)st.window, delta) | 1ull;
                st.a = (int32_t)g;
                st.b = seq;
                st.g = (int32_t)g;
            }
        }
        bool more = true;
        for (; jj < win; jj++) {
            if (s_key[jj] != key) { more = false; break; }
            if (!step(s_rec[jj], REV ? s_g0[jj] : 0u, REV ? s_ok[jj] : 0u)) { more = false; break; }
        }
        // A chain longer than the look-ahead continues from global memory.
        for (uint32_t i = base + jj; more && i < a.n; i++) {
            if (a.sk_out[i] != key) break;
            const WalkRec r = a.sv_out[i];
            uint32_t g0 = 0u, ok = 0u;
            if (REV) {
                const uint32_t p = r.p & kRecIdxMask;
                const uint2 go = gok_of(a, p);
                g0 = go.x; ok = go.y;
            }
            if (!step(r, g0, ok)) break;
        }
        if (dry) continue; // first of two passes: state is committed by the limit pass
        if (limit_pass && st.birth == a.serial && (int32_t)first_p > E) {
            // derived for a packet the reference never reached: forget it again
            __hip_atomic_store(&a.ctx_keys[slot], kTombKey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        a.ctx[slot] = st;
    }
    if (!chains) return;
    walk_sync();
    const uint32_t nmed = s_nmed;
    if (nmed == 0u) return;
    uint32_t med = threadIdx.x < nmed ? s_med[threadIdx.x] : 0u;
    // the chains' records are read from the staged window in place; walk_long's
    // per-step results go to arrays the one-lane walks no longer use
    LongWin pw;
    pw.rec = s_rec;
    pw.key = s_key;
    pw.g0 = REV ? s_g0 : s_start;
    pw.ok = REV ? s_ok : s_start;
    pw.base = base;
    pw.win = win;
    LongLds sm;
    sm.rec = s_rec;
    sm.roc = s_pkey;
    sm.g0 = REV ? s_g0 : s_start; // unused in place
    sm.ok = REV ? s_ok : s_start;
    sm.info = s_start;
    walk_sync();
#pragma unroll 1
    for (uint32_t m = 0; m < nmed; m++) {
        const uint32_t j = (uint32_t)__builtin_amdgcn_readlane((int)med, (int)m);
        const CtxState st = a.ctx[s_key[j]];
        walk_long<REV, SK>(a, base + j, sm, st, &pw);
    }
}

template <bool REV, bool SK, int PASS>
__global__ __launch_bounds__(kWalkBlock) void k_walk(BundleArgs a) {
    __shared__ WalkShared<REV> sh;
    walk_tile<REV, SK, PASS>(a, sh, blockIdx.x, gridDim.x);
}

// ====================================================== final status helper
// Final status of packet p (abort-aware); writes the caller's status/len.
__device__ __forceinline__ int32_t finish_status(const BundleArgs &a, uint32_t p) {
    // loads issued together, before the stores
    int32_t st = a.w_status[p];
    const uint32_t wl = a.w_len[p];
    if (st == kStPending) st = SRTP_STATUS_ERR_INTERNAL; // a walked packet no walk reached: never expected
    const bool thrown = a.abort_on_error && a.ctl->any_throw;
    if (st != SRTP_STATUS_SKIPPED && thrown) {
        const int32_t tid = packet_tid(a, p);
        if ((int32_t)p > a.e_min[tid]) st = SRTP_STATUS_NOT_PROCESSED;
    }
    a.status[p] = st;
    if (st != SRTP_STATUS_NOT_PROCESSED && st != SRTP_STATUS_SKIPPED && st != SRTP_STATUS_ERR_INTERNAL)
        a.len[p] = wl;
    return st;
}

__device__ __forceinline__ void make_iv_rtp(const KeySet *ks, const uint4 &hdr, uint32_t roc,
                                            uint32_t iv[4]) {
    // processPacketAESCM :482-525: salt ^ (0, SSRC, ROC, SEQ, 0)
    iv[0] = ks->salt[0];
    iv[1] = ks->salt[1] ^ hdr.z;        // bytes 8..11 = SSRC (BE in memory)
    iv[2] = ks->salt[2] ^ bswap(roc);
    iv[3] = ks->salt[3] ^ (hdr.x >> 16); // bytes 2..3 = SEQ
}

__device__ __forceinline__ void make_iv_rtcp(const KeySet *ks, const uint4 &hdr, uint32_t index,
                                             uint32_t iv[4]) {
    // SRTCPCryptoContext.processPacketAESCM :218-260: salt ^ (0, SSRC, 0, index, 0)
    iv[0] = ks->salt[0];
    iv[1] = ks->salt[1] ^ hdr.y;        // bytes 4..7 = RTCP SSRC
    iv[2] = ks->salt[2] ^ ((((index >> 24) & 0xffu) << 16) | (((index >> 16) & 0xffu) << 24));
    iv[3] = ks->salt[3] ^ (((index >> 8) & 0xffu) | ((index & 0xffu) << 8));
}

__device__ __forceinline__ void load_chunk(const uint8_t *pkt, int b, int lim, uint32_t d[16]) {
    const uint4 *qp = reinterpret_cast<const uint4 *>(pkt + 64 * b);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        uint4 v = make_uint4(0, 0, 0, 0);
        if (64 * b + 16 * m < lim) v = qp[m];
        d[4 * m] = v.x; d[4 * m + 1] = v.y; d[4 * m + 2] = v.z; d[4 * m + 3] = v.w;
    }
}

// Whole 64-B chunk b (inside the packet: no bounds checks, no branches).
__device__ __forceinline__ void load_chunk_full(const uint8_t *pkt, int b, uint32_t d[16]) {
    const uint4 *qp = reinterpret_cast<const uint4 *>(pkt + 64 * b);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const uint4 v = qp[m];
        d[4 * m] = v.x; d[4 * m + 1] = v.y; d[4 * m + 2] = v.z; d[4 * m + 3] = v.w;
    }
}

__device__ __forceinline__ void store_chunk_full(uint8_t *pkt, int b, const uint32_t d[16]) {
    uint4 *qp = reinterpret_cast<uint4 *>(pkt + 64 * b);
#pragma unroll
    for (int m = 0; m < 4; m++) qp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
}

// SRTP_TAIL_STEP: k_unprotect's fused loop takes the packet's ROC-carrying
// chunk in one more fused step (0.301 -> 0.296 ms per bundle).  The same for
// k_protect's last partial chunk was measured slower either way -- as a step
// after the loop (0.283 -> 0.299 ms: it spills) and as one more loop iteration
// with masked loads and stores (0.322 ms) -- and is not built
// (profiles/r03/kernel_experiments.md).
#ifndef SRTP_TAIL_STEP
#define SRTP_TAIL_STEP 1
#endif
__device__ __forceinline__ void store_chunk(uint8_t *pkt, int b, const Ctr &cs, const uint32_t d[16]) {
    uint4 *qp = reinterpret_cast<uint4 *>(pkt + 64 * b);
#pragma unroll
    for (int m = 0; m < 4; m++)
        if (64 * b + 16 * m < cs.end && 64 * b + 16 * m + 16 > cs.off)
            qp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
}

// A MacOnly instance (a small bundle: k_ctr_small ciphers the AES-CM +
// HMAC-SHA1 packets) needs the T-tables only for the other AES-CM packets of
// its workgroup (a NULL or Skein MAC): a workgroup of AES-CM + HMAC-SHA1
// packets alone skips the 128-KB fill.  Conservative: any other key set fills.
__device__ __forceinline__ bool mac_only_needs_te(const BundleArgs &a, uint32_t slot) {
    if (slot == kNoSlot) return false;
    const KeySet *ks = a.keysets + a.ctx[slot].ks;
    const int32_t ext = ks->ext, enc = ks->enc_type, auth = ks->auth_type;
    return !((ext == 0) & (enc == SRTP_AESCM_ENCRYPTION) & (auth == SRTP_HMACSHA1_AUTHENTICATION));
}

// ============================================================== k_protect
// Fused protect, one lane per packet: AES-CM in place (SRTPCipherCTR.process
// :94-121) + HMAC-SHA1 over the ciphertext (authenticatePacketHMAC :269-278)
// + trailer (RawPacket.append :203-220).  Packet bytes: one read, one write.
// Block b of a packet for the MAC: the 16-B pieces that start before lim
// (as the generic loops load them), zeros after.
__device__ __forceinline__ void load_block16(const uint8_t *pkt, int b, int lim, uint32_t w[16]) {
    // Branch-free: every piece is loaded -- one at or past lim from the
    // packet's first 16 bytes (inside its region), then zeroed -- so that the
    // compiler counts the loads in flight exactly: conditional loads made it
    // wait for all of them (vmcnt 0), the look-ahead's included, each block.
    const uint4 *qp = reinterpret_cast<const uint4 *>(pkt);
#pragma unroll
    for (int m = 0; m < 4; m++) {
        const int o = 64 * b + 16 * m;
        const bool ok = o < lim;
        const uint4 v = qp[ok ? (o >> 4) : 0];
        w[4 * m] = ok ? v.x : 0u; w[4 * m + 1] = ok ? v.y : 0u;
        w[4 * m + 2] = ok ? v.z : 0u; w[4 * m + 3] = ok ? v.w : 0u;
    }
}

// load_block16 for blocks below nb, zeros for the rest (the MAC's padding blocks)
__device__ __forceinline__ void load_or_zero16(const uint8_t *pkt, int b, int nb, int lim, uint32_t w[16]) {
    load_block16(pkt, b, b < nb ? lim : 0, w);
}

// The MAC-only loops' look-ahead: the next kMacAhead blocks of a packet held
// in registers, the oldest handed out and the one after the newest loaded.
constexpr int kMacAhead = 2; // ~3 us of loads in flight at ~1.5 us per block; each more costs 16 moves per block
struct MacRing {
    uint32_t q[kMacAhead][16];
    __device__ __forceinline__ void fill(const uint8_t *pkt, int b0, int nb, int lim) {
#pragma unroll
        for (int k = 0; k < kMacAhead; k++) load_or_zero16(pkt, b0 + k, nb, lim, q[k]);
    }
    // block b (the oldest) into w; block b + kMacAhead loaded behind it
    __device__ __forceinline__ void next(const uint8_t *pkt, int b, int nb, int lim, uint32_t w[16]) {
#pragma unroll
        for (int m = 0; m < 16; m++) w[m] = q[0][m];
#pragma unroll
        for (int k = 0; k + 1 < kMacAhead; k++)
#pragma unroll
            for (int m = 0; m < 16; m++) q[k][m] = q[k + 1][m];
        load_or_zero16(pkt, b + kMacAhead, nb, lim, q[kMacAhead - 1]);
        // a compiler-only barrier: without it the loop carries no loaded
        // values -- memory being unchanged, the compiler re-loads each block
        // where it is hashed, and the look-ahead is gone
        asm volatile("" ::: "memory");
    }
};

template <bool LK>
__device__ __forceinline__ void protect_one(const BundleArgs &a, const KeySet *__restrict__ ks,
                                            const char *__restrict__ lds, const TeBase &tb,
                                            uint32_t p, bool fused, bool mac_only = false) {
    uint8_t *pkt = a.seg + a.off[p];
    const bool do_enc = kf<LK>(ks->enc_type) == SRTP_AESCM_ENCRYPTION;
    // mac_only: k_ctr_small has ciphered the packet already (small bundles)
    const bool enc = do_enc && !mac_only;
    const bool do_mac = kf<LK>(ks->auth_type) != SRTP_NULL_AUTHENTICATION;
    const bool rtcp = kf<LK>(ks->kind) == SRTP_KIND_RTCP;
    const int T = (int)kf<LK>(ks->tag_len);
    const int L = (int)a.w_len[p] - (do_mac ? (T + (rtcp ? 4 : 0)) : 0);
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    const uint32_t cw = a.w_cw[p];
    Ctr cs;
    uint32_t suffix;
    if (!rtcp) {
        cs.off = rtp_header_len(pkt, hdr.x & 0xffu, (int)a.cap[p]);
        make_iv_rtp(ks, hdr, cw, cs.iv);
        suffix = cw;
    } else {
        cs.off = 8;
        make_iv_rtcp(ks, hdr, cw, cs.iv);
        suffix = do_enc ? (cw | 0x80000000u) : 0u;
    }
    cs.end = L;
#pragma unroll
    for (int k = 0; k < 4; k++) cs.carry[k] = 0u;
    PktKeys<LK> pk;
    pk_load<LK>(ks, pk);
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = kf<LK>(ks->ipad[k]);
    const int nb_data = (L + 63) >> 6;
    const int nb_inner = do_mac ? ((L + 12) >> 6) + 1 : 0;
    const int n_blocks = do_mac ? nb_inner + 1 : nb_data;
    int b = 0;
    // Steady state (AES-CM + HMAC, wave-uniform): iteration b encrypts chunk b
    // and hashes block b-1 -- a full data block, whose ciphertext c[] the
    // previous iteration produced -- in one interleaved step.  Chunks 0..B-1
    // are encrypted and blocks 0..B-2 hashed when it ends; block B-1 and the
    // rest go through the generic loop below.
    // (Chunks 1..B-1 lie wholly inside the packet: unconditional 64-B loads and
    // stores; bytes outside [off, end) are written back unchanged.)
    const int B = L >> 6;
    CtrPre cp; // AES-CM rounds 1-2 of this packet's counter blocks
    if (enc) ctr_precompute(lds, tb, pk_words(pk), cs.iv, cp);
    if (mac_only) {
        // the MAC over the ciphertext with kMacAhead blocks' loads in flight
        // while one is hashed: a lone packet's latency is this chain, and one
        // block of look-ahead left it waiting on memory
        MacRing q;
        q.fill(pkt, 0, nb_data, L);
        for (; b < n_blocks; b++) {
            uint32_t w[16];
            q.next(pkt, b, nb_data, L, w);
            if (b < nb_inner) inner_words(w, b, L, suffix);
            else outer_words<!LK>(w, h, ks);
            sha1_compress(h, w);
        }
    }
    if (fused && !mac_only && B >= 2) {
        uint32_t c[16];
        load_chunk(pkt, 0, L, c);
        pk_chunk_pre(lds, tb, pk, cp, cs, 0, c);
        store_chunk(pkt, 0, cs, c);
        const int hq = cs.off >> 4;
        const int nbw = SRTP_PRIO ? wave_max_i(B) : 0;
        for (b = 1; b < B; b++) {
            // packets past ~4 KB: the generic loop below finishes them
            if (ctr_pre_exhausted(4 * b - hq)) break;
            progress_prio(b, nbw);
            uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
            uint32_t K[16], d[16];
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = bswap(c[k]);
            pk_half<0>(lds, tb, pk, cp, 4 * b - hq, K, v, c);
            load_chunk_full(pkt, b, d);
            pk_half<1>(lds, tb, pk, cp, 4 * b - hq, K + 8, v, c);
#pragma unroll
            for (int k = 0; k < 5; k++) h[k] += v[k];
            ctr_apply_wave(cs, b, K, d);
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = d[k];
            store_chunk_full(pkt, b, d);
        }

        inner_words(c, b - 1, L, suffix); // block b-1 (B-1 may carry the suffix)
        sha1_compress(h, c);
    }
    // One AES site and one SHA-1 site: 64-B chunk b is loaded, encrypted in
    // place, stored, then hashed (inner blocks, then the outer block).
    for (; b < n_blocks; b++) {
        uint32_t w[16];
        uint4 *qp = reinterpret_cast<uint4 *>(pkt + 64 * b);
        if (b < nb_data) {
#pragma unroll
            for (int m = 0; m < 4; m++) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (64 * b + 16 * m < L) v = qp[m];
                w[4 * m] = v.x; w[4 * m + 1] = v.y; w[4 * m + 2] = v.z; w[4 * m + 3] = v.w;
            }
            if (enc && 64 * b + 64 > cs.off) {
                pk_chunk_pre(lds, tb, pk, cp, cs, b, w);
#pragma unroll
                for (int m = 0; m < 4; m++)
                    if (64 * b + 16 * m < L && 64 * b + 16 * m + 16 > cs.off)
                        qp[m] = make_uint4(w[4 * m], w[4 * m + 1], w[4 * m + 2], w[4 * m + 3]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) w[k] = 0u;
        }
        if (!do_mac) continue;
        if (b < nb_inner) {
            inner_words(w, b, L, suffix);
        } else {
            outer_words<!LK>(w, h, ks);
        }
        sha1_compress(h, w);
    }
    if (!do_mac) return;
    // append E|index (rbStore) then the tag, SRTCPCryptoContext :419-424
    if ((L & 3) == 0) { // a 4-byte-aligned trailer (packet regions start 16-B aligned): word stores
        trailer_write_aligned(reinterpret_cast<uint32_t *>(pkt + L), rtcp, suffix, h, T);
        return;
    }
    int o = L;
    if (rtcp) {
        pkt[o] = (uint8_t)(suffix >> 24); pkt[o + 1] = (uint8_t)(suffix >> 16);
        pkt[o + 2] = (uint8_t)(suffix >> 8); pkt[o + 3] = (uint8_t)suffix;
        o += 4;
    }
    tag_write(h, pkt + o, T);
}

#ifdef SRTP_STAMPS
// Diagnostic build (tools/stamps.sh): per wave, the realtime clock (100 MHz) at
// kernel entry, after the T-table fill and at the end (slots 0-2), the XCC id
// (slot 3) and the shader clock counter at the same points (slots 4-6).
#define STAMP(slot)                                                                        \
    do {                                                                                   \
        const unsigned long long _t = __builtin_amdgcn_s_memrealtime();                     \
        const unsigned long long _c = __builtin_amdgcn_s_memtime();                         \
        if ((threadIdx.x & 63u) == 0u) {                                                   \
            unsigned long long *_s =                                                       \
                a.stamps + (size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8; \
            _s[(slot)] = _t;                                                               \
            _s[4 + (slot)] = _c;                                                           \
        }                                                                                  \
    } while (0)
#define STAMP_XCC()                                                                        \
    do {                                                                                   \
        if ((threadIdx.x & 63u) == 0u)                                                     \
            a.stamps[(size_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + 3] = \
                (unsigned long long)__smid();                                             \
    } while (0)
#else
#define STAMP(slot) do {} while (0)
#define STAMP_XCC() do {} while (0)
#endif

// Adds this workgroup's status counts (s_cnt, LDS) to the engine counters:
// one 64-bit atomic per status present, on the workgroup's replica.
__device__ __forceinline__ void flush_status_counts(const BundleArgs &a, const uint32_t *s_cnt) {
    if (threadIdx.x < kTeCounters && s_cnt[threadIdx.x]) {
        const uint32_t rep = blockIdx.x & (uint32_t)(kCountReplicas - 1);
        atomicAdd(&a.counters[rep * kCtrStride + kCtrStatus + threadIdx.x],
                  (unsigned long long)s_cnt[threadIdx.x]);
    }
}

// MacOnly (a small bundle, BundleArgs::small_ctr): k_ctr_small has applied the
// AES-CM + HMAC-SHA1 packets' keystream; this kernel only MACs them.  A
// template, so the full-bundle kernel's code is what it was without it.
// (MacOnly instances run small bundles in workgroups of at most kMacBlock
// threads: registers for the MAC's look-ahead)
template <bool MacOnly>
__global__ __launch_bounds__(MacOnly ? kMacBlock : kProtectBlock) void k_protect(BundleArgs a) {
    // the status counts sit behind the T-table image
    __shared__ uint32_t s_te[kTeWords + kTeCounters];
    uint32_t *s_cnt = s_te + kTeWords;
    STAMP(0);
    STAMP_XCC();
    if (threadIdx.x < kTeCounters) s_cnt[threadIdx.x] = 0u;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p = i < a.n ? lane_packet(a, i) : i;
    if (!MacOnly || __syncthreads_or(i < a.n && mac_only_needs_te(a, a.p_slot[p])))
        fill_te4(s_te); // ends with a barrier
    STAMP(1);
    int32_t fs = -1;
    if (i < a.n) {
        fs = finish_status(a, p);
        atomicAdd(&s_cnt[status_counter(a, p, fs)], 1u);
    }
    __syncthreads();
    flush_status_counts(a, s_cnt);
    if (i >= a.n) return;
    bool todo = fs == SRTP_STATUS_OK;
    const uint32_t ks_id = todo ? a.ctx[a.p_slot[p]].ks : 0u;
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s_te);
    if (wave_mixes_keysets(todo, ks_id)) {
        // several key sets in this wave: the fused AES-CM + HMAC-SHA1 packets
        // run at once, each lane on its own key schedule; the rest (NULL
        // cipher or MAC, k_ext's ciphers) per key set below
        const KeySet *ks = a.keysets + ks_id;
        const bool lane = todo && ks->ext == 0u && ks->enc_type == SRTP_AESCM_ENCRYPTION &&
                          ks->auth_type == SRTP_HMACSHA1_AUTHENTICATION;
        if (lane) protect_one<true>(a, ks, lds, tb, p, !MacOnly, MacOnly);
        todo = todo && !lane;
    }
    for_each_keyset(todo, ks_id, [&](uint32_t ks_u) {
        const KeySet *ks = a.keysets + ks_u;
        if (sgpr(ks->ext)) return; // AES-F8 / AES-256-CM: k_ext
        const bool fused = sgpr(ks->enc_type) == SRTP_AESCM_ENCRYPTION &&
                           sgpr(ks->auth_type) != SRTP_NULL_AUTHENTICATION;
        const bool mac_only = MacOnly && fused && sgpr(ks->auth_type) == SRTP_HMACSHA1_AUTHENTICATION;
        // (a MacOnly instance never runs the fused loop: compiled out)
        protect_one<false>(a, ks, lds, tb, p, !MacOnly && fused, mac_only);
    });
    STAMP(2);
}

// ============================================================== ROC guess
// guessIndex (SRTPCryptoContext :457-475) against a context state: the ROC
// the walk would guess for `seq` were it the context's next packet.
__device__ __forceinline__ int32_t guess_roc(const CtxState &st, int32_t seq) {
    if (!(st.flags & 1u)) return st.a; // seqNumSet false: the ROC as is
    const int32_t s_l = st.b;
    if (s_l < 32768) return (seq - s_l > 32768) ? (int32_t)((uint32_t)st.a - 1u) : st.a;
    return (s_l - 32768 > seq) ? (int32_t)((uint32_t)st.a + 1u) : st.a;
}

// First sorted position of `key` (records are sorted by context), given
// sk[hi] == key: a lower bound over [0, hi].
__device__ __forceinline__ uint32_t chain_head(const uint32_t *__restrict__ sk, uint32_t hi, uint32_t key) {
    uint32_t lo = 0u;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sk[mid] < key) lo = mid + 1u;
        else hi = mid;
    }
    return lo;
}

// ============================================================== k_unprotect
// Unprotect, one lane per packet, before the walk: HMAC-SHA1 over the
// ciphertext (SRTPCryptoContext.authenticatePacket :237-266 /
// SRTCPCryptoContext :333-353) and, in the same pass, speculative in-place
// AES-CM decryption (:609-627 / :355-370) under the ROC guessed from the
// context state at bundle start.  Keeps the inner SHA-1 midstate before the
// ROC-carrying block and that block's ciphertext, so the walk can re-check a
// tag under another ROC cheaply; k_unprotect_fix repairs the rare packets the
// walk rejects or guesses differently.
template <bool LK>
__device__ __forceinline__ void unprotect_one(const BundleArgs &a, const KeySet *__restrict__ ks,
                                              const char *__restrict__ lds, const TeBase &tb,
                                              uint32_t p, const CtxState &st, bool fused,
                                              bool mac_only, bool save_state) {
    uint8_t *pkt = a.seg + a.off[p];
    const int L = (int)a.len[p];
    const int T = (int)kf<LK>(ks->tag_len);
    const bool rtp = kf<LK>(ks->kind) == SRTP_KIND_RTP;
    // HMAC-SHA1 here; a Skein-MAC key set's tags are checked by k_skein
    // (its key sets are k_ext's: no speculation, so nothing is done here but g0)
    const bool do_mac = kf<LK>(ks->auth_type) == SRTP_HMACSHA1_AUTHENTICATION;
    // speculative decryption: AES-128-CM only (k_ext deciphers the rest)
    const bool aes = kf<LK>(ks->enc_type) == SRTP_AESCM_ENCRYPTION && !kf<LK>(ks->ext);
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    Ctr cs;
    cs.off = 0;
    cs.iv[0] = cs.iv[1] = cs.iv[2] = cs.iv[3] = 0u;
    int end;       // bytes covered by the MAC and the decryption: [0, end) / [off, end)
    uint32_t suffix;
    bool spec = false;
    if (rtp) {
        const int32_t seq = (int32_t)(bswap(hdr.x) & 0xffffu);
        // guessIndex on the bundle-start state (for a packet deep in a long
        // chain, k_unprotect's state yields the chain's guess; see there)
        const int32_t g = guess_roc(st, seq);
        a.gok[2 * (size_t)(p)] = (uint32_t)g;
        end = do_mac ? (L - T > 0 ? L - T : 0) : L;
        suffix = (uint32_t)g;
        const uint32_t fl = a.flags ? a.flags[p] : 0u;
        if (aes && !(fl & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE))) {
            cs.off = rtp_header_len(pkt, hdr.x & 0xffu, (int)a.cap[p]);
            // Speculate only when the header fields the IV and the header length
            // are read from (SSRC, SEQ, CC, X, extension length) lie before the
            // decrypted region; a negative extension length can put them inside
            // it, and k_unprotect_fix must then still see the original bytes.
            const uint32_t b0 = hdr.x & 0xffu;
            const int fixed = 12 + 4 * (int)(b0 & 0x0fu) + ((b0 & 0x10u) ? 4 : 0);
            spec = cs.off >= fixed && !ctr_would_throw(cs.off, end - cs.off) && end - cs.off > 0;
            if (spec) make_iv_rtp(ks, hdr, (uint32_t)g, cs.iv);
        }
    } else {
        const int io = L - 4 - T;
        if (io < 0) { a.spec[p] = 0u; return; } // the reference throws here (k_walk): no decryption due
        suffix = ld_be32(pkt + io);
        end = do_mac ? (io > 0 ? io : 0) : L;
        if (aes && (suffix & 0x80000000u) && end - 8 > 0) {
            cs.off = 8;
            make_iv_rtcp(ks, hdr, suffix & 0x7FFFFFFFu, cs.iv);
            spec = true;
        }
    }
    // for k_unprotect_fix: decrypted here, AES-CM packet of the fused path,
    // RTP, DISCARD/SILENCE (so it needs no key-set lookup to decide a repair)
    a.spec[p] = (spec ? kSpecDid : 0u) | (aes ? kSpecAes : 0u) | (rtp ? kSpecRtp : 0u) |
                (rtp && a.flags && (a.flags[p] & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE)) ? kSpecSkip : 0u);
    if (!do_mac && !spec) return;
    // mac_only: k_ctr_small decrypts the packets marked kSpecDid (small bundles)
    cs.end = spec && !mac_only ? end : 0;
#pragma unroll
    for (int k = 0; k < 4; k++) cs.carry[k] = 0u;
    PktKeys<LK> pk;
    pk_load<LK>(ks, pk);
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = kf<LK>(ks->ipad[k]);
    const int nb_full = end >> 6;
    const int nb_data = (end + 63) >> 6;
    const int nb_inner = ((end + 12) >> 6) + 1;
    const int n_blocks = do_mac ? nb_inner + 1 : nb_data;
    int b = 0;
    if (fused && !mac_only && nb_full >= 2) {
        // AES-CM + HMAC, wave-uniform, over the full blocks before the
        // ROC-carrying one.  As in protect, iteration b computes the keystream
        // of chunk b beside the hash of block b-1 (loaded the iteration
        // before), so chunk b's load has half a chunk step to land.
        const int hq = cs.off >> 4;
        CtrPre cp;
        ctr_precompute(lds, tb, pk_words(pk), cs.iv, cp);
        uint32_t c[16];
        load_chunk_full(pkt, 0, c);
        {   // chunk 0 holds the header: generic keystream, masked below off
            uint32_t d[16];
#pragma unroll
            for (int k = 0; k < 16; k++) d[k] = c[k];
            pk_chunk_pre(lds, tb, pk, cp, cs, 0, d);
            store_chunk(pkt, 0, cs, d); // cs.end = 0 without speculation: no store
        }
        const int nbw = SRTP_PRIO ? wave_max_i(nb_full) : 0;
        for (b = 1; b < nb_full; b++) {
            if (ctr_pre_exhausted(4 * b - hq)) break; // generic loop finishes
            progress_prio(b, nbw);
            uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
            uint32_t K[16], d[16];
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = bswap(c[k]);
            pk_half<0>(lds, tb, pk, cp, 4 * b - hq, K, v, c);
            load_chunk_full(pkt, b, d);
            pk_half<1>(lds, tb, pk, cp, 4 * b - hq, K + 8, v, c);
#pragma unroll
            for (int k = 0; k < 5; k++) h[k] += v[k];
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = d[k]; // ciphertext of chunk b, hashed next
            ctr_apply_wave(cs, b, K, d); // cs.end = 0 without speculation: d unchanged
            store_chunk_full(pkt, b, d);
        }
        // The ROC-carrying chunk nb_full (MAC'd bytes up to end) in one more
        // fused step: its keystream beside the hash of block nb_full-1, the
        // midstate and ciphertext saved for the walk, decrypted in place --
        // instead of the MAC loop's reload and the decryption loop's
        // unoverlapped AES below.
        const bool ext = SRTP_TAIL_STEP && b == nb_full && 64 * nb_full < end &&
                         !ctr_pre_exhausted(4 * b - hq);
        if (ext) {
            uint32_t v[5] = {h[0], h[1], h[2], h[3], h[4]};
            uint32_t K[16], d[16];
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = bswap(c[k]);
            pk_half<0>(lds, tb, pk, cp, 4 * b - hq, K, v, c);
            load_chunk(pkt, b, end, d);
            pk_half<1>(lds, tb, pk, cp, 4 * b - hq, K + 8, v, c);
#pragma unroll
            for (int k = 0; k < 5; k++) h[k] += v[k];
            if (rtp && save_state) { // midstate + ciphertext of the ROC-carrying block
                uint32_t *mp = a.mid + 5 * (size_t)p;
#pragma unroll
                for (int k = 0; k < 5; k++) mp[k] = h[k];
                if (spec) {
                    uint4 *tp = reinterpret_cast<uint4 *>(a.tailc + 16 * (size_t)p);
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        tp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
                }
            }
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = d[k]; // ciphertext of block nb_full
            ctr_apply(cs, b, K, d); // cs.end = 0 without speculation: d unchanged
            store_chunk(pkt, b, cs, d);
            // the rest of the MAC here (nothing is left to decrypt: end lies in
            // this chunk), so that no AES state stays live past this step
            inner_words(c, b, end, suffix);
            sha1_compress(h, c);
            for (b = b + 1; b <= nb_inner; b++) {
                uint32_t w[16];
#pragma unroll
                for (int k = 0; k < 16; k++) w[k] = 0u;
                if (b < nb_inner) inner_words(w, b, end, suffix);
                else outer_words<!LK>(w, h, ks);
                sha1_compress(h, w);
            }
            a.gok[2 * (size_t)(p) + 1] = tag_matches_at(h, pkt, L - T, T) ? 1u : 0u;
            return;
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) c[k] = bswap(c[k]);
            sha1_compress(h, c); // block b-1, a full block before the ROC-carrying one
        }
    }
    // The blocks left after the fused loop: first the MAC over their
    // ciphertext, then their decryption -- two loops, so that no AES state
    // (round keys, counter, keystream carry) is live across SHA-1 and nothing
    // spills to scratch; the round keys are reloaded for the second loop.
    const int b_tail = b;
    if (do_mac && mac_only) {
        // as below, with kMacAhead blocks' loads in flight while one is hashed
        // (a lone packet's latency is this chain)
        MacRing q;
        q.fill(pkt, b, nb_data, end);
        for (; b < n_blocks; b++) {
            uint32_t d[16];
            q.next(pkt, b, nb_data, end, d);
            if (b == nb_full && rtp && save_state) { // midstate + ciphertext of the ROC-carrying block
                uint32_t *mp = a.mid + 5 * (size_t)p;
#pragma unroll
                for (int m = 0; m < 5; m++) mp[m] = h[m];
                if (spec) {
                    uint4 *tp = reinterpret_cast<uint4 *>(a.tailc + 16 * (size_t)p);
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        tp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
                }
            }
            if (b < nb_inner) inner_words(d, b, end, suffix);
            else outer_words<!LK>(d, h, ks);
            sha1_compress(h, d);
        }
        a.gok[2 * (size_t)(p) + 1] = tag_matches_at(h, pkt, L - T, T) ? 1u : 0u;
    } else if (do_mac) {
        for (; b < n_blocks; b++) {
            uint32_t d[16];
            const uint4 *qp = reinterpret_cast<const uint4 *>(pkt + 64 * b);
#pragma unroll
            for (int m = 0; m < 4; m++) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (b < nb_data && 64 * b + 16 * m < end) v = qp[m];
                d[4 * m] = v.x; d[4 * m + 1] = v.y; d[4 * m + 2] = v.z; d[4 * m + 3] = v.w;
            }
            if (b == nb_full && rtp && save_state) { // midstate + ciphertext of the ROC-carrying block
                uint32_t *mp = a.mid + 5 * (size_t)p;
#pragma unroll
                for (int k = 0; k < 5; k++) mp[k] = h[k];
                if (spec) {
                    uint4 *tp = reinterpret_cast<uint4 *>(a.tailc + 16 * (size_t)p);
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        tp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
                }
            }
            if (b < nb_inner) inner_words(d, b, end, suffix);
            else outer_words<!LK>(d, h, ks);
            sha1_compress(h, d);
        }
        a.gok[2 * (size_t)(p) + 1] = tag_matches_at(h, pkt, L - T, T) ? 1u : 0u;
    }
    if (spec && !mac_only) {
        // reload the round keys through an opaque copy of the key-set pointer:
        // with the plain pointer the compiler keeps the first load's VGPR copies
        // live across the MAC loop instead (44 VGPRs spilled to scratch)
        const KeySet *ks2 = ks;
        asm volatile("" : "+v"(ks2));
        PktKeys<LK> pk2;
        pk_load<LK>(ks2, pk2);
        for (int c = b_tail; c < nb_data; c++) {
            if (64 * c + 64 <= cs.off) continue;
            uint32_t d[16];
            uint4 *qp = reinterpret_cast<uint4 *>(pkt + 64 * c);
#pragma unroll
            for (int m = 0; m < 4; m++) {
                uint4 v = make_uint4(0, 0, 0, 0);
                if (64 * c + 16 * m < end) v = qp[m];
                d[4 * m] = v.x; d[4 * m + 1] = v.y; d[4 * m + 2] = v.z; d[4 * m + 3] = v.w;
            }
            pk_chunk(lds, tb, pk2, cs, c, d);
#pragma unroll
            for (int m = 0; m < 4; m++)
                if (64 * c + 16 * m < end && 64 * c + 16 * m + 16 > cs.off)
                    qp[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
        }
    }
}


template <bool MacOnly> // as k_protect's: k_ctr_small decrypts afterwards
__global__ __launch_bounds__(MacOnly ? kMacBlock : kUnprotectBlock) void k_unprotect(BundleArgs a) {
    __shared__ uint32_t s_te[kTeWords];
    STAMP(0);
    STAMP_XCC();
    // the packet's context state and whether it lies deep in a long chain
    // (its kLongRank-th predecessor in sort order has its context), loaded
    // while the T-tables fill
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < a.n;
    const uint32_t p = live ? lane_packet(a, i) : i;
    uint32_t slot = kNoSlot, pos = 0u;
    if (live) {
        slot = a.p_slot[p];
        pos = a.spos[p];
    }
    const bool todo = slot != kNoSlot;
    CtxState st = {};
    bool lng = false;
    uint32_t far = 0u;
    if (todo) {
        st = a.ctx[slot];
        far = a.far[slot];
        lng = pos >= kLongRank && a.sk_out[pos - kLongRank] == slot;
    }
    // The walk re-checks a tag (from the midstate and ciphertext saved here)
    // only under a ROC other than the one speculated on.  If every packet of
    // the context in this bundle lies within 16384 of its bundle-start s_l,
    // that s_l and all their SEQs lie within 32768 of each other, guessIndex
    // (:457-475) adds 0 to the ROC for every pair of them, and the ROC cannot
    // change within the bundle: the walk's ROC is the speculated one for every
    // packet and nothing need be saved.  Contexts without seqNumSet, deep
    // chains and contexts with a far packet (k_parse, BundleArgs::far) save it.
    const bool quiet = todo && !lng && (st.flags & 1u) && far != a.serial + 1u;
    if (!MacOnly || __syncthreads_or(todo && mac_only_needs_te(a, slot))) fill_te4(s_te);
    STAMP(1);
    if (!live) return;
    // The ROC speculated on is the walk's guess were the packet its context's
    // next: guessIndex on the bundle-start state, exact while no earlier
    // packet of the context in this bundle has wrapped.  Deep in a long chain
    // (one SSRC carrying thousands of packets in one bundle) the chain may
    // have wrapped on the way, maybe more than once: guess the ROC whose index
    // lies nearest the chain head's index plus the packet's rank in the chain
    // (exact for an in-order chain losing fewer than 32768 packets).  It is
    // handed over as a state whose guessIndex returns it (seqNumSet clear), so
    // nothing more stays live across the key-set loop.  A wrong guess only
    // costs the walk a re-check of the tag.
    if (lng) {
        const uint32_t h = chain_head(a.sk_out, pos - kLongRank, slot);
        const int32_t seq_h = (int32_t)(a.sv_out[h].word & 0xffffu);
        const int32_t seq = (int32_t)(a.sv_out[pos].word & 0xffffu); // RTP: the packet's SEQ
        const int64_t e = (int64_t)guess_roc(st, seq_h) * 65536 + seq_h + (int64_t)(pos - h);
        st.a = (int32_t)((e - seq + 32768) >> 16);
        st.flags &= ~1u;
    }
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s_te);
    bool rest = todo;
    if (wave_mixes_keysets(todo, st.ks)) { // see k_protect
        const KeySet *ks = a.keysets + st.ks;
        const bool lane = todo && ks->ext == 0u && ks->enc_type == SRTP_AESCM_ENCRYPTION &&
                          ks->auth_type == SRTP_HMACSHA1_AUTHENTICATION;
        if (lane) unprotect_one<true>(a, ks, lds, tb, p, st, !MacOnly, MacOnly, !quiet);
        rest = todo && !lane;
    }
    for_each_keyset(rest, st.ks, [&](uint32_t ks_u) {
        const KeySet *ks = a.keysets + ks_u;
        const bool fused = sgpr(ks->enc_type) == SRTP_AESCM_ENCRYPTION && !sgpr(ks->ext) &&
                           sgpr(ks->auth_type) != SRTP_NULL_AUTHENTICATION;
        const bool mac_only = MacOnly && fused && sgpr(ks->auth_type) == SRTP_HMACSHA1_AUTHENTICATION;
        unprotect_one<false>(a, ks, lds, tb, p, st, !MacOnly && fused, mac_only, !quiet);
    });
    STAMP(2);
}

// ============================================================== k_unprotect_fix
// Final statuses/lengths of an unprotect bundle, and the repair of packets
// whose speculative decryption the walk overturned: undo the keystream of the
// guessed ROC (or of the SRTCP trailer's index) and/or apply the walk's.
// Usually nothing needs repair and a workgroup exits after its statuses; when
// some do (replays, forged tags, ROC guesses overturned in-bundle -- a flood of
// them must not cost more than a decryption), the workgroup builds the LDS
// T-tables and repairs at full AES speed.
// Repairs are compacted within the workgroup first: the packets to repair
// are listed in LDS and their 64-B chunks spread over the lanes, one chunk
// per lane (counter-mode blocks are independent), so that a few scattered
// repairs (replays and forgeries of a faulty link: ~2.5 % of the packets)
// cost one short AES step instead of every wave that holds one walking its
// packet chunk by chunk (which cost almost an AES pass over the bundle).
__global__ __launch_bounds__(kAesBlock) void k_unprotect_fix(BundleArgs a) {
    __shared__ uint32_t s_te[kTeWords + kTeCounters];
    __shared__ uint2 s_rep[kAesBlock]; // {packet | did << 30 | need << 31, original length}
    __shared__ uint32_t s_nrep;
    uint32_t *s_cnt = s_te + kTeWords;
    if (threadIdx.x < kTeCounters) s_cnt[threadIdx.x] = 0u;
    if (threadIdx.x == 0) s_nrep = 0u;
    __syncthreads();
    const uint32_t p0 = blockIdx.x * blockDim.x + threadIdx.x;
    bool repair = false, did = false, need = false;
    int L0 = 0;
    if (p0 < a.n) {
        // every per-packet word first, all in flight together (the status
        // stores below would otherwise order the loads after them)
        L0 = (int)a.len[p0];
        const uint32_t slot = a.p_slot[p0];
        const uint32_t sw = a.spec[p0]; // k_unprotect's summary: no context / key-set loads
        const uint32_t cw = a.w_cw[p0], g0 = a.gok[2 * (size_t)(p0)];
        const int32_t st = finish_status(a, p0);
        atomicAdd(&s_cnt[status_counter(a, p0, st)], 1u);
        if (slot != kNoSlot) {
            did = (sw & kSpecDid) != 0u;
            const bool rtp = (sw & kSpecRtp) != 0u;
            if (st == SRTP_STATUS_OK && (sw & kSpecAes)) need = rtp ? !(sw & kSpecSkip) : (cw & 0x80000000u) != 0;
            repair = (did || need) && !(did && need && (!rtp || g0 == cw));
        }
    }
    {   // list this wave's repairs (one LDS atomic per wave)
        const unsigned long long m = __ballot(repair);
        if (m) {
            const uint32_t lane = threadIdx.x & 63u;
            const int first = __ffsll((long long)m) - 1;
            uint32_t base = 0u;
            if ((int)lane == first) base = atomicAdd(&s_nrep, (uint32_t)__popcll(m));
            base = (uint32_t)__builtin_amdgcn_readlane((int)base, first);
            if (repair) {
                const uint32_t k = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                s_rep[k] = make_uint2(p0 | (did ? 1u << 30 : 0u) | (need ? 1u << 31 : 0u), (uint32_t)L0);
            }
        }
    }
    __syncthreads();
    flush_status_counts(a, s_cnt);
    const uint32_t nrep = s_nrep;
    if (nrep == 0u) return; // the common case: speculation was right
    // Each listed packet's chunks become jobs, one chunk per lane: a packet's
    // keystream blocks are independent, so no lane walks a whole packet.
    // s_pref[k] = jobs of the packets before k (the T-table image is built
    // after this scan; its LDS is not used yet).
    uint32_t *s_pref = s_te; // [kAesBlock + 1]
    if (threadIdx.x < nrep) {
        const uint2 job = s_rep[threadIdx.x];
        s_pref[threadIdx.x + 1] = (job.y + 63u) >> 6; // chunks of [0, L0)
    }
    if (threadIdx.x == 0) s_pref[0] = 0u;
    __syncthreads();
    if (threadIdx.x == 0)
        for (uint32_t k = 1; k <= nrep; k++) s_pref[k] += s_pref[k - 1];
    __syncthreads();
    const uint32_t n_jobs = s_pref[nrep];
    // the job list is kept in registers (one round of up to 4 jobs per lane),
    // since the table fill below overwrites s_pref
    constexpr int kJobsPerLane = 4;
    uint32_t jk[kJobsPerLane], jc[kJobsPerLane];
    int n_mine = 0;
#pragma unroll
    for (int q = 0; q < kJobsPerLane; q++) {
        const uint32_t j = threadIdx.x + (uint32_t)q * kAesBlock;
        jk[q] = 0u;
        jc[q] = 0u;
        if (j < n_jobs) {
            uint32_t lo = 0u, hi = nrep; // last k with s_pref[k] <= j
            while (hi - lo > 1u) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_pref[mid] <= j) lo = mid;
                else hi = mid;
            }
            jk[q] = lo;
            jc[q] = j - s_pref[lo];
            n_mine = q + 1;
        }
    }
    const bool overflow = n_jobs > (uint32_t)kJobsPerLane * kAesBlock; // > 4096 chunks: whole packets
    __syncthreads();
    fill_te4(s_te);
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s_te);
    // (rare) more chunks than jobs: lane k < nrep walks packet k whole
    const int rounds = overflow ? 1 : n_mine;
    for (int q = 0; q < (overflow ? 1 : kJobsPerLane); q++) {
        bool act;
        uint32_t k, c_first, c_last;
        if (overflow) {
            act = threadIdx.x < nrep;
            k = threadIdx.x;
            c_first = 0u;
            c_last = 0xffffu;
        } else {
            act = q < rounds;
            k = jk[q];
            c_first = c_last = jc[q];
        }
        const uint2 job = act ? s_rep[k] : make_uint2(0u, 0u);
        const uint32_t p = job.x & 0x3fffffffu;
        const bool jdid = (job.x >> 30) & 1u;
        const bool jneed = (job.x >> 31) != 0u;
        const int jL0 = (int)job.y;
        const uint32_t ks_id = act ? a.ctx[a.p_slot[p]].ks : 0u;
        for_each_keyset(act, ks_id, [&](uint32_t ks_u) {
            const KeySet *ks = a.keysets + ks_u;
            RoundKeys rk;
            load_round_keys_uniform(ks, rk);
            uint8_t *pkt = a.seg + a.off[p];
            const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
            const int T = ks->tag_len;
            const bool mac = ks->auth_type != SRTP_NULL_AUTHENTICATION;
            Ctr spec, real;
            if (ks->kind == SRTP_KIND_RTP) {
                real.off = rtp_header_len(pkt, hdr.x & 0xffu, (int)a.cap[p]);
                real.end = mac ? (jL0 - T > 0 ? jL0 - T : 0) : jL0;
                make_iv_rtp(ks, hdr, a.gok[2 * (size_t)(p)], spec.iv);
                make_iv_rtp(ks, hdr, a.w_cw[p], real.iv);
            } else {
                real.off = 8;
                real.end = mac ? (jL0 - T - 4 > 0 ? jL0 - T - 4 : 0) : jL0;
                const uint32_t sidx = ld_be32(pkt + jL0 - 4 - T) & 0x7FFFFFFFu;
                make_iv_rtcp(ks, hdr, sidx, spec.iv);
                make_iv_rtcp(ks, hdr, a.w_cw[p] & 0x7FFFFFFFu, real.iv);
            }
            if (real.off < 0 || real.off > real.end) real.off = real.end; // nothing to cipher
            spec.off = real.off;
            spec.end = jdid ? real.end : 0;
            const int end = real.end;
            if (!jneed) real.end = 0;
            Ctr span = real;
            span.end = end;
            const int c0 = max((int)c_first, span.off >> 6);
            // keystream carry into chunk c0: block 4 c0 - off/16 - 1 (zero when
            // c0 holds `off`: the words before it are masked)
            const int hq = span.off >> 4;
#pragma unroll
            for (int k2 = 0; k2 < 4; k2++) spec.carry[k2] = real.carry[k2] = 0u;
            if (c0 > (span.off >> 6) && 64 * c0 < end) {
                uint32_t x[4], y[4];
                ctr_input(spec.iv, 4 * c0 - hq - 1, x);
                ctr_input(real.iv, 4 * c0 - hq - 1, y);
                aes_encrypt2(lds, tb, rk, x, y);
#pragma unroll
                for (int k2 = 0; k2 < 4; k2++) { spec.carry[k2] = x[k2]; real.carry[k2] = y[k2]; }
            }
            for (int c = c0; c <= (int)c_last && 64 * c < end; c++) {
                uint32_t d[16];
                load_chunk(pkt, c, end, d);
                if (jdid) ctr_chunk(lds, tb, rk, spec, c, d);
                if (jneed) ctr_chunk(lds, tb, rk, real, c, d);
                store_chunk(pkt, c, span, d);
            }
        });
        if (act && c_first == 0u) atomicAdd(&a.counters[kCtrRepaired], 1ull);
    }
}

// ============================================================== k_ext
// Packets of the key sets the fused kernels leave out -- AES-F8 (SRTPCipherF8;
// SDES F8_128_HMAC_SHA1_80) and AES-256-CM -- after the final statuses of
// k_protect / k_unprotect_fix.  Protect: encryption, then the
// HMAC over the ciphertext and the trailer.  Unprotect: k_unprotect already
// checked the tag (HMAC is over the ciphertext, independent of the cipher) and
// did not speculate, so only the accepted packets are deciphered here.  The F8
// keystream is a chain, S(j) = E(k_e, IV' ^ S(j-1) ^ j), so a lane walks its
// packet block by block.

// Round keys at p (wave-uniform) into SGPRs.
__device__ __forceinline__ void load_rk_uniform(const uint32_t *__restrict__ p, RoundKeys &rk) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < 11; i++) {
        const uint4 v = q[i];
        rk.k[4 * i] = sgpr(v.x); rk.k[4 * i + 1] = sgpr(v.y);
        rk.k[4 * i + 2] = sgpr(v.z); rk.k[4 * i + 3] = sgpr(v.w);
    }
}

// One packet's AES-F8 work: IV, ciphered region [off, off + len), and for
// protect the HMAC trailer.
struct F8Job {
    uint8_t *pkt;
    int off, len;   // ciphered region (off a multiple of 4; len <= 0: none)
    uint32_t iv[4]; // IV, little-endian words
    int L;          // protect: MAC length (the packet before its trailer)
    uint32_t suffix;
    bool rtcp;
};

__device__ __forceinline__ F8Job f8_job(const BundleArgs &a, const KeySet *ks, uint32_t p) {
    F8Job j;
    j.pkt = a.seg + a.off[p];
    const uint4 hdr = *reinterpret_cast<const uint4 *>(j.pkt);
    const int T = (int)sgpr(ks->tag_len);
    const bool mac = sgpr(ks->auth_type) != SRTP_NULL_AUTHENTICATION;
    const uint32_t cw = a.w_cw[p];
    j.rtcp = sgpr(ks->kind) == SRTP_KIND_RTCP;
    if (!j.rtcp) {
        // processPacketAESF8 :532-555: IV = 0 || header[1..11] || ROC_be
        j.iv[0] = hdr.x & 0xffffff00u; j.iv[1] = hdr.y; j.iv[2] = hdr.z; j.iv[3] = bswap(cw);
        j.L = (int)a.len[p] - (!a.reverse && mac ? T : 0);
        j.off = rtp_header_len(j.pkt, hdr.x & 0xffu, (int)a.cap[p]);
        j.len = j.L - j.off;
        j.suffix = cw;
    } else {
        // SRTCPCryptoContext.processPacketAESF8 :267-298: IV = 0^4 || (index |
        // E)_be || header[0..7]; ciphers [8, 8 + length - 4 - tag) of the length
        // at the call (protect: before the trailer; unprotect: after shrinking it)
        j.suffix = cw | 0x80000000u;
        j.iv[0] = 0u; j.iv[1] = bswap(j.suffix); j.iv[2] = hdr.x; j.iv[3] = hdr.y;
        j.L = (int)a.len[p] - (a.reverse ? 0 : 4 + T);
        j.off = 8;
        j.len = j.L - 4 - T;
    }
    return j;
}

// XOR keystream block S into job bytes [off + 16 jb, ...) within its region.
__device__ __forceinline__ void f8_xor_block(const F8Job &j, int jb, const uint32_t S[4]) {
    const int end = j.off + j.len;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int pos = j.off + 16 * jb + 4 * k;
        if (pos < end) {
            const int rem = end - pos;
            const uint32_t m = rem >= 4 ? ~0u : ((1u << (8 * rem)) - 1u);
            uint32_t *w = reinterpret_cast<uint32_t *>(j.pkt + pos);
            *w ^= S[k] & m;
        }
    }
}

// Running HMAC-SHA1 inner hash of one packet, fed 64-B blocks as soon as
// they are final (protect: once the F8 pass has ciphered them).
struct F8Mac {
    uint32_t h[5];
    int next;   // next inner block to hash
};

// Hash the packet's inner blocks that lie wholly below byte `upto` (all of
// them for upto = INT_MAX): the data [0, L) || suffix || padding of
// authenticatePacketHMAC :269-278.
__device__ void f8_mac_advance(const F8Job &j, F8Mac &m, int upto) {
    const int nb_data = (j.L + 63) >> 6;
    const int nb_inner = ((j.L + 12) >> 6) + 1;
    while (m.next < nb_inner && (upto == 0x7fffffff || 64 * m.next + 64 <= upto)) {
        const int b = m.next;
        uint32_t w[16];
        const uint4 *qp = reinterpret_cast<const uint4 *>(j.pkt + 64 * b);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint4 v = make_uint4(0, 0, 0, 0);
            if (b < nb_data && 64 * b + 16 * q < j.L) v = qp[q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        inner_words(w, b, j.L, j.suffix);
        sha1_compress(m.h, w);
        m.next++;
    }
}

// SRTPCipherF8.process :97-128 + processBlock :145-183 for two packets of one
// key set at once (the second may be absent: has1 false), so both blocks of
// the two-block AES round code do useful work: IV' = E(k_e ^ (k_s || 0x55..),
// IV), then S(j) = E(k_e, IV' ^ S(j-1) ^ j), S(-1) = 0, j big-endian in bytes
// 12..15, XORed over each packet's region.  With `mac` (protect) each packet's
// HMAC inner hash follows the ciphering block by block (the MAC is over the
// ciphertext), so the packet is read once more only from L1/L2.
template <class Cipher>
__device__ __forceinline__ void f8_pair(const Cipher &cipher, const KeySet *ks, const uint32_t ivp0[4],
                        const uint32_t ivp1[4], const F8Job &j0, const F8Job &j1, bool has1, bool mac,
                        F8Mac &m0, F8Mac &m1) {
    uint32_t p0[4], p1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) { p0[k] = ivp0[k]; p1[k] = has1 ? ivp1[k] : 0u; }
    if (mac) {
#pragma unroll
        for (int k = 0; k < 5; k++) m0.h[k] = m1.h[k] = sgpr(ks->ipad[k]);
        m0.next = m1.next = 0;
        // the header before the ciphered region is final from the start
        f8_mac_advance(j0, m0, j0.off);
        if (has1) f8_mac_advance(j1, m1, j1.off);
    }
    const int n0 = j0.len > 0 ? (j0.len + 15) >> 4 : 0;
    const int n1 = has1 && j1.len > 0 ? (j1.len + 15) >> 4 : 0;
    const int nb = max(n0, n1);
    uint32_t s0[4] = {0u, 0u, 0u, 0u}, s1[4] = {0u, 0u, 0u, 0u};
    for (int jb = 0; jb < nb; jb++) {
        uint32_t x[4], y[4];
#pragma unroll
        for (int k = 0; k < 4; k++) { x[k] = s0[k] ^ p0[k]; y[k] = s1[k] ^ p1[k]; }
        x[3] ^= bswap((uint32_t)jb);
        y[3] ^= bswap((uint32_t)jb);
        cipher.encrypt2(x, y);
#pragma unroll
        for (int k = 0; k < 4; k++) { s0[k] = x[k]; s1[k] = y[k]; }
        if (jb < n0) {
            f8_xor_block(j0, jb, s0);
            if (mac && jb + 1 < n0) f8_mac_advance(j0, m0, j0.off + 16 * (jb + 1));
        }
        if (jb < n1) {
            f8_xor_block(j1, jb, s1);
            if (mac && jb + 1 < n1) f8_mac_advance(j1, m1, j1.off + 16 * (jb + 1));
        }
    }
    if (mac) { // everything after the region is final: the remaining inner blocks
        f8_mac_advance(j0, m0, 0x7fffffff);
        if (has1) f8_mac_advance(j1, m1, 0x7fffffff);
    }
}

// Protect's trailer after the F8 pass: outer HMAC block, then the tag (SRTP)
// or E|index + tag (SRTCP; the policy check guarantees an HMAC trailer there).
__device__ __forceinline__ void f8_trailer(const KeySet *ks, const F8Job &j, F8Mac &m) {
    if (sgpr(ks->auth_type) == SRTP_NULL_AUTHENTICATION) return;
    const int T = (int)sgpr(ks->tag_len);
    uint32_t w[16];
    outer_words(w, m.h, ks);
    sha1_compress(m.h, w);
    int o = j.L;
    if (j.rtcp) {
        j.pkt[o] = (uint8_t)(j.suffix >> 24); j.pkt[o + 1] = (uint8_t)(j.suffix >> 16);
        j.pkt[o + 2] = (uint8_t)(j.suffix >> 8); j.pkt[o + 3] = (uint8_t)j.suffix;
        o += 4;
    }
    tag_write(m.h, j.pkt + o, T);
}

// ------------------------------------------------------------- AES-256-CM
// SRTPCipherCTR with a 32-byte session key (RFC 6188; BouncyCastle's AES engine
// runs 14 rounds for it): the same counter blocks as AES-128-CM, so a lane takes
// one packet and ciphers two blocks at a time; protect feeds the HMAC inner hash
// as the blocks become final, then writes the trailer, as for F8.
struct RoundKeys256 {
    uint32_t k[60];
};

__device__ __forceinline__ void load_rk256_uniform(const uint32_t *__restrict__ p, RoundKeys256 &rk) {
    const uint4 *q = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int i = 0; i < 15; i++) {
        const uint4 v = q[i];
        rk.k[4 * i] = sgpr(v.x); rk.k[4 * i + 1] = sgpr(v.y);
        rk.k[4 * i + 2] = sgpr(v.z); rk.k[4 * i + 3] = sgpr(v.w);
    }
}

__device__ __forceinline__ void aes256_encrypt2(const char *__restrict__ lds, const TeBase &tb,
                                                const RoundKeys256 &rk, uint32_t a[4], uint32_t b[4]) {
#pragma unroll
    for (int j = 0; j < 4; j++) { a[j] ^= rk.k[j]; b[j] ^= rk.k[j]; }
#pragma unroll
    for (int r = 1; r < 14; r++) aes_round2(lds, tb, rk.k + 4 * r, a, b);
    aes_last2(lds, tb, rk.k + 56, a, b);
}

// One AES-256-CM packet's job: the CTR IV and the ciphered region [off, L) --
// protect: the packet before its trailer; unprotect: after the final shrink
// (SRTPCryptoContext.processPacketAESCM :491-530, SRTCPCryptoContext :236-265).
__device__ __forceinline__ F8Job cm_job(const BundleArgs &a, const KeySet *ks, uint32_t p) {
    F8Job j;
    j.pkt = a.seg + a.off[p];
    const uint4 hdr = *reinterpret_cast<const uint4 *>(j.pkt);
    const int T = (int)sgpr(ks->tag_len);
    const bool mac = sgpr(ks->auth_type) != SRTP_NULL_AUTHENTICATION;
    const uint32_t cw = a.w_cw[p];
    j.rtcp = sgpr(ks->kind) == SRTP_KIND_RTCP;
    if (!j.rtcp) {
        make_iv_rtp(ks, hdr, cw, j.iv);
        j.L = (int)a.len[p] - (!a.reverse && mac ? T : 0);
        j.off = rtp_header_len(j.pkt, hdr.x & 0xffu, (int)a.cap[p]);
        j.suffix = cw;
    } else {
        make_iv_rtcp(ks, hdr, cw & 0x7FFFFFFFu, j.iv);
        j.L = (int)a.len[p] - (!a.reverse && mac ? 4 + T : 0);
        j.off = 8;
        j.suffix = (cw & 0x7FFFFFFFu) | 0x80000000u;
    }
    j.len = j.L - j.off;
    return j;
}

template <class Cipher>
__device__ __forceinline__ void cm_one(const Cipher &cipher, const KeySet *ks, const F8Job &j, bool mac) {
    F8Mac m;
    if (mac) {
#pragma unroll
        for (int k = 0; k < 5; k++) m.h[k] = sgpr(ks->ipad[k]);
        m.next = 0;
        f8_mac_advance(j, m, j.off);
    }
    const int nb = j.len > 0 ? (j.len + 15) >> 4 : 0;
    for (int jb = 0; jb < nb; jb += 2) {
        uint32_t x[4], y[4];
        ctr_input(j.iv, jb, x);
        ctr_input(j.iv, jb + 1, y);
        cipher.encrypt2(x, y);
        f8_xor_block(j, jb, x);
        if (jb + 1 < nb) f8_xor_block(j, jb + 1, y);
        if (mac) f8_mac_advance(j, m, j.off + 16 * min(jb + 2, nb));
    }
    if (mac) {
        f8_mac_advance(j, m, 0x7fffffff);
        f8_trailer(ks, j, m);
    }
}

// ------------------------------------------------------- block ciphers of k_ext
// Two blocks per call (the two-block AES round code, or two interleaved
// Twofish chains).
// The AES round keys are (re)loaded into SGPRs by each call -- scalar loads
// of one key set, cheap next to two blocks of rounds -- so no key array stays
// live across a packet's chain.
struct Aes128Cipher {
    const char *lds;
    TeBase tb;
    const uint32_t *rk; // 44 words, wave-uniform
    __device__ __forceinline__ void encrypt2(uint32_t a[4], uint32_t b[4]) const {
        RoundKeys r;
        load_rk_uniform(rk, r);
        aes_encrypt2(lds, tb, r, a, b);
    }
};
struct Aes256Cipher {
    const char *lds;
    TeBase tb;
    const uint32_t *rk; // 60 words, wave-uniform
    __device__ __forceinline__ void encrypt2(uint32_t a[4], uint32_t b[4]) const {
        RoundKeys256 r;
        load_rk256_uniform(rk, r);
        aes256_encrypt2(lds, tb, r, a, b);
    }
};

// AES-256 (14 rounds), or AES-128 for a Skein key set's AES-128-CM (the
// fused kernels' path is HMAC-only); wave-uniform choice.
struct AesCmCipher {
    const char *lds;
    TeBase tb;
    const uint32_t *rk;
    bool a256;
    __device__ __forceinline__ void encrypt2(uint32_t a[4], uint32_t b[4]) const {
        if (a256) {
            RoundKeys256 r;
            load_rk256_uniform(rk, r);
            aes256_encrypt2(lds, tb, r, a, b);
        } else {
            RoundKeys r;
            load_rk_uniform(rk, r);
            aes_encrypt2(lds, tb, r, a, b);
        }
    }
};

// Twofish (Schneier et al. 1998, 4.1-4.3) with the key schedule's g() tables
// read from HBM through the caches (4 KB per key, the same for the whole key
// set); the words are little-endian, like the AES state words.
struct TwofishCipher {
    const TwofishKeys *k;
    __device__ __forceinline__ uint32_t g(uint32_t x) const {
        const uint32_t *T = &k->T[0][0];
        return T[x & 255u] ^ T[256u + ((x >> 8) & 255u)] ^ T[512u + ((x >> 16) & 255u)] ^
               T[768u + (x >> 24)];
    }
    __device__ __forceinline__ void encrypt2(uint32_t a[4], uint32_t b[4]) const {
        const uint32_t *K = k->K;
#pragma unroll
        for (int i = 0; i < 4; i++) { a[i] ^= K[i]; b[i] ^= K[i]; }
#pragma unroll 2
        for (int r = 0; r < 16; r++) {
            const uint32_t ka = K[2 * r + 8], kb = K[2 * r + 9];
            const uint32_t ta0 = g(a[0]), ta1 = g(rotl(a[1], 8u));
            const uint32_t tb0 = g(b[0]), tb1 = g(rotl(b[1], 8u));
            const uint32_t na0 = rotl(a[2] ^ (ta0 + ta1 + ka), 31u);
            const uint32_t na1 = rotl(a[3], 1u) ^ (ta0 + 2u * ta1 + kb);
            const uint32_t nb0 = rotl(b[2] ^ (tb0 + tb1 + ka), 31u);
            const uint32_t nb1 = rotl(b[3], 1u) ^ (tb0 + 2u * tb1 + kb);
            a[2] = a[0]; a[3] = a[1]; a[0] = na0; a[1] = na1;
            b[2] = b[0]; b[3] = b[1]; b[0] = nb0; b[1] = nb1;
        }
        const uint32_t oa[4] = {a[2] ^ K[4], a[3] ^ K[5], a[0] ^ K[6], a[1] ^ K[7]};
        const uint32_t ob[4] = {b[2] ^ K[4], b[3] ^ K[5], b[0] ^ K[6], b[1] ^ K[7]};
#pragma unroll
        for (int i = 0; i < 4; i++) { a[i] = oa[i]; b[i] = ob[i]; }
    }
};

// This packet needs k_ext: final status OK, an ext key set, and for unprotect
// decryption is due (SRTP: no DISCARD/SILENCE flag; SRTCP: the E flag).
__device__ __forceinline__ bool ext_todo(const BundleArgs &a, uint32_t p, uint32_t *ks_id) {
    if (p >= a.n || a.status[p] != SRTP_STATUS_OK) return false;
    const uint32_t slot = a.p_slot[p];
    if (slot == kNoSlot) return false;
    *ks_id = a.ctx[slot].ks;
    const KeySet *ks = a.keysets + *ks_id;
    if (!ks->ext) return false;
    if (ks->enc_type == SRTP_NULL_ENCRYPTION) return false; // NULL cipher + Skein: k_skein only
    if (!a.reverse) return true;
    if (ks->kind == SRTP_KIND_RTP)
        return !((a.flags ? a.flags[p] : 0u) & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE));
    return (a.w_cw[p] & 0x80000000u) != 0;
}

// ============================================================== k_ext
// AES-F8 packets (SRTPCipherF8; SDES F8_128_HMAC_SHA1_80), after the final
// statuses of k_protect / k_unprotect_fix.  Protect: F8 encryption, then the
// HMAC over the ciphertext and the trailer.  Unprotect: k_unprotect already
// checked the tag (HMAC is over the ciphertext, independent of the cipher) and
// did not speculate, so only the accepted packets are deciphered here.  The F8
// keystream is a chain, so a lane walks packets block by block -- two packets
// per lane (2g, 2g+1) through the two-block AES rounds when they share a key
// set (packets of one transformer usually sit side by side), else one by one.
constexpr int kExtBlock = 512; // two packets per lane: 1024 packets per workgroup, one per CU

// One key set's packets in k_ext: j0 (and j1 when has1, the lane's pair).
__device__ __forceinline__ void ext_keyset(const BundleArgs &a, const char *__restrict__ lds, const TeBase &tb,
                           uint32_t ks_u, uint32_t q0, uint32_t q1, bool has1) {
    const KeySet *ks = a.keysets + ks_u;
    const int enc = (int)sgpr(ks->enc_type);
    const int auth = (int)sgpr(ks->auth_type);
    // HMAC fed as the blocks are ciphered; a Skein key set's trailer is
    // k_skein's, after this pass
    const bool mac = !a.reverse && auth == SRTP_HMACSHA1_AUTHENTICATION;
    if (enc == SRTP_AESCM_ENCRYPTION || enc == SRTP_TWOFISH_ENCRYPTION) { // counter mode
        const F8Job j0 = cm_job(a, ks, q0);
        if (enc == SRTP_AESCM_ENCRYPTION) { // AES-256-CM, or AES-128-CM of a Skein key set
            const bool a256 = sgpr(a.extkeys[ks_u].nr) == 14;
            const AesCmCipher c{lds, tb, a256 ? a.extkeys[ks_u].rk : ks->rk, a256};
            cm_one(c, ks, j0, mac);
            if (has1) cm_one(c, ks, cm_job(a, ks, q1), mac);
        } else {
            const TwofishCipher c{a.tfkeys + 2 * (size_t)ks_u};
            cm_one(c, ks, j0, mac);
            if (has1) cm_one(c, ks, cm_job(a, ks, q1), mac);
        }
        return;
    }
    // F8: IV' = E(k_e ^ (k_s || 0x55..), IV), then the chain under k_e
    const F8Job j0 = f8_job(a, ks, q0);
    F8Job j1 = j0;
    if (has1) j1 = f8_job(a, ks, q1);
    uint32_t p0[4], p1[4];
#pragma unroll
    for (int k = 0; k < 4; k++) { p0[k] = j0.iv[k]; p1[k] = has1 ? j1.iv[k] : 0u; }
    F8Mac m0, m1;
    if (enc == SRTP_AESF8_ENCRYPTION) {
        const Aes128Cipher ivc{lds, tb, a.extkeys[ks_u].rk};
        ivc.encrypt2(p0, p1);
        const Aes128Cipher c{lds, tb, ks->rk};
        f8_pair(c, ks, p0, p1, j0, j1, has1, mac, m0, m1);
    } else { // TWOFISHF8_ENCRYPTION
        const TwofishCipher ivc{a.tfkeys + 2 * (size_t)ks_u + 1};
        ivc.encrypt2(p0, p1);
        const TwofishCipher c{a.tfkeys + 2 * (size_t)ks_u};
        f8_pair(c, ks, p0, p1, j0, j1, has1, mac, m0, m1);
    }
    if (mac) {
        f8_trailer(ks, j0, m0);
        if (has1) f8_trailer(ks, j1, m1);
    }
}

__global__ __launch_bounds__(kExtBlock) void k_ext(BundleArgs a) {
    __shared__ uint32_t s_te[kTeWords];
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t q0 = 2 * g, q1 = 2 * g + 1;
    uint32_t k0 = 0, k1 = 0;
    const bool t0 = ext_todo(a, q0, &k0), t1 = ext_todo(a, q1, &k1);
    if (!__syncthreads_or(t0 || t1)) return;
    fill_te4(s_te);
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s_te);
    const bool pair = t0 && t1 && k0 == k1;
    const bool one0 = t0 && !pair, one1 = t1 && !pair;
    // pairs, and lone first packets (which take their key set's pass)
    for_each_keyset(pair || one0, t0 ? k0 : k1, [&](uint32_t ks_u) {
        ext_keyset(a, lds, tb, ks_u, pair || one0 ? q0 : q1, q1, pair);
    });
    for_each_keyset(one1, k1, [&](uint32_t ks_u) { // lone second packets
        ext_keyset(a, lds, tb, ks_u, q1, q1, false);
    });
}

// ============================================================== k_skein
// Skein-MAC key sets (engines that have them).  Unprotect, after k_unprotect
// (which set each packet's ROC guess g0, and left these packets in place):
// the tag check under g0 (SRTP) or of the packet and its E|index trailer
// (SRTCP), as authenticatePacket :237-266 / SRTCPCryptoContext :333-353 do
// with SkeinMac; the walk re-checks an SRTP tag whose ROC it guesses
// differently.  Protect, after k_ext ciphered them (final statuses): the
// trailer -- SRTCP's E|index word first (the MAC covers it; the NULL cipher
// writes index 0, transformPacket :391-427), then the tag.
constexpr int kSkeinBlock = 256;

__global__ __launch_bounds__(kSkeinBlock) void k_skein(BundleArgs a) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    bool todo = false;
    uint32_t ks_id = 0u;
    if (p < a.n && (a.reverse || a.status[p] == SRTP_STATUS_OK)) {
        const uint32_t slot = a.p_slot[p];
        if (slot != kNoSlot) {
            ks_id = a.ctx[slot].ks;
            todo = a.keysets[ks_id].auth_type == SRTP_SKEIN_AUTHENTICATION;
        }
    }
    for_each_keyset(todo, ks_id, [&](uint32_t ks_u) {
        const KeySet *ks = a.keysets + ks_u;
        const int T = (int)sgpr(ks->tag_len);
        const bool rtp = sgpr(ks->kind) == SRTP_KIND_RTP;
        uint8_t *pkt = a.seg + a.off[p];
        const int L = (int)a.len[p]; // unprotect: as received; protect: final, with the trailer
        int end, tag_at;
        uint32_t suffix;
        if (a.reverse) {
            if (rtp) {
                end = L - T > 0 ? L - T : 0;
                suffix = a.gok[2 * (size_t)(p)];
            } else {
                end = L - 4 - T;
                if (end < 0) return; // the reference throws here (k_walk)
                suffix = ld_be32(pkt + end);
            }
            tag_at = L - T;
        } else {
            const uint32_t cw = a.w_cw[p];
            if (rtp) {
                end = L - T;
                suffix = cw;
            } else {
                end = L - 4 - T;
                suffix = sgpr(ks->enc_type) != SRTP_NULL_ENCRYPTION ? ((cw & 0x7FFFFFFFu) | 0x80000000u) : 0u;
                pkt[end] = (uint8_t)(suffix >> 24); pkt[end + 1] = (uint8_t)(suffix >> 16);
                pkt[end + 2] = (uint8_t)(suffix >> 8); pkt[end + 3] = (uint8_t)suffix;
            }
            tag_at = L - T;
        }
        uint32_t tag[5];
        skein_mac<true>(a.skkeys + ks_u, pkt, end, suffix, tag);
        if (a.reverse) a.gok[2 * (size_t)(p) + 1] = tag_matches(tag, pkt + tag_at, T) ? 1u : 0u;
        else tag_write(tag, pkt + tag_at, T);
    });
}

// ============================================================== maintenance
__global__ void k_remove_transformer(uint64_t *keys, CtxState *ctx, uint32_t cap, uint32_t tid) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    uint64_t k = keys[i];
    if (k != kEmptyKey && k != kTombKey && (uint32_t)(k >> 32) == tid) {
        keys[i] = kTombKey;
        CtxState z = {};
        ctx[i] = z;
    }
}

// Context save / restore by key (srtp_contexts_save / _restore: the
// dispatcher's rollback of a transformer whose packets ran past a throw on
// another shard).  Restore keys are distinct, so concurrent inserts only race
// with each other the way k_parse's do (ctx_lookup_insert).
__global__ void k_ctx_save(const uint64_t *tab, const CtxState *ctx, uint32_t mask, const uint64_t *keys,
                           uint32_t n, CtxState *out, int32_t *present) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = keys[i];
    uint32_t h = (uint32_t)mix64(key) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        const uint64_t cur = tab[h];
        if (cur == key) {
            out[i] = ctx[h];
            present[i] = 1;
            return;
        }
        if (cur == kEmptyKey) break;
    }
    out[i] = CtxState{};
    present[i] = 0;
}

__global__ void k_ctx_restore(uint64_t *tab, CtxState *ctx, uint32_t mask, const uint64_t *keys, uint32_t n,
                              const CtxState *in, const int32_t *present, unsigned int *failed) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    BundleArgs a{};
    a.ctx_keys = tab;
    a.ctx = ctx;
    a.ctx_mask = mask;
    const CtxState st = in[i];
    bool created = false;
    const uint32_t slot = ctx_lookup_insert(a, keys[i], present[i] != 0, st.ks, &created);
    if (present[i]) {
        if (slot == kNoSlot) atomicAdd(failed, 1u);
        else ctx[slot] = st;
    } else if (slot != kNoSlot) {
        __hip_atomic_store(&tab[slot], kTombKey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ctx[slot] = CtxState{};
    }
}

__global__ void k_count_contexts(const uint64_t *keys, uint32_t cap, unsigned long long *out) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t k = i < cap ? keys[i] : kEmptyKey;
    const unsigned long long live = __ballot(k != kEmptyKey && k != kTombKey);
    const unsigned long long tomb = __ballot(k == kTombKey);
    if ((threadIdx.x & 63) == 0) {
        if (live) atomicAdd(&out[0], (unsigned long long)__popcll(live));
        if (tomb) atomicAdd(&out[1], (unsigned long long)__popcll(tomb));
    }
}

__global__ void k_rehash_collect(const uint64_t *keys, const CtxState *ctx, uint32_t cap,
                                 uint64_t *tmp_keys, CtxState *tmp_ctx, unsigned long long *n_live) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cap) return;
    const uint64_t k = keys[i];
    if (k == kEmptyKey || k == kTombKey) return;
    const unsigned long long j = atomicAdd(n_live, 1ull);
    tmp_keys[j] = k;
    tmp_ctx[j] = ctx[i];
}

__global__ void k_rehash_insert(uint64_t *keys, CtxState *ctx, uint32_t mask,
                                const uint64_t *tmp_keys, const CtxState *tmp_ctx, uint32_t n) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t key = tmp_keys[j];
    uint32_t h = (uint32_t)mix64(key) & mask;
    // the table holds fewer live keys than slots: an empty slot exists
    for (uint32_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        const unsigned long long prev = atomicCAS((unsigned long long *)&keys[h],
                                                  (unsigned long long)kEmptyKey,
                                                  (unsigned long long)key);
        if (prev == kEmptyKey) {
            ctx[h] = tmp_ctx[j];
            return;
        }
    }
}

// ============================================================== launchers
static inline dim3 grid_for(uint32_t n) { return dim3((n + kBlock - 1) / kBlock); }

hipError_t launch_parse(const BundleArgs &a, hipStream_t s) {
    if (a.sort_bits > 8)
        hipLaunchKernelGGL(k_parse<1 << kSortWideMaxBits>, dim3((a.n + kParseBlock - 1) / kParseBlock),
                           dim3(kParseBlock), 0, s, a);
    else
        hipLaunchKernelGGL(k_parse<256>, dim3((a.n + kParseBlock - 1) / kParseBlock), dim3(kParseBlock), 0, s, a);
    return hipGetLastError();
}
// Workgroup size of the AES kernels for a bundle of n packets.  A workgroup
// holds the 128-KB T-table image, so a CU runs one at a time, and its waves
// share the CU's four SIMDs: 16 waves per CU give the best throughput on a
// full bundle, but a small bundle (the per-packet path's, an aggregator lane's)
// packed 16 waves to a CU finishes in the time of its few busy CUs while the
// rest idle.  So the waves are spread over every CU, at least 4 per
// workgroup (one per SIMD: the image is filled by the workgroup's threads)
// and at most max_block / 64.  A full bundle (2^18 packets = 16 waves per CU)
// keeps 1024-thread workgroups (profiles/r04/kernel_experiments.md 5).
static uint32_t aes_block(uint32_t n, uint32_t max_block) {
    static std::atomic<int> cus[64]; // CUs per device, looked up once (any thread)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return max_block;
    int c = cus[dev].load(std::memory_order_relaxed);
    if (c <= 0) {
        if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) return max_block;
        cus[dev].store(c, std::memory_order_relaxed);
    }
    const uint32_t waves = (n + 63u) / 64u, per_cu = (waves + (uint32_t)c - 1u) / (uint32_t)c;
    return 64u * std::min<uint32_t>(max_block / 64u, std::max<uint32_t>(4u, per_cu));
}

hipError_t launch_unprotect(const BundleArgs &a, hipStream_t s) {
    const uint32_t b = aes_block(a.n, (uint32_t)kUnprotectBlock);
    if (a.small_ctr) {
        const uint32_t bm = std::min<uint32_t>(b, (uint32_t)kMacBlock);
        hipLaunchKernelGGL(k_unprotect<true>, dim3((a.n + bm - 1) / bm), dim3(bm), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_unprotect<false>, dim3((a.n + b - 1) / b), dim3(b), 0, s, a);
    }
    return hipGetLastError();
}
hipError_t launch_skein(const BundleArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_skein, dim3((a.n + kSkeinBlock - 1) / kSkeinBlock), dim3(kSkeinBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_walk(const BundleArgs &a, int limit_pass, hipStream_t s) {
    const uint32_t spans = (a.n + kWalkSpan - 1) / kWalkSpan;
    const dim3 grid(spans);
    if (a.reverse && a.has_skein) {
        if (limit_pass) hipLaunchKernelGGL((k_walk<true, true, 1>), grid, dim3(kWalkBlock), 0, s, a);
        else hipLaunchKernelGGL((k_walk<true, true, 0>), grid, dim3(kWalkBlock), 0, s, a);
    } else if (a.reverse) {
        if (limit_pass) hipLaunchKernelGGL((k_walk<true, false, 1>), grid, dim3(kWalkBlock), 0, s, a);
        else hipLaunchKernelGGL((k_walk<true, false, 0>), grid, dim3(kWalkBlock), 0, s, a);
    } else {
        if (limit_pass) hipLaunchKernelGGL((k_walk<false, false, 1>), grid, dim3(kWalkBlock), 0, s, a);
        else hipLaunchKernelGGL((k_walk<false, false, 0>), grid, dim3(kWalkBlock), 0, s, a);
    }
    return hipGetLastError();
}
// ------------------------------------------------ small bundles' AES-CM
// In a bundle of a few waves the fused kernels are one lane walking each
// packet's chunks with every LDS latency exposed (~100 us for a lone 1200-B
// packet: most of a per-packet call's round trip).  With BundleArgs::small_ctr
// this kernel applies the keystream of the AES-CM + HMAC-SHA1 packets instead,
// one wave per packet and a lane per pair of counter blocks, and the
// fused kernels only MAC them: protect runs it before k_protect (which MACs
// the ciphertext and appends the trailer), unprotect after k_unprotect (which
// MACs the ciphertext, checks the tag, saves the walk's re-check state and
// marks the packets it speculates on, kSpecDid) and before the walk -- the
// same bytes, in the same order, as the fused kernels leave.
constexpr int kCtrSmallBlock = 256;

__device__ __forceinline__ bool small_ctr_ks(const KeySet *ks) {
    // the three fields loaded together (no short-circuit chain of loads)
    const int32_t ext = ks->ext, enc = ks->enc_type, auth = ks->auth_type;
    return (ext == 0) & (enc == SRTP_AESCM_ENCRYPTION) & (auth == SRTP_HMACSHA1_AUTHENTICATION);
}

// finish_status without its stores (k_protect makes them)
__device__ __forceinline__ int32_t peek_status(const BundleArgs &a, uint32_t p) {
    int32_t st = a.w_status[p];
    if (st == kStPending) st = SRTP_STATUS_ERR_INTERNAL;
    if (st != SRTP_STATUS_SKIPPED && a.abort_on_error && a.ctl->any_throw &&
        (int32_t)p > a.e_min[packet_tid(a, p)])
        st = SRTP_STATUS_NOT_PROCESSED;
    return st;
}

// packet p's keystream job: [start, end) under iv with key set ks, or false.
// The per-packet words are loaded together up front (one memory round trip,
// not one per test), then the context's key set and the packet header.
__device__ __forceinline__ bool ctr_small_job(const BundleArgs &a, uint32_t p, int &start, int &end,
                                              uint32_t iv[4], const KeySet *&ks) {
    const uint32_t slot = a.p_slot[p];
    const uint32_t o = a.off[p], cap = a.cap[p];
    const uint32_t L = a.reverse ? a.len[p] : a.w_len[p];
    const uint32_t cw = a.reverse ? a.gok[2 * (size_t)(p)] : a.w_cw[p];
    const uint32_t sp = a.reverse ? a.spec[p] : 0u;
    if (slot == kNoSlot) return false;
    if (a.reverse && !(sp & kSpecDid)) return false; // k_unprotect did not speculate
    if (!a.reverse && peek_status(a, p) != SRTP_STATUS_OK) return false;
    ks = a.keysets + a.ctx[slot].ks;
    const uint8_t *pkt = a.seg + o;
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    if (!small_ctr_ks(ks)) return false;
    const bool rtcp = ks->kind == SRTP_KIND_RTCP;
    const int T = ks->tag_len;
    if (!a.reverse) { // protect_one's region and IV
        end = (int)L - T - (rtcp ? 4 : 0);
        if (rtcp) {
            start = 8;
            make_iv_rtcp(ks, hdr, cw, iv);
        } else {
            start = rtp_header_len(pkt, hdr.x & 0xffu, (int)cap);
            make_iv_rtp(ks, hdr, cw, iv);
        }
    } else { // unprotect_one's speculative decryption
        if (rtcp) {
            const int io = (int)L - 4 - T;
            start = 8;
            end = io;
            make_iv_rtcp(ks, hdr, ld_be32(pkt + io) & 0x7FFFFFFFu, iv);
        } else {
            start = rtp_header_len(pkt, hdr.x & 0xffu, (int)cap);
            end = (int)L - T;
            make_iv_rtp(ks, hdr, cw, iv);
        }
    }
    return end > start;
}

// XOR keystream block x over up to 16 bytes (lim) at dst
__device__ __forceinline__ void xor_ks16(uint8_t *dst, int lim, const uint32_t x[4]) {
#pragma unroll
    for (int i = 0; i < 16; i++)
        if (i < lim) dst[i] ^= (uint8_t)(x[i >> 2] >> (8 * (i & 3)));
}

// XOR keystream blocks x, y over the 32 bytes at pkt + o, up to end: o is a
// multiple of 4 (a 16-B aligned packet, a header of whole words), so the two
// blocks are eight words -- all eight loaded before any store, the bytes of
// the last word past end XORed with zero (only this lane touches that word
// in this kernel)
__device__ __forceinline__ void xor_ks32(uint8_t *pkt, int o, int end, const uint32_t x[4], const uint32_t y[4]) {
    uint32_t *w = reinterpret_cast<uint32_t *>(pkt + o);
    uint32_t v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = o + 4 * i < end ? w[i] : 0u;
    // every result before the first store: one wait for the eight loads, not
    // one per (conditional) store
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const int r = end - (o + 4 * i);
        const uint32_t k = i < 4 ? x[i] : y[i - 4];
        v[i] ^= r >= 4 ? k : (r > 0 ? k & ((1u << (8 * r)) - 1u) : 0u);
    }
    // the compiler sinks the XORs into the conditional stores and then waits
    // for memory before each one: wait once (vmcnt 0) here instead
    __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
    for (int i = 0; i < 8; i++)
        if (o + 4 * i < end) w[i] = v[i];
}

__global__ __launch_bounds__(kCtrSmallBlock) void k_ctr_small(BundleArgs a) {
    __shared__ uint32_t s_te[kTeWords];
    fill_te4(s_te); // ends with a barrier
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s_te);
    // a wave per packet: every lane works out the packet's job (the same loads
    // across the wave), then the lanes take its counter-block pairs
    const uint32_t waves = gridDim.x * (kCtrSmallBlock / 64);
    const int lane = (int)(threadIdx.x & 63u);
    for (uint32_t p = blockIdx.x * (kCtrSmallBlock / 64) + (threadIdx.x >> 6); p < a.n; p += waves) {
        int start = 0, end = 0;
        uint32_t iv[4];
        const KeySet *ks = nullptr;
        if (!ctr_small_job(a, p, start, end, iv, ks)) continue;
        uint32_t k0[4];
#pragma unroll
        for (int k = 0; k < 4; k++) k0[k] = ks->rk[k];
        uint8_t *pkt = a.seg + a.off[p];
        const int nblk = (end - start + 15) >> 4;
        for (int j = 2 * lane; j < nblk; j += 128) {
            uint32_t x[4], y[4];
            ctr_input(iv, j, x);
            ctr_input(iv, j + 1, y);
            aes_encrypt2_v(lds, tb, k0, x, y);
            if ((start & 3) == 0) {
                xor_ks32(pkt, start + 16 * j, end, x, y);
            } else { // not a header of whole words: byte by byte
                xor_ks16(pkt + start + 16 * j, end - (start + 16 * j), x);
                if (j + 1 < nblk) xor_ks16(pkt + start + 16 * (j + 1), end - (start + 16 * (j + 1)), y);
            }
        }
    }
}

hipError_t launch_ctr_small(const BundleArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    // one workgroup per CU at most (each fills the 128-KB T-table image)
    const uint32_t wgs = (a.n + kCtrSmallBlock / 64 - 1) / (kCtrSmallBlock / 64);
    hipLaunchKernelGGL(k_ctr_small, dim3(wgs < 256u ? wgs : 256u), dim3(kCtrSmallBlock), 0, s, a);
    return hipGetLastError();
}

// ====================================================== the split path (wide)
// A bundle larger than k_ctr_small's (BundleArgs::small_ctr == 2, engines whose
// key sets are all AES-CM or NULL cipher with HMAC-SHA1) runs the cipher and
// the MAC as two kernels with nothing in common but the packet bytes:
//   protect:   walk -> k_ctr_wide (keystream)  -> k_mac_wide (MAC, trailer, statuses)
//   unprotect: k_mac_wide (tag check, ROC guess, re-check state) -> walk
//              -> k_ctr_wide (final statuses, decryption of the accepted packets)
// The MAC is over the ciphertext (SRTPCryptoContext.java:237-266 checks it
// before processPacketAESCM :609-627 deciphers), so unprotect deciphers after
// the walk with the walk's ROC: no speculation, nothing to repair.  Neither
// kernel holds AES and SHA-1 state at once: k_ctr_wide is the 128-KB T-table
// image and few registers (LDS-bound), k_mac_wide no LDS and few registers
// (VALU-bound), so one direction's k_mac_wide fills the register file beside
// the other direction's k_ctr_wide on the same CUs.
//
// k_ctr_wide: every wave on its own, over groups of G consecutive packets
// taken from a ticket counter.  The group's first G lanes work out its packet
// jobs (region, counter precompute, key set; unprotect: the final statuses)
// into the wave's LDS slot; then the group's counter-block pairs go to the
// lanes 64 at a time, consecutive pairs to consecutive lanes, so a wave's
// loads and stores cover 2 KB of one packet's payload contiguously (the fused
// kernels' lane-per-packet pattern touches 64 packets per instruction).  No
// workgroup barrier after the T-table fill: a wave waiting on its next jobs'
// loads leaves the LDS to the other fifteen.  The workgroup's LDS is the
// 128-KB image plus 9 KB, so that the other direction's sort and walk still
// fit beside it on the CU.
constexpr int kWideBlock = 1024;
constexpr int kWideGMax = 16;                        // packets per group
constexpr int kWideWaveWords = 8 * kWideGMax + 20;   // jobs [G][8], prefix [G + 1] (16-B aligned slot)
constexpr int kWideOffWave = kTeWords;               // the image stays at LDS 0
constexpr int kWideWords = kWideOffWave + (kWideBlock / 64) * kWideWaveWords;

// Unprotect's job for packet p: its final status (k_unprotect_fix's, which
// this path does not run) and, for an accepted AES-CM packet, the region and
// IV under the walk's ROC / SRTCP index (processPacketAESCM :482-525,
// SRTCPCryptoContext :218-260).
__device__ __forceinline__ bool wide_job_rev(const BundleArgs &a, uint32_t p, uint32_t *s_cnt, int &start,
                                             int &end, uint32_t iv[4], const KeySet *&ks) {
    // every per-packet word first (finish_status stores after its loads)
    const int L0 = (int)a.len[p];
    const uint32_t slot = a.p_slot[p];
    const uint32_t sw = a.spec[p];
    const uint32_t cw = a.w_cw[p];
    const uint32_t o = a.off[p], cap = a.cap[p];
    const int32_t st = finish_status(a, p);
    atomicAdd(&s_cnt[status_counter(a, p, st)], 1u);
    if (slot == kNoSlot || st != SRTP_STATUS_OK || !(sw & kSpecAes)) return false;
    const bool rtp = (sw & kSpecRtp) != 0u;
    if (rtp ? (sw & kSpecSkip) != 0u : !(cw & 0x80000000u)) return false; // DISCARD/SILENCE; SRTCP E clear
    ks = a.keysets + a.ctx[slot].ks;
    const uint8_t *pkt = a.seg + o;
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    const int T = ks->tag_len;
    const bool mac = ks->auth_type != SRTP_NULL_AUTHENTICATION;
    if (rtp) {
        start = rtp_header_len(pkt, hdr.x & 0xffu, (int)cap);
        end = mac ? max(L0 - T, 0) : L0;
        make_iv_rtp(ks, hdr, cw, iv);
    } else {
        start = 8;
        end = mac ? max(L0 - T - 4, 0) : L0;
        make_iv_rtcp(ks, hdr, cw & 0x7FFFFFFFu, iv);
    }
    if (start < 0 || start > end) start = end;
    return end > start;
}

// k_ctr_jobs: each packet's keystream job, one lane per packet (all their
// dependent loads in flight at once across the grid), into the packet's tailc
// scratch, which the split path does not otherwise use: {IV}, {first byte of
// the region in the segment, region length, key set, 0} (length 0: none).
// Unprotect: also every packet's final status and length.
constexpr int kJobBlock = 256;
template <bool REV>
__global__ __launch_bounds__(kJobBlock) void k_ctr_jobs(BundleArgs a) {
    __shared__ uint32_t s_cnt[kTeCounters];
    if (REV) {
        if (threadIdx.x < kTeCounters) s_cnt[threadIdx.x] = 0u;
        __syncthreads();
    }
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < a.n) {
        int start = 0, end = 0;
        uint32_t iv[4] = {0u, 0u, 0u, 0u};
        const KeySet *ks = nullptr;
        const bool ok = REV ? wide_job_rev(a, p, s_cnt, start, end, iv, ks) : ctr_small_job(a, p, start, end, iv, ks);
        uint4 *jp = reinterpret_cast<uint4 *>(a.tailc + 16 * (size_t)p);
        jp[0] = make_uint4(iv[0], iv[1], iv[2], iv[3]);
        jp[1] = ok ? make_uint4(a.off[p] + (uint32_t)start, (uint32_t)(end - start), (uint32_t)(ks - a.keysets), 0u)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
    if (REV) {
        __syncthreads();
        flush_status_counts(a, s_cnt);
    }
}

// k_ctr_wide: wave w of W takes the groups of G consecutive packets w, w + W,
// ... (no ticket: one counter on one address serialised 16k atomics).  The
// group's first G lanes load its jobs (fetched one group ahead), make the
// counter precompute and put {CtrPre, first byte, kb | length << 8, packet}
// in the wave's LDS slot with the pair prefix; then the pairs.
template <bool REV>
__global__ __launch_bounds__(kWideBlock) void k_ctr_wide(BundleArgs a, uint32_t G) {
    __shared__ uint32_t s[kWideWords];
    fill_te4(s); // ends with a barrier
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s);
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t *ws = s + kWideOffWave + (int)(threadIdx.x >> 6) * kWideWaveWords;
    uint32_t *pre = ws + 8 * kWideGMax;
    const uint32_t n_groups = (a.n + G - 1u) / G;
    const uint32_t W = gridDim.x * (kWideBlock / 64);
    uint32_t top = 1u; // binary-search span: the largest power of two <= G
    while (2u * top <= G) top <<= 1;
    const uint4 *J = reinterpret_cast<const uint4 *>(a.tailc);
    uint32_t grp = blockIdx.x * (kWideBlock / 64) + (threadIdx.x >> 6);
    uint4 nj0 = make_uint4(0u, 0u, 0u, 0u), nj1 = nj0;
    if (grp < n_groups && (uint32_t)lane < min(G, a.n - grp * G)) {
        const size_t p = (size_t)grp * G + (uint32_t)lane;
        nj0 = J[4 * p];
        nj1 = J[4 * p + 1];
    }
#pragma unroll 1
    for (; grp < n_groups; grp += W) {
        const uint32_t first = grp * G;
        const uint32_t cnt = min(G, a.n - first);
        const uint4 cj0 = nj0, cj1 = nj1;
        const uint32_t nx = grp + W; // the next group's jobs, landing during this one
        if (nx < n_groups && (uint32_t)lane < min(G, a.n - nx * G)) {
            const size_t p = (size_t)nx * G + (uint32_t)lane;
            nj0 = J[4 * p];
            nj1 = J[4 * p + 1];
        }
        const bool has = (uint32_t)lane < cnt && cj1.y != 0u;
        const unsigned long long m = __ballot(has);
        if (m == 0ull) continue;
        const uint32_t ks0 = (uint32_t)__builtin_amdgcn_readlane((int)cj1.z, __ffsll((long long)m) - 1);
        const bool uni = __ballot(has && cj1.z != ks0) == 0ull;
        RoundKeys rk;
        if (uni) load_round_keys_uniform(a.keysets + ks0, rk);
        const uint32_t np = has ? (((cj1.y + 15u) >> 4) + 1u) >> 1 : 0u;
        if (has) {
            const uint32_t iv[4] = {cj0.x, cj0.y, cj0.z, cj0.w};
            CtrPre cp;
            if (uni) {
                ctr_precompute(lds, tb, rk.k, iv, cp);
            } else {
                uint32_t r12[12];
                const uint4 *q = reinterpret_cast<const uint4 *>(a.keysets[cj1.z].rk);
#pragma unroll
                for (int i = 0; i < 3; i++) {
                    const uint4 v = q[i];
                    r12[4 * i] = v.x; r12[4 * i + 1] = v.y; r12[4 * i + 2] = v.z; r12[4 * i + 3] = v.w;
                }
                ctr_precompute(lds, tb, r12, iv, cp);
            }
            uint4 *jp = reinterpret_cast<uint4 *>(ws + 8 * lane);
            jp[0] = make_uint4(cp.p0, cp.r[0], cp.r[1], cp.r[2]);
            jp[1] = make_uint4(cp.r[3], cj1.x, cp.kb | (cj1.y << 8), first + (uint32_t)lane);
        }
        uint32_t incl = np; // inclusive prefix of the pair counts over the group's lanes
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = (uint32_t)__shfl_up((int)incl, o);
            if (lane >= o) incl += t;
        }
        if ((uint32_t)lane < cnt) pre[lane] = incl - np;
        const uint32_t total = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)incl, 63));
        // the slot was written by this wave's lanes: LDS ops of a wave complete in order
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 1
        for (uint32_t c0 = 0; c0 < total; c0 += 64u) {
            const uint32_t g = c0 + (uint32_t)lane;
            const bool act = g < total;
            // the packet of pair g: the last q with pre[q] <= g (packets
            // without pairs share their successor's prefix and are skipped)
            uint32_t q = 0u;
            for (uint32_t st = top; st; st >>= 1)
                if (q + st < cnt && pre[q + st] <= g) q += st;
            const uint4 *jp = reinterpret_cast<const uint4 *>(ws + 8 * q);
            const uint4 j0w = jp[0], j1w = jp[1];
            CtrPre cp;
            cp.p0 = j0w.x; cp.r[0] = j0w.y; cp.r[1] = j0w.z; cp.r[2] = j0w.w;
            cp.r[3] = j1w.x; cp.kb = j1w.z & 0xffu;
            const int j = act ? 2 * (int)(g - pre[q]) : 0;
            const size_t pj = act ? j1w.w : first; // an idle lane's q may be a stale slot
            // the pair's 32 bytes, loaded before the rounds (their latency hides
            // behind them); the packet's last, partial pair loads after, masked
            uint8_t *dst = a.seg + j1w.y + 16u * (uint32_t)j;
            const int rem = (int)(j1w.z >> 8) - 16 * j;
            const bool whole = act && rem >= 32;
            uint4 d0 = make_uint4(0u, 0u, 0u, 0u), d1 = d0;
            if (whole) {
                d0 = reinterpret_cast<const uint4 *>(dst)[0];
                d1 = reinterpret_cast<const uint4 *>(dst)[1];
            }
            uint32_t x[4], y[4];
            const bool far = __ballot(act && j + 1 >= 256) != 0ull; // IV byte 14 set: full rounds
            if (uni) {
                if (!far) {
                    ctr_first2(lds, tb, cp, j, j + 1, x, y);
#pragma unroll
                    for (int r = 3; r < 10; r++) aes_round2(lds, tb, rk.k + 4 * r, x, y);
                    aes_last2(lds, tb, rk.k + 40, x, y);
                } else {
                    const uint4 ivw = J[4 * pj];
                    const uint32_t iv[4] = {ivw.x, ivw.y, ivw.z, ivw.w};
                    ctr_input(iv, j, x);
                    ctr_input(iv, j + 1, y);
                    aes_encrypt2(lds, tb, rk, x, y);
                }
            } else { // several key sets in the group: each lane on its own schedule
                const uint4 *kq = reinterpret_cast<const uint4 *>(a.keysets[J[4 * pj + 1].z].rk);
                if (!far) {
                    const uint4 k2 = kq[2];
                    ctr_first2(lds, tb, cp, j, j + 1, x, y);
                    uint32_t kk[4] = {k2.x, k2.y, k2.z, k2.w};
#pragma unroll
                    for (int r = 3; r < 10; r++) {
                        key_next(lds, tb, kk, kRcon[r]);
                        aes_round2_asm_v(x, y, tb.b, kk);
                    }
                    key_next(lds, tb, kk, kRcon[10]);
                    aes_last2_asm_v(x, y, tb.b, kk);
                } else {
                    const uint4 k0 = kq[0], ivw = J[4 * pj];
                    const uint32_t iv[4] = {ivw.x, ivw.y, ivw.z, ivw.w};
                    const uint32_t kk[4] = {k0.x, k0.y, k0.z, k0.w};
                    ctr_input(iv, j, x);
                    ctr_input(iv, j + 1, y);
                    aes_encrypt2_v(lds, tb, kk, x, y);
                }
            }
            if (whole) {
                d0.x ^= x[0]; d0.y ^= x[1]; d0.z ^= x[2]; d0.w ^= x[3];
                d1.x ^= y[0]; d1.y ^= y[1]; d1.z ^= y[2]; d1.w ^= y[3];
                reinterpret_cast<uint4 *>(dst)[0] = d0;
                reinterpret_cast<uint4 *>(dst)[1] = d1;
            } else if (act) {
                xor_ks32(dst, 0, rem, x, y);
            }
        }
        // the slot is rewritten by the next group's lanes only after every
        // lane's reads above (the wave's LDS ops complete in order)
    }
}

// k_mac_wide: the HMAC-SHA1 of the split path, one lane per packet (lanes in
// length-class order), no LDS but the status counts, one block of look-ahead
// (other waves hide the rest at this occupancy).  Protect (after k_ctr_wide):
// final status, the MAC over the ciphertext and the trailer, as k_protect's
// MacOnly instance (authenticatePacketHMAC :269-278, RawPacket.append
// :203-220).  Unprotect (before the walk): as k_unprotect's MacOnly instance
// without speculation -- the ROC guess, the tag check under it, the walk's
// re-check midstate.
constexpr int kMacWideBlock = 256;

#ifndef SRTP_MAC_AHEAD
#define SRTP_MAC_AHEAD 1
#endif
__device__ __forceinline__ void mac_stream(const uint8_t *pkt, int end, uint32_t suffix, const KeySet *ks,
                                           uint32_t h[5], uint32_t *mid_out, int mid_b) {
    const int nb_data = (end + 63) >> 6;
    const int nb_inner = ((end + 12) >> 6) + 1;
    const int n_blocks = nb_inner + 1;
#if SRTP_MAC_AHEAD
    uint32_t nx[16];
    load_or_zero16(pkt, 0, nb_data, end, nx);
#endif
#pragma unroll 1
    for (int b = 0; b < n_blocks; b++) {
        uint32_t w[16];
#if SRTP_MAC_AHEAD
#pragma unroll
        for (int m = 0; m < 16; m++) w[m] = nx[m];
        load_or_zero16(pkt, b + 1, nb_data, end, nx);
        asm volatile("" ::: "memory"); // keep the look-ahead (see MacRing::next)
#else
        load_or_zero16(pkt, b, nb_data, end, w); // the other waves hide the load
#endif
        if (b == mid_b && mid_out) {
#pragma unroll
            for (int k = 0; k < 5; k++) mid_out[k] = h[k];
        }
        if (b < nb_inner) inner_words(w, b, end, suffix);
        else outer_words<false>(w, h, ks);
        sha1_compress(h, w);
    }
}

// ------------------------------------------- a packet's HMAC-SHA1 by a wave
// (k_small, which has at most eight packets per workgroup: one per wave.)  A
// lone packet's MAC is its call's longest chain: one lane hashing 20 blocks at
// ~7.5 VALU per round, with the schedule words in the chain and each block's
// load exposed.  Here the wave's lanes first expand the message schedule of up
// to kWaveMacBlocks blocks at once (lane b: block b's W[t] + K_t, t < 80, into
// a row of the wave's LDS), and lane 0 then compresses the rows: five VALU per
// round (e + W + K, f, rotl(a, 5), the three-way add, rotl(b, 30)) and one
// 16-B LDS read per four rounds.
constexpr int kWaveMacBlocks = 32;  // blocks per schedule chunk
constexpr int kWaveMacStride = 84;  // words per row: 80, padded to 16-B rows (4-way bank conflicts on the writes)
constexpr int kWaveMacWords = kWaveMacBlocks * kWaveMacStride;

__device__ __forceinline__ uint32_t sha1_k(int t) {
    return t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
}

// one block's W[t] + K_t (t < 80) into row
__device__ __forceinline__ void sha1_schedule_row(uint32_t w[16], uint32_t *row) {
#pragma unroll
    for (int t = 0; t < 80; t += 4) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int tt = t + u;
            uint32_t wt;
            if (tt < 16) {
                wt = w[tt];
            } else {
                wt = rotl(xor3(w[(tt - 3) & 15], w[(tt - 8) & 15], w[(tt - 14) & 15]) ^ w[tt & 15], 1);
                w[tt & 15] = wt;
            }
            v[u] = wt + sha1_k(tt);
        }
        *reinterpret_cast<uint4 *>(row + t) = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// sha1_compress with the schedule (+ K) read from a row
__device__ __forceinline__ void sha1_compress_kw(uint32_t h[5], const uint32_t *row) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; t += 4) {
        const uint4 q = *reinterpret_cast<const uint4 *>(row + t);
        const uint32_t kw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int tt = t + u;
            uint32_t f;
            if (tt < 20) f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
            else if (tt < 40) f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
            else if (tt < 60) f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
            else f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
            const uint32_t tmp = rotl(a, 5) + f + (e + kw[u]);
            e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
        }
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// mac_stream by the calling wave (every lane the same packet); h is the
// final HMAC state in lane 0.  sched: the wave's kWaveMacWords of LDS.
__device__ __forceinline__ void mac_wave(const uint8_t *pkt, int end, uint32_t suffix, const KeySet *ks,
                                         uint32_t h[5], uint32_t *mid_out, int mid_b, uint32_t *sched) {
    const int lane = (int)(threadIdx.x & 63u);
    const int nb_data = (end + 63) >> 6;
    const int nb_inner = ((end + 12) >> 6) + 1;
#pragma unroll 1
    for (int b0 = 0; b0 < nb_inner; b0 += kWaveMacBlocks) {
        const int b = b0 + lane;
        if (lane < kWaveMacBlocks && b < nb_inner) {
            uint32_t w[16];
            load_or_zero16(pkt, b, nb_data, end, w);
            inner_words(w, b, end, suffix);
            sha1_schedule_row(w, sched + lane * kWaveMacStride);
        }
        walk_sync(); // the rows, before lane 0 reads them
        if (lane == 0) {
            const int bn = min(nb_inner - b0, kWaveMacBlocks);
#pragma unroll 1
            for (int k = 0; k < bn; k++) {
                if (b0 + k == mid_b && mid_out) {
#pragma unroll
                    for (int q = 0; q < 5; q++) mid_out[q] = h[q];
                }
                sha1_compress_kw(h, sched + k * kWaveMacStride);
            }
        }
        walk_sync(); // lane 0 done with the rows
    }
    if (lane == 0) {
        uint32_t w[16];
        outer_words<false>(w, h, ks);
        sha1_compress(h, w);
    }
}

// Protect, packet p with final status OK: the MAC over the ciphertext and the
// trailer (k_protect's MacOnly instance: authenticatePacketHMAC :269-278,
// RawPacket.append :203-220).
template <bool WAVE>
__device__ __forceinline__ void mac_seal(const BundleArgs &a, uint32_t p, uint32_t *sched) {
    const KeySet *ks = a.keysets + a.ctx[a.p_slot[p]].ks;
    uint8_t *pkt = a.seg + a.off[p];
    const bool rtcp = ks->kind == SRTP_KIND_RTCP;
    const int T = ks->tag_len;
    const int L = (int)a.w_len[p] - T - (rtcp ? 4 : 0);
    const uint32_t cw = a.w_cw[p];
    const uint32_t suffix = !rtcp ? cw : (ks->enc_type == SRTP_AESCM_ENCRYPTION ? (cw | 0x80000000u) : 0u);
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = ks->ipad[k];
    if (WAVE) {
        mac_wave(pkt, L, suffix, ks, h, nullptr, -1, sched);
        if ((threadIdx.x & 63u) != 0u) return; // lane 0 holds the tag
    } else {
        mac_stream(pkt, L, suffix, ks, h, nullptr, -1);
    }
    if ((L & 3) == 0) {
        trailer_write_aligned(reinterpret_cast<uint32_t *>(pkt + L), rtcp, suffix, h, T);
    } else {
        int o = L;
        if (rtcp) {
            pkt[o] = (uint8_t)(suffix >> 24); pkt[o + 1] = (uint8_t)(suffix >> 16);
            pkt[o + 2] = (uint8_t)(suffix >> 8); pkt[o + 3] = (uint8_t)suffix;
            o += 4;
        }
        tag_write(h, pkt + o, T);
    }
}

// Unprotect, packet p before the walk: k_unprotect's prologue (context state,
// long-chain guess, quiet), the ROC guess, the tag check under it and the
// walk's re-check midstate (k_unprotect's MacOnly instance without
// speculation).
// WAVE: the whole wave on packet p (k_small), its stores from lane 0.
template <bool WAVE>
__device__ __forceinline__ void mac_check(const BundleArgs &a, uint32_t p, uint32_t *sched) {
    const bool lead = !WAVE || (threadIdx.x & 63u) == 0u;
    const uint32_t slot = a.p_slot[p];
    if (slot == kNoSlot) return;
    const uint32_t pos = a.spos[p];
    CtxState st = a.ctx[slot];
    const uint32_t far = a.far[slot];
    const bool lng = pos >= kLongRank && a.sk_out[pos - kLongRank] == slot;
    const bool quiet = !lng && (st.flags & 1u) && far != a.serial + 1u;
    if (lng) {
        const uint32_t hh = chain_head(a.sk_out, pos - kLongRank, slot);
        const int32_t seq_h = (int32_t)(a.sv_out[hh].word & 0xffffu);
        const int32_t seq = (int32_t)(a.sv_out[pos].word & 0xffffu);
        const int64_t e = (int64_t)guess_roc(st, seq_h) * 65536 + seq_h + (int64_t)(pos - hh);
        st.a = (int32_t)((e - seq + 32768) >> 16);
        st.flags &= ~1u;
    }
    const KeySet *ks = a.keysets + st.ks;
    uint8_t *pkt = a.seg + a.off[p];
    const int L = (int)a.len[p];
    const int T = ks->tag_len;
    const bool rtp = ks->kind == SRTP_KIND_RTP;
    const bool aes = ks->enc_type == SRTP_AESCM_ENCRYPTION;
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    int end;
    uint32_t suffix;
    if (rtp) {
        const int32_t seq = (int32_t)(bswap(hdr.x) & 0xffffu);
        const int32_t g = guess_roc(st, seq);
        if (lead) a.gok[2 * (size_t)p] = (uint32_t)g;
        end = max(L - T, 0);
        suffix = (uint32_t)g;
    } else {
        const int io = L - 4 - T;
        if (io < 0) { // the walk throws (no decryption due)
            if (lead) a.spec[p] = 0u;
            return;
        }
        suffix = ld_be32(pkt + io);
        end = io;
    }
    const uint32_t spec = (aes ? kSpecAes : 0u) | (rtp ? kSpecRtp : 0u) |
                          (rtp && a.flags && (a.flags[p] & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE)) ? kSpecSkip : 0u);
    if (lead) a.spec[p] = spec;
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = ks->ipad[k];
    uint32_t *const mid = (rtp && !quiet) ? a.mid + 5 * (size_t)p : nullptr;
    if (WAVE) mac_wave(pkt, end, suffix, ks, h, mid, end >> 6, sched);
    else mac_stream(pkt, end, suffix, ks, h, mid, end >> 6);
    if (lead) a.gok[2 * (size_t)p + 1] = tag_matches_at(h, pkt, L - T, T) ? 1u : 0u;
}

__device__ __forceinline__ void mac_seal_one(const BundleArgs &a, uint32_t p) { mac_seal<false>(a, p, nullptr); }
__device__ __forceinline__ void mac_check_one(const BundleArgs &a, uint32_t p) { mac_check<false>(a, p, nullptr); }

template <bool REV>
__global__ __launch_bounds__(kMacWideBlock) void k_mac_wide(BundleArgs a) {
    __shared__ uint32_t s_cnt[kTeCounters];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool live = i < a.n;
    const uint32_t p = live ? lane_packet(a, i) : i;
    if (!REV) {
        if (threadIdx.x < kTeCounters) s_cnt[threadIdx.x] = 0u;
        __syncthreads();
        int32_t fs = -1;
        if (live) {
            fs = finish_status(a, p);
            atomicAdd(&s_cnt[status_counter(a, p, fs)], 1u);
        }
        __syncthreads();
        flush_status_counts(a, s_cnt);
        if (fs == SRTP_STATUS_OK) mac_seal_one(a, p);
        return;
    }
    if (live) mac_check_one(a, p);
}

hipError_t launch_ctr_wide(const BundleArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const dim3 jg((a.n + kJobBlock - 1) / kJobBlock);
    if (a.reverse) hipLaunchKernelGGL(k_ctr_jobs<true>, jg, dim3(kJobBlock), 0, s, a);
    else hipLaunchKernelGGL(k_ctr_jobs<false>, jg, dim3(kJobBlock), 0, s, a);
    // Groups of 16 packets, four per wave of 256 workgroups x 16 waves on a
    // full bundle.  A smaller bundle keeps groups of at least two packets (a
    // 1200-B packet is 38 counter-block pairs: one group of one packet leaves
    // 26 lanes idle) and two groups per wave, so that it takes only the CUs
    // its work fills: each workgroup builds the 128-KB T-table image, and a
    // bundle that holds every CU's LDS for one round of work keeps another
    // bundle in flight (the aggregator's lanes keep two) off the GPU.
    uint32_t G = (uint32_t)kWideGMax;
    while (G > 2u && (a.n + G - 1u) / G < 4u * 4096u) G >>= 1;
    const uint32_t groups = (a.n + G - 1u) / G;
    const uint32_t waves = groups >= 4u * 4096u ? 4096u : (groups + 1u) / 2u;
    const uint32_t wgs = (waves + 15u) / 16u;
    const dim3 grid(wgs < 256u ? wgs : 256u);
    if (a.reverse) hipLaunchKernelGGL(k_ctr_wide<true>, grid, dim3(kWideBlock), 0, s, a, G);
    else hipLaunchKernelGGL(k_ctr_wide<false>, grid, dim3(kWideBlock), 0, s, a, G);
    return hipGetLastError();
}

hipError_t launch_mac_wide(const BundleArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const dim3 grid((a.n + kMacWideBlock - 1) / kMacWideBlock);
    if (a.reverse) hipLaunchKernelGGL(k_mac_wide<true>, grid, dim3(kMacWideBlock), 0, s, a);
    else hipLaunchKernelGGL(k_mac_wide<false>, grid, dim3(kMacWideBlock), 0, s, a);
    return hipGetLastError();
}

// ================================================= small bundles in one launch
// k_small: a bundle of up to kSmallMaxN packets (the per-packet callers' bundles:
// a lone synchronous call is a bundle of one) in one launch, its phases
// separated by barriers instead of kernel boundaries -- each boundary of the
// multi-kernel chain costs a small bundle a launch gap of ~4 us, and its
// parse, sort and walk kernels are all latency.  The phases are the split
// path's.  Workgroup 0, thread t on packet t:
//   parse (parse_one) -> sort (each record's rank among the n keys, stable)
//   -> unprotect: the tag check under the ROC guess (mac_check)
//   -> the walk (wave 0, walk_tile: one tile, as n < kLongMin; abort-on-throw:
//      the dry and the limit pass back to back)
// then every workgroup of the grid (one per kSmallPerWg packets) on its
// packets g, g + G, ...:
//   -> keystream jobs (unprotect: the final statuses, wide_job_rev), their
//      counter-block pairs over the workgroup's lanes (k_ctr_small's AES with
//      per-lane keys: one CU's LDS would bound a 255-packet bundle's keystream)
//   -> protect: final statuses, MAC and trailer (mac_seal).
// The other workgroups fill their T-table image meanwhile and wait for
// workgroup 0's flag (BundleCtl::small_ready, agent-scope release/acquire);
// workgroup 0 never waits on them, and every workgroup ends once its packets
// are done.
// The MACs: a lane per packet, except for the lone packet of a 1-packet
// bundle (kSmallWaveMacN), which has the wave (mac_wave: the lanes expand the
// schedule, one lane compresses -- a lone call's k_small 52 -> 41 us; with
// more packets the workgroup's MAC waves would share SIMDs and lose to the
// lane per packet).
// LDS: the 128-KB T-table image at 0 (the AES asm's addressing) -- which holds
// the wave MACs' schedules while no keystream runs (such an unprotect bundle
// fills it after the walk) -- then the status counts and one region that
// holds in turn the sort keys, the walk's arrays and the jobs.
constexpr int kSmallBlock = 512;
constexpr uint32_t kSmallPerWg = 16;    // packets per workgroup (the grid: at most 16)
#ifndef SRTP_SMALL_WAVE_MAC_N
#define SRTP_SMALL_WAVE_MAC_N 1
#endif
// bundles of up to this many packets: a wave per MAC (the lone call; with
// more, the workgroup's MAC waves would share SIMDs, profiles/r06
// kernel_experiments.md §3)
constexpr uint32_t kSmallWaveMacN = SRTP_SMALL_WAVE_MAC_N;
static_assert(kSmallMaxN < kLongMin && kSmallMaxN < (uint32_t)kSmallBlock && kSmallMaxN <= (uint32_t)kWalkSpan,
              "k_small: one walk tile, one record per thread");
static_assert((int)kSmallWaveMacN * kWaveMacWords <= kTeWords && kSmallWaveMacN <= kSmallPerWg,
              "k_small: the wave MACs' schedules inside the T-table image");
constexpr int kSmallJob = 8; // words per packet: iv[4], packet offset, region start, end, key set
constexpr int kSmallOffCnt = kTeWords;
constexpr int kSmallOffR = kSmallOffCnt + kTeCounters;
constexpr int kSmallOffPre = kSmallJob * (int)kSmallPerWg; // the pair prefix [kSmallPerWg + 1]
constexpr int kSmallJobsWords = kSmallOffPre + (int)kSmallPerWg + 4;
constexpr int kSmallWalkWords = (int)(sizeof(WalkShared<true>) / 4);
constexpr int kSmallRWords = kSmallWalkWords > kSmallJobsWords ? kSmallWalkWords : kSmallJobsWords;
static_assert(kSmallOffR % 4 == 0 && sizeof(WalkShared<true>) % 4 == 0, "k_small: 16-B aligned region");
static_assert((kSmallOffR + kSmallRWords) * 4 <= 160 * 1024, "k_small: LDS");

// Direct mode (BundleArgs::pk_host): workgroup 0 reads the packed block from
// the pinned host copy first -- every load of a thread in flight before its
// stores, so the block costs a PCIe round trip or two, not one per 8 KB --
// and each workgroup writes its packets' lengths, statuses and regions back.
constexpr int kPullPer = 8; // 16-B pieces per thread per round trip
__device__ __forceinline__ void small_pull(const BundleArgs &a) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.pk_host);
    uint4 *dst = reinterpret_cast<uint4 *>(a.pk_dev);
    const uint32_t n16 = a.pk_bytes >> 4;
    for (uint32_t i0 = 0; i0 < n16; i0 += kPullPer * kSmallBlock) {
        uint4 v[kPullPer];
#pragma unroll
        for (int k = 0; k < kPullPer; k++) {
            const uint32_t i = i0 + (uint32_t)k * kSmallBlock + threadIdx.x;
            if (i < n16) v[k] = src[i];
        }
#pragma unroll
        for (int k = 0; k < kPullPer; k++) {
            const uint32_t i = i0 + (uint32_t)k * kSmallBlock + threadIdx.x;
            if (i < n16) dst[i] = v[k];
        }
    }
}

// the workgroup's packets g + G * i (i < m) back to the host copy
__device__ __forceinline__ void small_push(const BundleArgs &a, uint32_t g, uint32_t G, uint32_t m) {
    uint8_t *const host = const_cast<uint8_t *>(a.pk_host);
    auto hp = [&](const void *d) { return host + (reinterpret_cast<const uint8_t *>(d) - a.pk_dev); };
    const uint32_t t = threadIdx.x;
    if (t < m) {
        const uint32_t p = g + G * t;
        *reinterpret_cast<uint32_t *>(hp(a.len + p)) = a.len[p];
        *reinterpret_cast<int32_t *>(hp(a.status + p)) = a.status[p];
    }
    for (uint32_t i = 0; i < m; i++) {
        const uint32_t p = g + G * i;
        const uint4 *src = reinterpret_cast<const uint4 *>(a.seg + a.off[p]);
        uint4 *dst = reinterpret_cast<uint4 *>(hp(a.seg + a.off[p]));
        const uint32_t n16 = (a.cap[p] + 15u) >> 4;
        for (uint32_t c = t; c < n16; c += kSmallBlock) dst[c] = src[c];
    }
}

template <bool REV>
__global__ __launch_bounds__(kSmallBlock) void k_small(BundleArgs a) {
    __shared__ uint32_t s[kSmallOffR + kSmallRWords];
    if (a.pk_host && blockIdx.x == 0) {
        small_pull(a);
        __syncthreads();
    }
    uint32_t *const s_cnt = s + kSmallOffCnt;
    uint32_t *const r = s + kSmallOffR;
    const uint32_t t = threadIdx.x, n = a.n, g = blockIdx.x, G = gridDim.x;
    const uint32_t wv = t >> 6;
    const bool wave_mac = n <= kSmallWaveMacN; // (then G == 1)
    if (t < kTeCounters) s_cnt[t] = 0u;
    // the T-table image now, unless it first holds an unprotect's wave MACs
    if (!REV || !wave_mac) fill_te4(s); // ends with a barrier
    if (g == 0) {
        // the next bundle's control block and abort limits (as k_parse)
        if (t == 0) *a.ctl_next = BundleCtl{};
        if (a.abort_on_error)
            for (uint32_t i = t; i < a.n_transformers; i += kSmallBlock) a.e_min_next[i] = 0x7f7f7f7f;
        // 1. parse
        uint32_t key = 0u;
        if (t < n) {
            key = parse_one(a, t);
            r[t] = key;
        }
        __syncthreads();
        // 2. sort: the sorted arrays and (unprotect) each packet's position, as
        // k_sort_tile leaves them (stable by key; invalid packets' keys last)
        if (t < n) {
            uint32_t rank = 0u;
            for (uint32_t q = 0; q < n; q++) {
                const uint32_t kq = r[q];
                rank += (kq < key || (kq == key && q < t)) ? 1u : 0u;
            }
            a.sk_out[rank] = key;
            a.sv_out[rank] = a.sv_in[t];
            if (REV && key <= a.ctx_mask) a.spos[t] = rank;
        }
        __syncthreads();
        // 3. unprotect: the tag checks before the walk
        if (REV) {
            if (wave_mac) {
                if (wv < n) mac_check<true>(a, wv, s + wv * kWaveMacWords);
            } else if (t < n) {
                mac_check<false>(a, t, nullptr);
            }
            __syncthreads();
        }
        // 4. the walk; abort-on-throw with a packet that may throw: the dry
        // pass, then the limit pass (k_walk's two launches)
        if (t < 64) {
            WalkShared<REV> &sh = *reinterpret_cast<WalkShared<REV> *>(r);
            walk_tile<REV, false, 0>(a, sh, 0u, 1u);
            if (a.abort_on_error && a.ctl->any_throw) {
                walk_sync();
                walk_tile<REV, false, 1>(a, sh, 0u, 1u);
            }
        }
        __syncthreads();
        // everything the other workgroups read, visible at agent scope first
        if (G > 1 && t == 0) {
            __threadfence();
            __hip_atomic_store(&a.ctl->small_ready, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        if (t == 0)
            while (__hip_atomic_load(&a.ctl->small_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < 2u)
                __builtin_amdgcn_s_sleep(2);
        __syncthreads();
    }
    if (REV && wave_mac) fill_te4(s); // ends with a barrier
    // 5. this workgroup's packets p = g + G * i: keystream jobs and their pair
    // counts, then the pairs' prefix
    const uint32_t m = n > g ? (n - g + G - 1u) / G : 0u;
    uint32_t *const job = r;
    uint32_t *const pre = r + kSmallOffPre;
    if (t < kSmallPerWg) {
        uint32_t pairs = 0u;
        if (t < m) {
            const uint32_t p = g + G * t;
            int start = 0, end = 0;
            uint32_t iv[4] = {0u, 0u, 0u, 0u};
            const KeySet *ks = nullptr;
            const bool ok = REV ? wide_job_rev(a, p, s_cnt, start, end, iv, ks) : ctr_small_job(a, p, start, end, iv, ks);
            uint4 *jp = reinterpret_cast<uint4 *>(job + kSmallJob * t);
            jp[0] = make_uint4(iv[0], iv[1], iv[2], iv[3]);
            jp[1] = make_uint4(a.off[p], (uint32_t)start, (uint32_t)end, ok ? (uint32_t)(ks - a.keysets) : 0u);
            pairs = ok ? (uint32_t)(end - start + 31) >> 5 : 0u;
        }
        uint32_t x = pairs; // inclusive prefix over the workgroup's packets
#pragma unroll
        for (int o = 1; o < (int)kSmallPerWg; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o, (int)kSmallPerWg);
            if ((int)t >= o) x += y;
        }
        pre[t] = x - pairs;
        if (t == kSmallPerWg - 1u) pre[kSmallPerWg] = x;
    }
    __syncthreads();
    // 6. the pairs, consecutive pairs of a packet on consecutive lanes
    const uint32_t total = pre[kSmallPerWg];
    const TeBase tb = te_base();
    const char *lds = reinterpret_cast<const char *>(s);
    for (uint32_t q = t; q < total; q += kSmallBlock) {
        uint32_t i = 0u; // the last packet whose pairs start at or before q
#pragma unroll
        for (uint32_t k = 1; k < kSmallPerWg; k++) i += (k < m && pre[k] <= q) ? 1u : 0u;
        const uint4 j0 = *reinterpret_cast<const uint4 *>(job + kSmallJob * i);
        const uint4 j1 = *reinterpret_cast<const uint4 *>(job + kSmallJob * i + 4);
        const uint32_t iv[4] = {j0.x, j0.y, j0.z, j0.w};
        const int start = (int)j1.y, end = (int)j1.z;
        const int j = 2 * (int)(q - pre[i]);
        const uint4 kw = *reinterpret_cast<const uint4 *>(a.keysets[j1.w].rk);
        const uint32_t k0[4] = {kw.x, kw.y, kw.z, kw.w};
        uint32_t x[4], y[4];
        ctr_input(iv, j, x);
        ctr_input(iv, j + 1, y);
        aes_encrypt2_v(lds, tb, k0, x, y);
        uint8_t *pkt = a.seg + j1.x;
        if ((start & 3) == 0) {
            xor_ks32(pkt, start + 16 * j, end, x, y);
        } else { // not a header of whole words: byte by byte
            xor_ks16(pkt + start + 16 * j, end - (start + 16 * j), x);
            if (start + 16 * (j + 1) < end) xor_ks16(pkt + start + 16 * (j + 1), end - (start + 16 * (j + 1)), y);
        }
    }
    __syncthreads();
    // 7. protect: final statuses, then the MAC over the ciphertext and the
    // trailer (the T-table image is free again for the wave MACs)
    uint32_t *const s_fs = r + kSmallOffPre; // the prefix is no longer needed
    const uint32_t p = g + G * t;
    int32_t fs = -1;
    if (!REV && t < m) {
        fs = finish_status(a, p);
        atomicAdd(&s_cnt[status_counter(a, p, fs)], 1u);
    }
    __syncthreads(); // every lane past the prefix
    if (!REV && t < m) s_fs[t] = (uint32_t)fs;
    __syncthreads();
    flush_status_counts(a, s_cnt);
    if (!REV) {
        if (wave_mac) {
            if (wv < m && (int32_t)s_fs[wv] == SRTP_STATUS_OK) mac_seal<true>(a, wv, s + wv * kWaveMacWords);
        } else if (fs == SRTP_STATUS_OK) {
            mac_seal<false>(a, p, nullptr);
        }
    }
    if (a.pk_host) {
        __syncthreads(); // every packet's bytes final
        small_push(a, g, G, m);
    }
}

hipError_t launch_small(const BundleArgs &a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    if (a.n > kSmallMaxN) return hipErrorInvalidValue;
    const dim3 grid((a.n + kSmallPerWg - 1u) / kSmallPerWg); // at most 16
    if (a.reverse) hipLaunchKernelGGL(k_small<true>, grid, dim3(kSmallBlock), 0, s, a);
    else hipLaunchKernelGGL(k_small<false>, grid, dim3(kSmallBlock), 0, s, a);
    return hipGetLastError();
}

// ========================================== gather / scatter of host bundles
// A dispatcher shard's chunk of an interleaved host bundle in registered
// (device-mapped) memory: its packets' regions are read from the caller's
// segment over PCIe into the slot's device segment (k_gather_regions), and
// written back after the bundle (k_scatter_regions) -- by the GPU, instead of
// a host copy into and out of the pinned slot (srtp_pipeline_submit_gather).
// A wave moves two packet regions at a time, 16 B per lane per instruction (a
// wave-instruction moves 1 KB of one region): every load of both regions (up
// to 2 KB each) is issued before any store, so reads over PCIe keep 4 KB per
// wave in flight instead of waiting out a round trip per KB.
constexpr int kGatherBlock = 256;
template <bool ToDevice>
__global__ __launch_bounds__(kGatherBlock) void k_move_regions(uint8_t *dseg, const uint32_t *doff,
                                                               const uint32_t *cap, uint8_t *host,
                                                               const uint32_t *src, uint32_t n) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * (kGatherBlock / 64);
    for (uint32_t j = 2u * (blockIdx.x * (kGatherBlock / 64) + (threadIdx.x >> 6)); j < n; j += 2u * waves) {
        const bool two = j + 1u < n;
        const uint32_t wa = ((cap[j] + 15u) & ~15u) / 16u, wb = two ? ((cap[j + 1] + 15u) & ~15u) / 16u : 0u;
        uint4 *da = reinterpret_cast<uint4 *>(dseg + doff[j]);
        uint4 *ha = reinterpret_cast<uint4 *>(host + src[j]);
        uint4 *db = reinterpret_cast<uint4 *>(dseg + doff[two ? j + 1 : j]);
        uint4 *hb = reinterpret_cast<uint4 *>(host + src[two ? j + 1 : j]);
        uint4 *fa = ToDevice ? ha : da, *ta = ToDevice ? da : ha;
        uint4 *fb = ToDevice ? hb : db, *tb = ToDevice ? db : hb;
        for (uint32_t o = lane; o < max(wa, wb); o += 128u) {
            const bool a0 = o < wa, a1 = o + 64u < wa, b0 = o < wb, b1 = o + 64u < wb;
            uint4 x0, x1, y0, y1;
            if (a0) x0 = fa[o];
            if (a1) x1 = fa[o + 64u];
            if (b0) y0 = fb[o];
            if (b1) y1 = fb[o + 64u];
            if (a0) ta[o] = x0;
            if (a1) ta[o + 64u] = x1;
            if (b0) tb[o] = y0;
            if (b1) tb[o + 64u] = y1;
        }
    }
}

hipError_t launch_move_regions(bool to_device, uint8_t *dseg, const uint32_t *doff, const uint32_t *cap,
                               uint8_t *host, const uint32_t *src, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t wgs = std::min<uint32_t>((n + 7u) / 8u, 4096u); // two regions per wave
    if (to_device)
        hipLaunchKernelGGL(k_move_regions<true>, dim3(wgs), dim3(kGatherBlock), 0, s, dseg, doff, cap, host, src, n);
    else
        hipLaunchKernelGGL(k_move_regions<false>, dim3(wgs), dim3(kGatherBlock), 0, s, dseg, doff, cap, host, src, n);
    return hipGetLastError();
}

hipError_t launch_protect(const BundleArgs &a, hipStream_t s) {
    const uint32_t b = aes_block(a.n, (uint32_t)kProtectBlock);
    if (a.small_ctr) {
        const uint32_t bm = std::min<uint32_t>(b, (uint32_t)kMacBlock);
        hipLaunchKernelGGL(k_protect<true>, dim3((a.n + bm - 1) / bm), dim3(bm), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_protect<false>, dim3((a.n + b - 1) / b), dim3(b), 0, s, a);
    }
    return hipGetLastError();
}
hipError_t launch_unprotect_fix(const BundleArgs &a, hipStream_t s) {
    hipLaunchKernelGGL(k_unprotect_fix, dim3((a.n + kAesBlock - 1) / kAesBlock), dim3(kAesBlock), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_ext(const BundleArgs &a, hipStream_t s) {
    const uint32_t lanes = (a.n + 1) / 2; // two packets per lane
    hipLaunchKernelGGL(k_ext, dim3((lanes + kExtBlock - 1) / kExtBlock), dim3(kExtBlock), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_remove_transformer(uint64_t *keys, CtxState *ctx, uint32_t cap, uint32_t tid,
                                     hipStream_t s) {
    hipLaunchKernelGGL(k_remove_transformer, grid_for(cap), dim3(kBlock), 0, s, keys, ctx, cap, tid);
    return hipGetLastError();
}
hipError_t launch_ctx_save(const uint64_t *tab, const CtxState *ctx, uint32_t mask, const uint64_t *keys,
                           uint32_t n, CtxState *out, int32_t *present, hipStream_t s) {
    hipLaunchKernelGGL(k_ctx_save, grid_for(n), dim3(kBlock), 0, s, tab, ctx, mask, keys, n, out, present);
    return hipGetLastError();
}
hipError_t launch_ctx_restore(uint64_t *tab, CtxState *ctx, uint32_t mask, const uint64_t *keys, uint32_t n,
                              const CtxState *in, const int32_t *present, unsigned int *failed,
                              hipStream_t s) {
    hipLaunchKernelGGL(k_ctx_restore, grid_for(n), dim3(kBlock), 0, s, tab, ctx, mask, keys, n, in, present,
                       failed);
    return hipGetLastError();
}
hipError_t launch_count_contexts(const uint64_t *keys, uint32_t cap, unsigned long long *out,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_count_contexts, grid_for(cap), dim3(kBlock), 0, s, keys, cap, out);
    return hipGetLastError();
}
hipError_t launch_rehash_collect(const uint64_t *keys, const CtxState *ctx, uint32_t cap,
                                 uint64_t *tmp_keys, CtxState *tmp_ctx, unsigned long long *n_live,
                                 hipStream_t s) {
    hipLaunchKernelGGL(k_rehash_collect, grid_for(cap), dim3(kBlock), 0, s, keys, ctx, cap, tmp_keys,
                       tmp_ctx, n_live);
    return hipGetLastError();
}
hipError_t launch_rehash_insert(uint64_t *keys, CtxState *ctx, uint32_t mask, const uint64_t *tmp_keys,
                                const CtxState *tmp_ctx, uint32_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_rehash_insert, grid_for(n), dim3(kBlock), 0, s, keys, ctx, mask, tmp_keys,
                       tmp_ctx, n);
    return hipGetLastError();
}
hipError_t upload_tables(const uint32_t te0[256]) {
    return hipMemcpyToSymbol(HIP_SYMBOL(d_te0), te0, 256 * sizeof(uint32_t));
}

} // namespace srtp
