// split_bench.hip -- would a split protect beat the fused k_protect?
//
// k_protect runs AES-CM and HMAC-SHA1 fused, one workgroup of 16 waves per CU
// (the 128-KB T-table image, 128 VGPRs): the PMC passes show it latency-bound
// (waves waiting 44 % of their cycles, LDS busy 0.49, VALU 0.37).  Split into
// two kernels each could run at its own best occupancy:
//   k_ctr: AES-CM keystream XOR only, in place; with the 2-table image (64 KB,
//          aes_asm.py tables=2) two workgroups fit a CU -- up to 32 waves;
//   k_mac: HMAC-SHA1 over the ciphertext + the tag; VALU only, no LDS;
// at the cost of reading the packet twice.  This tool times the variants on
// the bench workload (2^18 x 1200-B RTP packets, 10k SSRCs, first bundle of
// each stream: ROC 0) and checks every byte of the split result against the
// engine's own protect of the same bundle (C ABI), whose k_protect time it
// also reports (srtp_engine_set_timing, same process and GPU).
//
//   split_bench [reps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/srtp_mi355x.h"
#include "../libjitsi_amd/csrc/host_crypto.h"

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

constexpr int kN = 1 << 18, kLen = 1200, kStride = 1216, kSsrc = 10000, kTag = 10;

__device__ uint32_t d_te0[256];

#include "aes_bench_rounds.inc"

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
    return n ? __builtin_amdgcn_alignbit(x, x, 32u - n) : x;
}
__device__ __forceinline__ uint32_t sgpr(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct Keys {
    uint32_t rk[44], ipad[5], opad[5], salt[4];
};

// ------------------------------------------------------------------ k_ctr
template <int T>
__device__ __forceinline__ uint32_t tl(const char *lds, const uint32_t *bs, uint32_t s, int k, int t) {
    // entry (byte k of s) of table t; with two tables T2/T3 are rotl16 of T0/T1
    const int tt = T == 4 ? t : (t & 1);
    const uint32_t v = *reinterpret_cast<const uint32_t *>(
        lds + __builtin_amdgcn_perm(s, bs[tt], (T == 4 ? 0x0c020000u : 0x0c0c0000u) | ((4u + (uint32_t)k) << 8)));
    return (T == 2 && t >= 2) ? rotl(v, 16) : v;
}

// WPE: waves per SIMD asked of the register allocator (2 workgroups of the
// 2-table image fit a CU's LDS: 1024 threads x 2 = 8 waves per SIMD)
template <int T, int THREADS, int WPE>
__global__ __attribute__((amdgpu_flat_work_group_size(1, THREADS), amdgpu_waves_per_eu(WPE, WPE))) void k_ctr(uint8_t *seg, const Keys *kg) {
    constexpr int WORDS = T == 4 ? 32768 : 16384;
    __shared__ uint32_t s_te[WORDS];
    for (int i = threadIdx.x; i < WORDS; i += THREADS) {
        const int t = T == 4 ? (((i >> 14) << 1) | ((i >> 5) & 1)) : ((i >> 5) & 1);
        s_te[i] = rotl(d_te0[(i >> 6) & 255], 8u * (uint32_t)t);
    }
    __syncthreads();
    asm volatile("" ::"s"(s_te) : "memory");
    const char *lds = reinterpret_cast<const char *>(s_te);
    const uint32_t c4 = (threadIdx.x & 31u) << 2;
    uint32_t bs[4];
#pragma unroll
    for (int t = 0; t < 4; t++)
        bs[t] = T == 4 ? ((uint32_t)((t >> 1) << 16) | (uint32_t)((t & 1) << 7) | c4)
                       : ((uint32_t)((t & 1) << 7) | c4);
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; i++) rk[i] = sgpr(kg->rk[i]);
    const uint32_t p = blockIdx.x * THREADS + threadIdx.x;
    if (p >= (uint32_t)kN) return;
    uint8_t *pkt = seg + (size_t)p * kStride;
    const uint4 hdr = *reinterpret_cast<const uint4 *>(pkt);
    uint32_t iv[4];
    iv[0] = sgpr(kg->salt[0]);
    iv[1] = sgpr(kg->salt[1]) ^ hdr.z;
    iv[2] = sgpr(kg->salt[2]); // ROC 0
    iv[3] = sgpr(kg->salt[3]) ^ (hdr.x >> 16);
    // rounds 1-2 precomputed (srtp_kernels.hip ctr_precompute / ctr_first2)
    const uint32_t w0 = iv[0] ^ rk[0], w1 = iv[1] ^ rk[1], w2 = iv[2] ^ rk[2], w3 = iv[3] ^ rk[3];
    const uint32_t kb = w3 >> 24;
    const uint32_t p0 = xor3(tl<T>(lds, bs, w0, 0, 0), tl<T>(lds, bs, w1, 1, 1), tl<T>(lds, bs, w2, 2, 2)) ^ rk[4];
    const uint32_t u1 = xor3(tl<T>(lds, bs, w1, 0, 0), tl<T>(lds, bs, w2, 1, 1), tl<T>(lds, bs, w3, 2, 2)) ^
                        tl<T>(lds, bs, w0, 3, 3) ^ rk[5];
    const uint32_t u2 = xor3(tl<T>(lds, bs, w2, 0, 0), tl<T>(lds, bs, w3, 1, 1), tl<T>(lds, bs, w0, 2, 2)) ^
                        tl<T>(lds, bs, w1, 3, 3) ^ rk[6];
    const uint32_t u3 = xor3(tl<T>(lds, bs, w3, 0, 0), tl<T>(lds, bs, w0, 1, 1), tl<T>(lds, bs, w1, 2, 2)) ^
                        tl<T>(lds, bs, w2, 3, 3) ^ rk[7];
    uint32_t r[4];
    r[0] = xor3(tl<T>(lds, bs, u1, 1, 1), tl<T>(lds, bs, u2, 2, 2), tl<T>(lds, bs, u3, 3, 3)) ^ rk[8];
    r[1] = xor3(tl<T>(lds, bs, u1, 0, 0), tl<T>(lds, bs, u2, 1, 1), tl<T>(lds, bs, u3, 2, 2)) ^ rk[9];
    r[2] = xor3(tl<T>(lds, bs, u2, 0, 0), tl<T>(lds, bs, u3, 1, 1), tl<T>(lds, bs, u1, 3, 3)) ^ rk[10];
    r[3] = xor3(tl<T>(lds, bs, u3, 0, 0), tl<T>(lds, bs, u1, 2, 2), tl<T>(lds, bs, u2, 3, 3)) ^ rk[11];
    // payload [12, 1200): keystream word i -> packet word 3 + i; 75 blocks,
    // chunk c (bytes 64c..64c+63) takes blocks 4c-1 .. 4c+2 (carry of 3 words)
    uint32_t carry[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int c = 0; c < 19; c++) {
        uint32_t K[16];
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {
            const int ja = 4 * c + 2 * pr, jb = ja + 1;
            uint32_t s[2][4];
            const uint32_t xa = (uint32_t)ja ^ kb, xb = (uint32_t)jb ^ kb;
            const uint32_t ua = p0 ^ tl<T>(lds, bs, xa, 0, 3), ub = p0 ^ tl<T>(lds, bs, xb, 0, 3);
            s[0][0] = r[0] ^ tl<T>(lds, bs, ua, 0, 0); s[1][0] = r[0] ^ tl<T>(lds, bs, ub, 0, 0);
            s[0][1] = r[1] ^ tl<T>(lds, bs, ua, 3, 3); s[1][1] = r[1] ^ tl<T>(lds, bs, ub, 3, 3);
            s[0][2] = r[2] ^ tl<T>(lds, bs, ua, 2, 2); s[1][2] = r[2] ^ tl<T>(lds, bs, ub, 2, 2);
            s[0][3] = r[3] ^ tl<T>(lds, bs, ua, 1, 1); s[1][3] = r[3] ^ tl<T>(lds, bs, ub, 1, 1);
#pragma unroll
            for (int rr = 3; rr < 10; rr++) {
                if constexpr (T == 4) aes_mid_n2_t4(s[0], s[1], bs, rk + 4 * rr);
                else aes_mid_n2_t2(s[0], s[1], bs, rk + 4 * rr);
            }
            if constexpr (T == 4) aes_last_n2_t4(s[0], s[1], bs, rk + 40);
            else aes_last_n2_t2(s[0], s[1], bs, rk + 40);
#pragma unroll
            for (int k = 0; k < 4; k++) { K[8 * pr + k] = s[0][k]; K[8 * pr + 4 + k] = s[1][k]; }
        }
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 64 * c);
        uint32_t d[16];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint4 v = q[m];
            d[4 * m] = v.x; d[4 * m + 1] = v.y; d[4 * m + 2] = v.z; d[4 * m + 3] = v.w;
        }
        // word i of the chunk takes keystream word 16c + i - 3
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint32_t ks = i >= 3 ? K[i - 3] : carry[1 + i];
            const int pos = 64 * c + 4 * i;
            if (pos >= 12 && pos < kLen) d[i] ^= ks;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) carry[k] = K[12 + k];
#pragma unroll
        for (int m = 0; m < 4; m++)
            if (64 * c + 16 * m < kLen) q[m] = make_uint4(d[4 * m], d[4 * m + 1], d[4 * m + 2], d[4 * m + 3]);
    }
}

// ------------------------------------------------------------------ k_mac
__device__ __forceinline__ void sha1c(uint32_t h[5], uint32_t w[16]) {
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
        else if (t < 40) { f = xor3(b, c, d); k = 0x6ED9EBA1u; }
        else if (t < 60) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); k = 0x8F1BBCDCu; }
        else { f = xor3(b, c, d); k = 0xCA62C1D6u; }
        const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

template <int THREADS, int MINW>
__global__ __launch_bounds__(THREADS, MINW) void k_mac(uint8_t *seg, const Keys *kg) {
    const uint32_t p = blockIdx.x * THREADS + threadIdx.x;
    if (p >= (uint32_t)kN) return;
    uint8_t *pkt = seg + (size_t)p * kStride;
    uint32_t h[5];
#pragma unroll
    for (int k = 0; k < 5; k++) h[k] = sgpr(kg->ipad[k]);
    // inner: packet[0, 1200) || ROC (0) || 0x80 .. || bit length of 64 + 1204
    const uint4 *q = reinterpret_cast<const uint4 *>(pkt);
#pragma unroll 1
    for (int b = 0; b < 18; b++) {
        uint32_t w[16];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const uint4 v = q[4 * b + m];
            w[4 * m] = bswap(v.x); w[4 * m + 1] = bswap(v.y); w[4 * m + 2] = bswap(v.z); w[4 * m + 3] = bswap(v.w);
        }
        sha1c(h, w);
    }
    {
        uint32_t w[16];
#pragma unroll
        for (int m = 0; m < 3; m++) { // bytes 1152..1199
            const uint4 v = q[72 + m];
            w[4 * m] = bswap(v.x); w[4 * m + 1] = bswap(v.y); w[4 * m + 2] = bswap(v.z); w[4 * m + 3] = bswap(v.w);
        }
        w[12] = 0u;          // ROC 0
        w[13] = 0x80000000u;
        w[14] = 0u;
        w[15] = (64u + 1204u) * 8u;
        sha1c(h, w);
    }
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 5; k++) { w[k] = h[k]; h[k] = sgpr(kg->opad[k]); }
    w[5] = 0x80000000u;
#pragma unroll
    for (int k = 6; k < 15; k++) w[k] = 0u;
    w[15] = (64 + 20) * 8;
    sha1c(h, w);
    uint8_t *tag = pkt + kLen;
#pragma unroll
    for (int i = 0; i < kTag; i++) tag[i] = (uint8_t)(h[i / 4] >> (24 - 8 * (i % 4)));
}

// ------------------------------------------------------------------ host
static uint64_t rng_state = 0x5EED0002ull;
static uint32_t rnd() {
    rng_state = rng_state * 6364136223846793005ull + 1442695040888963407ull;
    return (uint32_t)(rng_state >> 32);
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    const size_t bytes = (size_t)kN * kStride;
    std::vector<uint8_t> h_seg(bytes, 0);
    std::vector<uint32_t> off(kN), len(kN, kLen), cap(kN, kStride);
    std::vector<uint32_t> ssrc(kSsrc), seq0(kSsrc);
    for (int s = 0; s < kSsrc; s++) { ssrc[s] = rnd() | 1u; seq0[s] = rnd() & 0x7fffu; } // no seq wrap: ROC 0
    for (int i = 0; i < kN; i++) {
        uint8_t *p = &h_seg[(size_t)i * kStride];
        off[i] = (uint32_t)i * kStride;
        for (int k = 12; k < kLen; k++) p[k] = (uint8_t)rnd();
        const int s = i % kSsrc;
        const uint32_t sq = (seq0[s] + (uint32_t)(i / kSsrc)) & 0xffffu;
        p[0] = 0x80; p[1] = 96; p[2] = (uint8_t)(sq >> 8); p[3] = (uint8_t)sq;
        p[4] = p[5] = p[6] = p[7] = 0;
        p[8] = (uint8_t)(ssrc[s] >> 24); p[9] = (uint8_t)(ssrc[s] >> 16);
        p[10] = (uint8_t)(ssrc[s] >> 8); p[11] = (uint8_t)ssrc[s];
    }
    uint8_t mk[16], ms[14];
    for (auto &x : mk) x = (uint8_t)rnd();
    for (auto &x : ms) x = (uint8_t)rnd();
    // the engine's protect of the bundle: the reference result and the fused time
    srtp_engine_opts o;
    srtp_engine_opts_default(&o);
    o.max_contexts = 1u << 15;
    o.max_batch = kN;
    srtp_engine *e = nullptr;
    if (srtp_engine_create(&o, &e) != SRTP_OK) { printf("engine create failed\n"); return 1; }
    srtp_policy pol = {SRTP_AESCM_ENCRYPTION, 16, SRTP_HMACSHA1_AUTHENTICATION, 20, kTag, 14};
    int32_t f = -1, t = -1;
    srtp_factory_create(e, 1, mk, 16, ms, 14, &pol, &pol, &f);
    srtp_transformer_create(e, SRTP_KIND_RTP, f, f, &t);
    uint8_t *d_ref, *d_seg;
    uint32_t *d_off, *d_len, *d_cap;
    int32_t *d_st;
    CHECK(hipMalloc(&d_ref, bytes));
    CHECK(hipMalloc(&d_seg, bytes));
    CHECK(hipMalloc(&d_off, kN * 4));
    CHECK(hipMalloc(&d_len, kN * 4));
    CHECK(hipMalloc(&d_cap, kN * 4));
    CHECK(hipMalloc(&d_st, kN * 4));
    CHECK(hipMemcpy(d_ref, h_seg.data(), bytes, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_off, off.data(), kN * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_len, len.data(), kN * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d_cap, cap.data(), kN * 4, hipMemcpyHostToDevice));
    srtp_engine_set_timing(e, 1);
    if (srtp_transform_device(e, 0, nullptr, t, d_ref, d_off, d_len, d_cap, nullptr, d_st, kN, nullptr) != SRTP_OK) {
        printf("engine protect failed: %s\n", srtp_engine_last_error(e));
        return 1;
    }
    CHECK(hipDeviceSynchronize());
    double ms_st[SRTP_NUM_STAGES];
    uint64_t cnt[SRTP_NUM_STAGES];
    srtp_engine_read_timing(e, ms_st, cnt);
    std::vector<uint8_t> ref(bytes);
    CHECK(hipMemcpy(ref.data(), d_ref, bytes, hipMemcpyDeviceToHost));
    // fused k_protect time over `reps` further protects of the same packets
    // (the same indices: the sender's contexts do not move)
    CHECK(hipMemcpy(d_seg, h_seg.data(), bytes, hipMemcpyHostToDevice));
    for (int r = 0; r < reps + 3; r++) {
        if (r == 3) srtp_engine_read_timing(e, ms_st, cnt);
        CHECK(hipMemcpy(d_len, len.data(), kN * 4, hipMemcpyHostToDevice));
        if (srtp_transform_device(e, 0, nullptr, t, d_seg, d_off, d_len, d_cap, nullptr, d_st, kN, nullptr) !=
            SRTP_OK) {
            printf("engine protect failed: %s\n", srtp_engine_last_error(e));
            return 1;
        }
    }
    CHECK(hipDeviceSynchronize());
    srtp_engine_read_timing(e, ms_st, cnt);
    printf("{\"kernel\": \"k_protect (fused, engine)\", \"us\": %.1f}\n",
           1e3 * ms_st[SRTP_STAGE_PROTECT] / (double)(cnt[SRTP_STAGE_PROTECT] ? cnt[SRTP_STAGE_PROTECT] : 1));
    srtp_engine_destroy(e);
    // keys for the split kernels
    Keys K;
    uint8_t enc[16], auth[20], salt[14];
    srtp::derive_session_keys(mk, ms, false, enc, auth, salt);
    srtp::aes128_expand_le(enc, K.rk);
    srtp::hmac_sha1_midstates(auth, K.ipad, K.opad);
    uint8_t s16[16] = {0};
    memcpy(s16, salt, 14);
    for (int i = 0; i < 4; i++)
        K.salt[i] = (uint32_t)s16[4 * i] | ((uint32_t)s16[4 * i + 1] << 8) | ((uint32_t)s16[4 * i + 2] << 16) |
                    ((uint32_t)s16[4 * i + 3] << 24);
    uint32_t te0[256];
    srtp::aes_te0_le(te0);
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(d_te0), te0, sizeof te0));
    Keys *d_keys;
    CHECK(hipMalloc(&d_keys, sizeof K));
    CHECK(hipMemcpy(d_keys, &K, sizeof K, hipMemcpyHostToDevice));
    hipEvent_t e0, e1, e2;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventCreate(&e2));
    auto run = [&](const char *name, auto &&ctr, auto &&mac) {
        CHECK(hipMemcpy(d_seg, h_seg.data(), bytes, hipMemcpyHostToDevice));
        ctr();
        mac();
        CHECK(hipDeviceSynchronize());
        std::vector<uint8_t> got(bytes);
        CHECK(hipMemcpy(got.data(), d_seg, bytes, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int i = 0; i < kN; i++)
            bad += memcmp(&got[(size_t)i * kStride], &ref[(size_t)i * kStride], kLen + kTag) != 0;
        float a = 0, b = 0;
        for (int r = 0; r < 3; r++) { ctr(); mac(); }
        float ta = 0, tb = 0;
        for (int r = 0; r < reps; r++) {
            CHECK(hipEventRecord(e0));
            ctr();
            CHECK(hipEventRecord(e1));
            mac();
            CHECK(hipEventRecord(e2));
            CHECK(hipEventSynchronize(e2));
            CHECK(hipEventElapsedTime(&a, e0, e1));
            CHECK(hipEventElapsedTime(&b, e1, e2));
            ta += a;
            tb += b;
        }
        printf("{\"variant\": \"%s\", \"ctr_us\": %.1f, \"mac_us\": %.1f, \"total_us\": %.1f, "
               "\"packets_differing_from_engine\": %zu}\n",
               name, 1e3 * ta / reps, 1e3 * tb / reps, 1e3 * (ta + tb) / reps, bad);
        fflush(stdout);
    };
    auto mac256 = [&] { hipLaunchKernelGGL((k_mac<256, 1>), dim3(kN / 256), dim3(256), 0, 0, d_seg, d_keys); };
    run("ctr T4 1024x1 + mac 256",
        [&] { hipLaunchKernelGGL((k_ctr<4, 1024, 4>), dim3(kN / 1024), dim3(1024), 0, 0, d_seg, d_keys); }, mac256);
    run("ctr T2 1024x1 + mac 256",
        [&] { hipLaunchKernelGGL((k_ctr<2, 1024, 4>), dim3(kN / 1024), dim3(1024), 0, 0, d_seg, d_keys); }, mac256);
    run("ctr T2 1024x2 + mac 256",
        [&] { hipLaunchKernelGGL((k_ctr<2, 1024, 8>), dim3(kN / 1024), dim3(1024), 0, 0, d_seg, d_keys); }, mac256);
    run("ctr T2 768x2 + mac 256",
        [&] { hipLaunchKernelGGL((k_ctr<2, 768, 6>), dim3((kN + 767) / 768), dim3(768), 0, 0, d_seg, d_keys); },
        mac256);
    run("ctr T2 512x2 + mac 256",
        [&] { hipLaunchKernelGGL((k_ctr<2, 512, 4>), dim3(kN / 512), dim3(512), 0, 0, d_seg, d_keys); }, mac256);
    run("ctr T4 1024x1 + mac 64",
        [&] { hipLaunchKernelGGL((k_ctr<4, 1024, 4>), dim3(kN / 1024), dim3(1024), 0, 0, d_seg, d_keys); },
        [&] { hipLaunchKernelGGL((k_mac<64, 1>), dim3(kN / 64), dim3(64), 0, 0, d_seg, d_keys); });
    return 0;
}
