// aes_bench.hip -- AES-128 CTR keystream throughput of the T-table round variants
// (tools/gen_aes_bench.py): blocks interleaved per wave (2 / 4), LDS tables
// (4 x 32 copies = 128 KB, or 2 x 32 copies = 64 KB + rotations), workgroup
// size and occupancy.  Every lane computes `nblk` counter blocks of its own IV
// and XOR-folds them; all variants must produce identical output, checked
// against a byte-wise host AES for a few lanes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ uint32_t d_te0[256];

#include "aes_bench_rounds.inc"

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) { return n ? __builtin_amdgcn_alignbit(x, x, 32u - n) : x; }
__device__ __forceinline__ uint32_t sgpr(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

template <int NB, int T>
__device__ __forceinline__ void mid(uint32_t (*s)[4], const uint32_t *bs, const uint32_t *rk) {
    if constexpr (NB == 2 && T == 4) aes_mid_n2_t4(s[0], s[1], bs, rk);
    if constexpr (NB == 2 && T == 2) aes_mid_n2_t2(s[0], s[1], bs, rk);
    if constexpr (NB == 4 && T == 4) aes_mid_n4_t4(s[0], s[1], s[2], s[3], bs, rk);
    if constexpr (NB == 4 && T == 2) aes_mid_n4_t2(s[0], s[1], s[2], s[3], bs, rk);
}
template <int NB, int T>
__device__ __forceinline__ void last(uint32_t (*s)[4], const uint32_t *bs, const uint32_t *rk) {
    if constexpr (NB == 2 && T == 4) aes_last_n2_t4(s[0], s[1], bs, rk);
    if constexpr (NB == 2 && T == 2) aes_last_n2_t2(s[0], s[1], bs, rk);
    if constexpr (NB == 4 && T == 4) aes_last_n4_t4(s[0], s[1], s[2], s[3], bs, rk);
    if constexpr (NB == 4 && T == 2) aes_last_n4_t2(s[0], s[1], s[2], s[3], bs, rk);
}

template <int NB, int T, int THREADS, int MINW>
__global__ __launch_bounds__(THREADS, MINW) void k_aes(uint32_t *out, const uint32_t *rkg, int nblk) {
    constexpr int WORDS = T == 4 ? 32768 : 16384;
    __shared__ uint32_t s_te[WORDS];
    for (int i = threadIdx.x; i < WORDS; i += THREADS) {
        const int t = T == 4 ? (((i >> 14) << 1) | ((i >> 5) & 1)) : ((i >> 5) & 1);
        s_te[i] = rotl(d_te0[(i >> 6) & 255], 8u * (uint32_t)t);
    }
    __syncthreads();
    asm volatile("" ::"s"(s_te) : "memory");
    const uint32_t c4 = (threadIdx.x & 31u) << 2;
    uint32_t bs[4];
#pragma unroll
    for (int t = 0; t < 4; t++)
        bs[t] = T == 4 ? ((uint32_t)((t >> 1) << 16) | (uint32_t)((t & 1) << 7) | c4)
                       : ((uint32_t)((t & 1) << 7) | c4);
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; i++) rk[i] = sgpr(rkg[i]);
    const uint32_t gid = blockIdx.x * THREADS + threadIdx.x;
    const uint32_t iv[4] = {gid, 0x01234567u, 0x89abcdefu ^ (gid * 3u), 0x0000a5a5u};
    uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll 1
    for (int j = 0; j < nblk; j += NB) {
        uint32_t s[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++) {
            const uint32_t c = (uint32_t)(j + b);
            s[b][0] = iv[0] ^ rk[0]; s[b][1] = iv[1] ^ rk[1]; s[b][2] = iv[2] ^ rk[2];
            s[b][3] = (iv[3] | (((c >> 8) & 0xffu) << 16) | ((c & 0xffu) << 24)) ^ rk[3];
        }
#pragma unroll
        for (int r = 1; r < 10; r++) mid<NB, T>(s, bs, rk + 4 * r);
        last<NB, T>(s, bs, rk + 40);
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] ^= s[b][k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) out[4 * gid + k] = acc[k];
}

// ---------------------------------------------------------------- AES + SHA-1 mix
__device__ __forceinline__ void sha1c(uint32_t h[5], uint32_t w[16]) {
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
        uint32_t wt;
        if (t < 16) wt = w[t];
        else { wt = rotl(__builtin_amdgcn_bitop3_b32(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15], 0x96) ^ w[t & 15], 1); w[t & 15] = wt; }
        uint32_t f, k;
        if (t < 20) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); k = 0x5A827999u; }
        else if (t < 40) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0x6ED9EBA1u; }
        else if (t < 60) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); k = 0x8F1BBCDCu; }
        else { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96); k = 0xCA62C1D6u; }
        uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// MODE 0: every wave per step: 4 AES blocks then 1 SHA-1 compression.
// MODE 1: waves in two groups ((wave >> 2) & 1), two phases per step with a
//         workgroup barrier between: a group does its 4 AES blocks while the
//         other does its SHA-1 compression, then they swap.
template <int MODE>
__global__ __launch_bounds__(1024) void k_mix(uint32_t *out, const uint32_t *rkg, int steps) {
    __shared__ uint32_t s_te[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) {
        const int t = ((i >> 14) << 1) | ((i >> 5) & 1);
        s_te[i] = rotl(d_te0[(i >> 6) & 255], 8u * (uint32_t)t);
    }
    __syncthreads();
    asm volatile("" ::"s"(s_te) : "memory");
    const uint32_t c4 = (threadIdx.x & 31u) << 2;
    uint32_t bs[4];
#pragma unroll
    for (int t = 0; t < 4; t++) bs[t] = (uint32_t)((t >> 1) << 16) | (uint32_t)((t & 1) << 7) | c4;
    uint32_t rk[44];
#pragma unroll
    for (int i = 0; i < 44; i++) rk[i] = sgpr(rkg[i]);
    const uint32_t gid = blockIdx.x * 1024 + threadIdx.x;
    const uint32_t iv[4] = {gid, 0x01234567u, 0x89abcdefu ^ (gid * 3u), 0x0000a5a5u};
    uint32_t acc[4] = {0, 0, 0, 0}, h[5] = {gid, 1, 2, 3, 4}, w[16];
#pragma unroll
    for (int k = 0; k < 16; k++) w[k] = gid * 7u + k;
    const int grp = (threadIdx.x >> 8) & 1;
    auto aes4 = [&](int j) {
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {
            uint32_t s[2][4];
#pragma unroll
            for (int b = 0; b < 2; b++) {
                const uint32_t c = (uint32_t)(j + 2 * pr + b);
                s[b][0] = iv[0] ^ rk[0]; s[b][1] = iv[1] ^ rk[1]; s[b][2] = iv[2] ^ rk[2];
                s[b][3] = (iv[3] | (((c >> 8) & 0xffu) << 16) | ((c & 0xffu) << 24)) ^ rk[3];
            }
#pragma unroll
            for (int r = 1; r < 10; r++) mid<2, 4>(s, bs, rk + 4 * r);
            last<2, 4>(s, bs, rk + 40);
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int k = 0; k < 4; k++) acc[k] ^= s[b][k];
        }
    };
    auto sha = [&]() {
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] ^= acc[k & 3];
        sha1c(h, w);
    };
#pragma unroll 1
    for (int st = 0; st < steps; st++) {
        if (MODE == 0) {
            aes4(4 * st);
            sha();
        } else {
            if (grp == 0) aes4(4 * st); else sha();
            __syncthreads();
            if (grp == 0) sha(); else aes4(4 * st);
            __syncthreads();
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) out[4 * gid + k] = acc[k] ^ h[k] ^ h[4];
}

// ---------------------------------------------------------------- host AES
static uint8_t SB[256];
static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }
static void make_sbox() {
    uint8_t p = 1, q = 1;
    do {
        p = p ^ (uint8_t)(p << 1) ^ ((p & 0x80) ? 0x1b : 0);
        q ^= q << 1; q ^= q << 2; q ^= q << 4; if (q & 0x80) q ^= 0x09;
        uint8_t x = q ^ (uint8_t)((q << 1) | (q >> 7)) ^ (uint8_t)((q << 2) | (q >> 6)) ^
                    (uint8_t)((q << 3) | (q >> 5)) ^ (uint8_t)((q << 4) | (q >> 4));
        SB[p] = x ^ 0x63;
    } while (p != 1);
    SB[0] = 0x63;
}
static void expand(const uint8_t key[16], uint8_t rk[176]) {
    memcpy(rk, key, 16);
    uint8_t rc = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t u = t[0];
            t[0] = SB[t[1]] ^ rc; t[1] = SB[t[2]]; t[2] = SB[t[3]]; t[3] = SB[u];
            rc = xt(rc);
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 4) + k] ^ t[k];
    }
}
static void enc(const uint8_t rk[176], uint8_t s[16]) {
    for (int i = 0; i < 16; i++) s[i] ^= rk[i];
    for (int r = 1; r <= 10; r++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int w = 0; w < 4; w++) t[4 * c + w] = SB[s[4 * ((c + w) & 3) + w]];
        if (r < 10)
            for (int c = 0; c < 4; c++) {
                uint8_t *a = t + 4 * c, a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], x = a0 ^ a1 ^ a2 ^ a3;
                a[0] ^= x ^ xt(a0 ^ a1); a[1] ^= x ^ xt(a1 ^ a2); a[2] ^= x ^ xt(a2 ^ a3); a[3] ^= x ^ xt(a3 ^ a0);
            }
        for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk[16 * r + i];
    }
}

struct Variant {
    const char *name;
    void (*launch)(int grid, uint32_t *out, const uint32_t *rk, int nblk);
    const void *fn;
    int threads;
};

template <int NB, int T, int TH, int MW>
static void launch(int grid, uint32_t *out, const uint32_t *rk, int nblk) {
    hipLaunchKernelGGL((k_aes<NB, T, TH, MW>), dim3(grid), dim3(TH), 0, 0, out, rk, nblk);
}
#define V(name, NB, T, TH, MW) {name, launch<NB, T, TH, MW>, (const void *)k_aes<NB, T, TH, MW>, TH}

int main() {
    make_sbox();
    uint32_t te0[256];
    for (int x = 0; x < 256; x++) {
        uint8_t s = SB[x], s2 = xt(s), s3 = s2 ^ s;
        te0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
    CHECK(hipMemcpyToSymbol(HIP_SYMBOL(d_te0), te0, sizeof te0));
    uint8_t key[16], rkb[176];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(0x2b + 17 * i);
    expand(key, rkb);
    uint32_t rkw[44];
    memcpy(rkw, rkb, 176);  // little-endian column words
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const int nblk = 76 * 8;
    Variant vs[] = {
        V("n2_t4_1024 (product)", 2, 4, 1024, 1),
        V("n4_t4_1024", 4, 4, 1024, 1),
        V("n2_t2_1024_8w", 2, 2, 1024, 8),
        V("n2_t2_512_4w", 2, 2, 512, 4),
        V("n4_t2_1024_6w", 4, 2, 1024, 5),
        V("n2_t2_768_6w", 2, 2, 768, 6),
        V("n2_t4_768", 2, 4, 768, 1),
        V("n2_t4_512", 2, 4, 512, 1),
        V("n4_t4_768", 4, 4, 768, 1),
        V("n4_t4_512", 4, 4, 512, 1),
    };
    const int nv = sizeof vs / sizeof vs[0];
    uint32_t *d_rk, *d_out;
    CHECK(hipMalloc(&d_rk, sizeof rkw));
    CHECK(hipMemcpy(d_rk, rkw, sizeof rkw, hipMemcpyHostToDevice));
    const size_t max_lanes = (size_t)cus * 2048;
    CHECK(hipMalloc(&d_out, max_lanes * 16));
    std::vector<uint32_t> ref;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int v = 0; v < nv; v++) {
        int per_cu = 0;
        CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, vs[v].fn, vs[v].threads, 0));
        if (per_cu < 1) { printf("%-24s does not fit\n", vs[v].name); continue; }
        const int grid = cus * per_cu;
        const size_t lanes = (size_t)grid * vs[v].threads;
        vs[v].launch(grid, d_out, d_rk, nblk);
        CHECK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            CHECK(hipEventRecord(e0));
            vs[v].launch(grid, d_out, d_rk, nblk);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        std::vector<uint32_t> h(lanes * 4);
        CHECK(hipMemcpy(h.data(), d_out, lanes * 16, hipMemcpyDeviceToHost));
        int bad = 0;
        for (size_t lane : {(size_t)0, (size_t)1, (size_t)777, lanes - 1}) {
            uint32_t acc[4] = {0, 0, 0, 0};
            const uint32_t gid = (uint32_t)lane;
            const uint32_t iv[4] = {gid, 0x01234567u, 0x89abcdefu ^ (gid * 3u), 0x0000a5a5u};
            for (int j = 0; j < nblk; j++) {
                uint32_t w[4] = {iv[0], iv[1], iv[2], iv[3] | (((uint32_t)j >> 8 & 0xff) << 16) | (((uint32_t)j & 0xff) << 24)};
                uint8_t s[16];
                memcpy(s, w, 16);
                enc(rkb, s);
                memcpy(w, s, 16);
                for (int k = 0; k < 4; k++) acc[k] ^= w[k];
            }
            for (int k = 0; k < 4; k++) bad += acc[k] != h[4 * lane + k];
        }
        const double blocks = (double)lanes * nblk;
        const double ns_per_block_cu = best * 1e6 / (blocks / cus);
        printf("%-24s wg/CU %d  %8.3f ms  %7.1f Gblk/s  %6.3f ns/blk/CU (%5.2f cyc @2.1GHz)  %s\n",
               vs[v].name, per_cu, best, blocks / best / 1e6, ns_per_block_cu, ns_per_block_cu * 2.1,
               bad ? "MISMATCH" : "ok");
    }
    for (int mode = 0; mode < 2; mode++) {
        const int steps = 152;
        float best = 1e30f;
        for (int rep = 0; rep < 4; rep++) {
            CHECK(hipEventRecord(e0));
            if (mode == 0) hipLaunchKernelGGL(k_mix<0>, dim3(cus), dim3(1024), 0, 0, d_out, d_rk, steps);
            else hipLaunchKernelGGL(k_mix<1>, dim3(cus), dim3(1024), 0, 0, d_out, d_rk, steps);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        const double blocks = (double)cus * 1024 * steps * 4;
        printf("mix %s: %.3f ms  %.3f ns/blk/CU (4 AES blocks + 1 SHA-1 compression per lane-step)\n",
               mode ? "phase-split" : "fused      ", best, best * 1e6 / (blocks / cus));
    }
    return 0;
}
