// line_bench.hip -- does the AES kernels' memory pattern waste HBM traffic
// because each 128-B line is read in two 64-B halves a whole chunk step apart
// (not product code)?  2^18 packets of 1200 B at a stride of 1216 B (the
// bench segment: packet starts alternate between 0 and 64 mod 128) or 1280 B
// (every packet line-aligned).  One lane per packet, 1024-thread workgroups
// holding 128 KB of LDS (one per CU, as k_protect), read-modify-write of 19
// 64-B chunks per packet with D dependent VALU operations per chunk step
// standing in for the crypto (so a step lasts as long as in the kernel).
//   mode 0: each step loads its 64-B chunk (the kernels' pattern today)
//   mode 1: even steps load 128 B (chunks b and b+1) into registers
//   mode 2: even steps load chunk b into registers and chunk b+1 into the
//           wave's LDS staging area (ds_write_b128), odd steps read it back
//   mode 3: quad-coalesced LDS-DMA loads (global_load_lds_dwordx4: lane 4q+m
//           fetches piece m of packet 4q+i's chunk, so one instruction covers
//           16 whole 64-B chunks) of chunk b+1 issued as soon as chunk b has
//           been read from the wave's staging area; per-lane stores
//   mode 4: as 3, but the results go back through the staging area and out
//           as quad-coalesced stores (the DMA of chunk b+1 then waits for them)
//   mode 5: per-lane loads (mode 0), quad-coalesced stores through the staging area
//   mode 6: per-lane loads, quad-coalesced stores after a DPP 4x4 transpose in the quad
//   line_bench [reps]   -> one JSON line per (mode, stride, delay)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kPackets = 1 << 18, kChunks = 19, kThreads = 1024;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 as_u4(u32x4 t) { return make_uint4(t.x, t.y, t.z, t.w); }
__device__ __forceinline__ u32x4 as_v4(uint4 t) { return u32x4{t.x, t.y, t.z, t.w}; }
constexpr int kTableWords = 16384; // 64 KB stands in for the T-table image

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

// LDS-DMA of 16 B per lane: LDS[lds + 16 * lane] = *src (the guide's glds16 recipe)
__device__ __forceinline__ void glds16(const void *src, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}

template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
// r[reg][lane-in-quad] transposed over the quad (two stages of quad_perm swaps)
__device__ __forceinline__ void quad_transpose4(uint32_t r[4], uint32_t lane) {
    {   // stage 1: swap with lane ^ 1
        const bool hi = lane & 1u;
        const uint32_t a1 = qdpp<0xB1>(r[1]), a0 = qdpp<0xB1>(r[0]), a3 = qdpp<0xB1>(r[3]), a2 = qdpp<0xB1>(r[2]);
        const uint32_t n0 = hi ? a1 : r[0], n1 = hi ? r[1] : a0, n2 = hi ? a3 : r[2], n3 = hi ? r[3] : a2;
        r[0] = n0; r[1] = n1; r[2] = n2; r[3] = n3;
    }
    {   // stage 2: swap with lane ^ 2
        const bool hi = lane & 2u;
        const uint32_t a2 = qdpp<0x4E>(r[2]), a0 = qdpp<0x4E>(r[0]), a3 = qdpp<0x4E>(r[3]), a1 = qdpp<0x4E>(r[1]);
        const uint32_t n0 = hi ? a2 : r[0], n2 = hi ? r[2] : a0, n1 = hi ? a3 : r[1], n3 = hi ? r[3] : a1;
        r[0] = n0; r[1] = n1; r[2] = n2; r[3] = n3;
    }
}

__device__ __forceinline__ uint32_t spin(uint32_t x, int n) {
#pragma unroll 1
    for (int i = 0; i < n; i++) x = __builtin_amdgcn_alignbit(x, x ^ 0x9e3779b9u, 7) + 0x7f4a7c15u;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_lines(uint8_t *seg, uint32_t stride, int delay) {
    // 64 KB "table" + 64 KB staging (16 waves x 64 lanes x 64 B): 128 KB, one WG per CU
    __shared__ uint4 s_tab[kTableWords / 4];
    __shared__ uint4 s_stage[kThreads * 4 + 64]; // 16 waves x 4160 B for modes 3-4
    if (threadIdx.x == 0) s_tab[0] = make_uint4(0, 0, 0, 0);
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    uint8_t *pkt = seg + (size_t)p * stride;
    uint32_t acc = p;
    uint4 hold[4];
    if (MODE == 5 || MODE == 6) {
        const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
        const uint32_t q = lane >> 2, m = lane & 3u;
        const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)((uint32_t)(uintptr_t)s_stage + wv * 4160u));
        uint8_t *wseg = seg + (size_t)(blockIdx.x * kThreads + (threadIdx.x & ~63u)) * stride;
        auto dst = [&](int b, int i) { return wseg + (size_t)(4 * q + i) * stride + 64 * b + 16 * m; };
        const uint32_t rd = base + (lane & 3u) * 1040u + (lane >> 2) * 64u;
        for (int b = 0; b < kChunks; b++) {
            acc = spin(acc, delay);
            const uint4 *qi = reinterpret_cast<const uint4 *>(pkt + 64 * b);
            uint4 v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = qi[j];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j].x ^= acc & 1u;
            if (MODE == 5) {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(rd), "v"(as_v4(v[j])), "i"(16 * j) : "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    u32x4 t;
                    asm volatile("ds_read_b128 %0, %1" : "=v"(t) : "v"(base + 1040u * i + 16u * lane) : "memory");
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    *reinterpret_cast<uint4 *>(dst(b, i)) = as_u4(t);
                }
            } else {
                // d[4j + e] = word e of piece j; after the transpose of each word
                // column e across the quad, lane m holds word e of piece m of packet 4q+j
                uint32_t w[4][4];
#pragma unroll
                for (int e = 0; e < 4; e++) {
                    uint32_t r[4] = {(&v[0].x)[e], (&v[1].x)[e], (&v[2].x)[e], (&v[3].x)[e]};
                    quad_transpose4(r, lane);
#pragma unroll
                    for (int j = 0; j < 4; j++) w[j][e] = r[j];
                }
#pragma unroll
                for (int i = 0; i < 4; i++)
                    *reinterpret_cast<uint4 *>(dst(b, i)) = make_uint4(w[i][0], w[i][1], w[i][2], w[i][3]);
            }
        }
        if (acc == 0x12345678u) s_tab[threadIdx.x & 7].x = acc;
        return;
    }
    if (MODE >= 3) { // staging area of this wave: 4 slots of 1 KB (+16 B skew each)
        const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
        const uint32_t q = lane >> 2, m = lane & 3u;
        const uint32_t base = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)((uint32_t)(uintptr_t)s_stage + wv * 4160u));
        uint8_t *wseg = seg + (size_t)(blockIdx.x * kThreads + (threadIdx.x & ~63u)) * stride;
        // lane 4q+m, slot i: piece m of packet 4q+i of the wave
        auto src = [&](int b, int i) { return wseg + (size_t)(4 * q + i) * stride + 64 * b + 16 * m; };
        // own packet P = lane reads piece j from slot (P & 3), lane 4(P>>2)+j
        const uint32_t rd = base + (lane & 3u) * 1040u + (lane >> 2) * 64u;
#pragma unroll
        for (int i = 0; i < 4; i++) glds16(src(0, i), base + 1040u * i);
        for (int b = 0; b < kChunks; b++) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint4 v[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                u32x4 t;
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(t) : "v"(rd), "i"(16 * j) : "memory");
                v[j] = as_u4(t);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (MODE == 3 && b + 1 < kChunks) {
#pragma unroll
                for (int i = 0; i < 4; i++) glds16(src(b + 1, i), base + 1040u * i);
            }
            acc = spin(acc, delay);
#pragma unroll
            for (int j = 0; j < 4; j++) v[j].x ^= acc & 1u;
            if (MODE == 3) {
                uint4 *qo = reinterpret_cast<uint4 *>(pkt + 64 * b);
#pragma unroll
                for (int j = 0; j < 4; j++) qo[j] = v[j];
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    asm volatile("ds_write_b128 %0, %1 offset:%2" :: "v"(rd), "v"(as_v4(v[j])), "i"(16 * j) : "memory");
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    u32x4 t;
                    asm volatile("ds_read_b128 %0, %1" : "=v"(t) : "v"(base + 1040u * i + 16u * lane) : "memory");
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    *reinterpret_cast<uint4 *>(src(b, i)) = as_u4(t);
                }
                if (b + 1 < kChunks) {
#pragma unroll
                    for (int i = 0; i < 4; i++) glds16(src(b + 1, i), base + 1040u * i);
                }
            }
        }
        if (acc == 0x12345678u) s_tab[threadIdx.x & 7].x = acc;
        return;
    }
    for (int b = 0; b < kChunks; b++) {
        acc = spin(acc, delay);
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 64 * b);
        uint4 v[4];
        if (MODE == 0 || b == kChunks - 1 && (b & 1) == 0) {
#pragma unroll
            for (int m = 0; m < 4; m++) v[m] = q[m];
        } else if ((b & 1) == 0) {
#pragma unroll
            for (int m = 0; m < 4; m++) v[m] = q[m];
            if (MODE == 1) {
#pragma unroll
                for (int m = 0; m < 4; m++) hold[m] = q[4 + m];
            } else {
                uint4 t[4];
#pragma unroll
                for (int m = 0; m < 4; m++) t[m] = q[4 + m];
#pragma unroll
                for (int m = 0; m < 4; m++) s_stage[m * kThreads + threadIdx.x] = t[m];
            }
        } else {
            if (MODE == 1) {
#pragma unroll
                for (int m = 0; m < 4; m++) v[m] = hold[m];
            } else {
#pragma unroll
                for (int m = 0; m < 4; m++) v[m] = s_stage[m * kThreads + threadIdx.x];
            }
        }
#pragma unroll
        for (int m = 0; m < 4; m++) {
            v[m].x ^= acc & 1u;
            q[m] = v[m];
        }
    }
    if (acc == 0x12345678u) s_tab[threadIdx.x & 7].x = acc; // keep the spin
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const size_t bytes = (size_t)kPackets * 1280 + 4096;
    uint8_t *seg;
    CHECK(hipMalloc(&seg, bytes));
    CHECK(hipMemset(seg, 1, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int delays[] = {0, 150, 300};
    const uint32_t strides[] = {1216, 1280};
    for (int delay : delays)
        for (uint32_t stride : strides)
            for (int mode = 0; mode < 7; mode++) {
                auto launch = [&] {
                    const dim3 g(kPackets / kThreads), t(kThreads);
                    if (mode == 0) hipLaunchKernelGGL(k_lines<0>, g, t, 0, 0, seg, stride, delay);
                    else if (mode == 1) hipLaunchKernelGGL(k_lines<1>, g, t, 0, 0, seg, stride, delay);
                    else if (mode == 2) hipLaunchKernelGGL(k_lines<2>, g, t, 0, 0, seg, stride, delay);
                    else if (mode == 3) hipLaunchKernelGGL(k_lines<3>, g, t, 0, 0, seg, stride, delay);
                    else if (mode == 4) hipLaunchKernelGGL(k_lines<4>, g, t, 0, 0, seg, stride, delay);
                    else if (mode == 5) hipLaunchKernelGGL(k_lines<5>, g, t, 0, 0, seg, stride, delay);
                    else hipLaunchKernelGGL(k_lines<6>, g, t, 0, 0, seg, stride, delay);
                };
                for (int r = 0; r < 3; r++) launch();
                CHECK(hipEventRecord(e0));
                for (int r = 0; r < reps; r++) launch();
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double us = 1e3 * ms / reps;
                const double moved = 2.0 * kPackets * 64.0 * kChunks;
                printf("{\"mode\": %d, \"stride\": %u, \"delay\": %d, \"us\": %.1f, \"tbps\": %.2f}\n", mode,
                       stride, delay, us, moved / us / 1e6);
                fflush(stdout);
            }
    return 0;
}
