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
//   line_bench [reps]   -> one JSON line per (mode, stride, delay)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int kPackets = 1 << 18, kChunks = 19, kThreads = 1024;
constexpr int kTableWords = 16384; // 64 KB stands in for the T-table image

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ uint32_t spin(uint32_t x, int n) {
#pragma unroll 1
    for (int i = 0; i < n; i++) x = __builtin_amdgcn_alignbit(x, x ^ 0x9e3779b9u, 7) + 0x7f4a7c15u;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_lines(uint8_t *seg, uint32_t stride, int delay) {
    // 64 KB "table" + 64 KB staging (16 waves x 64 lanes x 64 B): 128 KB, one WG per CU
    __shared__ uint4 s_tab[kTableWords / 4];
    __shared__ uint4 s_stage[kThreads * 4];
    if (threadIdx.x == 0) s_tab[0] = make_uint4(0, 0, 0, 0);
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    uint8_t *pkt = seg + (size_t)p * stride;
    uint32_t acc = p;
    uint4 hold[4];
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
            for (int mode = 0; mode < 3; mode++) {
                auto launch = [&] {
                    if (mode == 0) hipLaunchKernelGGL(k_lines<0>, dim3(kPackets / kThreads), dim3(kThreads), 0, 0, seg, stride, delay);
                    else if (mode == 1) hipLaunchKernelGGL(k_lines<1>, dim3(kPackets / kThreads), dim3(kThreads), 0, 0, seg, stride, delay);
                    else hipLaunchKernelGGL(k_lines<2>, dim3(kPackets / kThreads), dim3(kThreads), 0, 0, seg, stride, delay);
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
