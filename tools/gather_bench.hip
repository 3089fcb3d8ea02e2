// gather_bench.hip -- could the vector L1 (TCP) serve part of the AES
// T-table lookups beside the LDS (not product code)?  Random 4-byte lookups
// from a 256-entry (1 KB) table, per lane, dependent in chains of 8 like an
// AES round's columns, one 1024-thread workgroup per CU holding 128 KB of LDS
// (as the AES kernels).  Modes:
//   lds   : every lookup a ds_read_b32 from a 32x-replicated LDS image
//   l1    : every lookup a global_load_dword from the 1-KB table (L1-resident)
//   mix:k : k of every 8 lookups from L1, the rest from LDS
// Prints lookups per CU per clock (2.4 GHz assumed) and the time per launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                                               \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);                   \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

constexpr int kThreads = 1024, kIters = 2048, kChains = 8;

template <int NL1>
__global__ __launch_bounds__(kThreads) void k_gather(const uint32_t *__restrict__ tab, uint32_t *out) {
    __shared__ uint32_t s_te[32768]; // 128 KB: 256 entries x 32 replicas x 4 tables
    for (int i = threadIdx.x; i < 32768; i += kThreads) s_te[i] = tab[(i >> 5) & 255] ^ (uint32_t)(i >> 13);
    __syncthreads();
    const uint32_t lane32 = threadIdx.x & 31u;
    uint32_t x[kChains];
#pragma unroll
    for (int c = 0; c < kChains; c++) x[c] = (blockIdx.x * kThreads + threadIdx.x) * 2654435761u + c * 40503u;
#pragma unroll 1
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) {
            const uint32_t idx = (x[c] >> 8) & 255u;
            uint32_t v;
            if (c < NL1) v = tab[idx];
            else v = s_te[(idx << 5) | lane32];
            x[c] = (x[c] << 3 | x[c] >> 29) ^ v;
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int c = 0; c < kChains; c++) r ^= x[c];
    if (r == 0x12345678u) out[0] = r;
}

int main() {
    uint32_t *tab, *out;
    CHECK(hipMalloc(&tab, 4096));
    CHECK(hipMalloc(&out, 64));
    uint32_t h[1024];
    for (int i = 0; i < 1024; i++) h[i] = i * 2654435761u;
    CHECK(hipMemcpy(tab, h, sizeof h, hipMemcpyHostToDevice));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto kern) {
        for (int r = 0; r < 2; r++) hipLaunchKernelGGL(kern, dim3(cus), dim3(kThreads), 0, 0, tab, out);
        CHECK(hipEventRecord(e0));
        const int reps = 5;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(cus), dim3(kThreads), 0, 0, tab, out);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        const double lookups_per_cu = (double)kThreads * kIters * kChains;
        printf("{\"mode\": \"%s\", \"us\": %.1f, \"lookups_per_cu_per_clk\": %.2f}\n", name, us,
               lookups_per_cu / (us * 1e-6 * 2.4e9));
        fflush(stdout);
        return 0;
    };
    run("lds", k_gather<0>);
    run("mix:1", k_gather<1>);
    run("mix:2", k_gather<2>);
    run("mix:3", k_gather<3>);
    run("mix:4", k_gather<4>);
    run("l1", k_gather<8>);
    return 0;
}
