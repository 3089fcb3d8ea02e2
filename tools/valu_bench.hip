// valu_bench.hip -- issue-rate micro-benchmark for the instructions the AES/SHA-1
// loops are made of (v_perm_b32, v_bitop3_b32, v_alignbit_b32, v_add3_u32,
// v_xor_b32, ds_read_b32), 16 waves per CU as in k_protect.  Reports cycles
// per wave-instruction per SIMD from s_memtime deltas (shader clock).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP4(x) x x x x
// 8 independent accumulators: each instruction reads registers written 5-7
// instructions earlier, so issue rate (not latency) is measured.
#define B3(ins, sfx) REP4(ins " %0, %5, %6, %7" sfx "\n" ins " %1, %6, %7, %0" sfx "\n" ins " %2, %7, %0, %1" sfx "\n" ins " %3, %0, %1, %2" sfx "\n" \
                           ins " %4, %1, %2, %3" sfx "\n" ins " %5, %2, %3, %4" sfx "\n" ins " %6, %3, %4, %5" sfx "\n" ins " %7, %4, %5, %6" sfx "\n")
#define B2(ins) REP4(ins " %0, %5, %6\n" ins " %1, %6, %7\n" ins " %2, %7, %0\n" ins " %3, %0, %1\n" \
                     ins " %4, %1, %2\n" ins " %5, %2, %3\n" ins " %6, %3, %4\n" ins " %7, %4, %5\n")
#define BS(ins) REP4(ins " %0, %5, %6, %8\n" ins " %1, %6, %7, %8\n" ins " %2, %7, %0, %8\n" ins " %3, %0, %1, %8\n" \
                     ins " %4, %1, %2, %8\n" ins " %5, %2, %3, %8\n" ins " %6, %3, %4, %8\n" ins " %7, %4, %5, %8\n")
#define R8 "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]), "+v"(r[5]), "+v"(r[6]), "+v"(r[7])

template <int K>
__global__ __launch_bounds__(1024) void k_valu(uint32_t *out, uint64_t *cyc, int iters) {
    uint32_t r[8];
    for (int k = 0; k < 8; k++) r[k] = threadIdx.x * (k + 1) ^ (0x1234567u * k);
    uint32_t s0 = 0x0c020400u;
    __syncthreads();
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if (K == 0) asm volatile(B3("v_perm_b32", "") : R8);
        if (K == 1) asm volatile(B3("v_bitop3_b32", " bitop3:0x96") : R8);
        if (K == 2) asm volatile(B3("v_alignbit_b32", "") : R8);
        if (K == 3) asm volatile(B3("v_add3_u32", "") : R8);
        if (K == 4) asm volatile(B2("v_xor_b32") : R8);
        if (K == 5) asm volatile(B2("v_add_u32") : R8);
        if (K == 6) asm volatile(BS("v_perm_b32") : R8 : "s"(s0));
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int k = 0; k < 8; k++) x ^= r[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// ds_read_b32 throughput: lane l reads bank (l & 31) of a 128 KB LDS image
__global__ __launch_bounds__(1024) void k_lds(uint32_t *out, uint64_t *cyc, int iters) {
    __shared__ uint32_t s[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) s[i] = i;
    __syncthreads();
    uint32_t base = (threadIdx.x & 31u) << 2, acc = 0;
    uint32_t a0 = base, a1 = base + 128, a2 = base + 256, a3 = base + 384;
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        uint32_t r[16];
        asm volatile(
            "ds_read_b32 %0, %16\n ds_read_b32 %1, %17\n ds_read_b32 %2, %18\n ds_read_b32 %3, %19\n"
            "ds_read_b32 %4, %16 offset:512\n ds_read_b32 %5, %17 offset:512\n ds_read_b32 %6, %18 offset:512\n ds_read_b32 %7, %19 offset:512\n"
            "ds_read_b32 %8, %16 offset:1024\n ds_read_b32 %9, %17 offset:1024\n ds_read_b32 %10, %18 offset:1024\n ds_read_b32 %11, %19 offset:1024\n"
            "ds_read_b32 %12, %16 offset:1536\n ds_read_b32 %13, %17 offset:1536\n ds_read_b32 %14, %18 offset:1536\n ds_read_b32 %15, %19 offset:1536\n"
            "s_waitcnt lgkmcnt(0)\n"
            : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]),
              "=&v"(r[8]), "=&v"(r[9]), "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]), "=&v"(r[15])
            : "v"(a0), "v"(a1), "v"(a2), "v"(a3) : "memory");
        for (int k = 0; k < 16; k++) acc ^= r[k];
        a0 = (a0 + (acc & 0x7f00u)) & 0x1ff7cu; // data-dependent next address, same bank
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// mixed: 16 ds_read_b32 + 32 independent v_perm_b32 per iteration in one wave
__global__ __launch_bounds__(1024) void k_mix(uint32_t *out, uint64_t *cyc, int iters) {
    __shared__ uint32_t s[32768];
    for (int i = threadIdx.x; i < 32768; i += 1024) s[i] = i;
    __syncthreads();
    uint32_t base = (threadIdx.x & 31u) << 2, acc = 0;
    uint32_t a0 = base, a1 = base + 128, a2 = base + 256, a3 = base + 384;
    uint32_t r[8];
    for (int k = 0; k < 8; k++) r[k] = threadIdx.x * (k + 1);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        uint32_t q[16];
        asm volatile(
            "ds_read_b32 %0, %16\n ds_read_b32 %1, %17\n ds_read_b32 %2, %18\n ds_read_b32 %3, %19\n"
            "ds_read_b32 %4, %16 offset:512\n ds_read_b32 %5, %17 offset:512\n ds_read_b32 %6, %18 offset:512\n ds_read_b32 %7, %19 offset:512\n"
            "ds_read_b32 %8, %16 offset:1024\n ds_read_b32 %9, %17 offset:1024\n ds_read_b32 %10, %18 offset:1024\n ds_read_b32 %11, %19 offset:1024\n"
            "ds_read_b32 %12, %16 offset:1536\n ds_read_b32 %13, %17 offset:1536\n ds_read_b32 %14, %18 offset:1536\n ds_read_b32 %15, %19 offset:1536\n"
            : "=&v"(q[0]), "=&v"(q[1]), "=&v"(q[2]), "=&v"(q[3]), "=&v"(q[4]), "=&v"(q[5]), "=&v"(q[6]), "=&v"(q[7]),
              "=&v"(q[8]), "=&v"(q[9]), "=&v"(q[10]), "=&v"(q[11]), "=&v"(q[12]), "=&v"(q[13]), "=&v"(q[14]), "=&v"(q[15])
            : "v"(a0), "v"(a1), "v"(a2), "v"(a3) : "memory");
        asm volatile(B3("v_perm_b32", "") : R8);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int k = 0; k < 16; k++) acc ^= q[k];
        a0 = (a0 + (acc & 0x7f00u)) & 0x1ff7cu;
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = acc;
    for (int k = 0; k < 8; k++) x ^= r[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// one wave per CU (64-thread workgroups): K = 0, 32 independent v_add3_u32
// per iteration (8 accumulators, as B3); K = 1, a chain of 32 v_add3_u32 each
// reading the previous one's result; K = 2, the chain with one independent
// v_add3_u32 between each dependent pair (the SHA-1 compress loop's shape)
template <int K>
__global__ __launch_bounds__(1024) void k_one(uint32_t *out, uint64_t *cyc, int iters) {
    uint32_t r[8];
    for (int k = 0; k < 8; k++) r[k] = threadIdx.x * (k + 1) ^ (0x1234567u * k);
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; i++) {
        if (K == 0) asm volatile(B3("v_add3_u32", "") : R8);
        if (K == 1) asm volatile(REP4(REP4("v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %0, %0, %2, %1\n"))
                                 : "+v"(r[0]) : "v"(r[1]), "v"(r[2]));
        if (K == 2) asm volatile(REP4(REP4("v_add3_u32 %0, %0, %1, %2\n" "v_add3_u32 %3, %3, %2, %1\n"))
                                 : "+v"(r[0]), "+v"(r[3]) : "v"(r[1]), "v"(r[2]));
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t x = 0;
    for (int k = 0; k < 8; k++) x ^= r[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount, blocks = cus, iters = 2000;
    uint32_t *out; uint64_t *cyc; hipMalloc(&out, blocks * 1024 * 4); hipMalloc(&cyc, blocks * 8);
    uint64_t h[1024];
    const char *names[] = {"v_perm_b32(vgpr sel)", "v_bitop3_b32", "v_alignbit_b32", "v_add3_u32", "v_xor_b32", "v_add_u32", "v_perm_b32(sgpr sel)"};
    auto report = [&](const char *name, double instrs_per_wave_iter) {
        hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
        double avg = 0; for (int i = 0; i < blocks; i++) avg += h[i]; avg /= blocks;
        // 16 waves per CU = 4 per SIMD
        double per = avg / (iters * instrs_per_wave_iter * 4.0);
        printf("%-22s %7.2f cycles per wave-instruction per SIMD (4 waves/SIMD)\n", name, per);
    };
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto wall = [&](const char *name, auto &&launch, double wave_instrs) {
        launch(); hipDeviceSynchronize();
        hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
        double avg = 0; for (int i = 0; i < blocks; i++) avg += h[i]; avg /= blocks;
        // per CU: 16 waves x wave_instrs per iteration
        printf("%-22s wall %.3f ms: %.3f ns per wave-instr per CU;  memtime ticks/ns %.3f\n", name, ms,
               ms * 1e6 / (iters * 16.0 * wave_instrs), avg / (ms * 1e6));
    };
    wall("v_xor_b32", [&] { k_valu<4><<<blocks, 1024>>>(out, cyc, iters); }, 32);
    wall("v_perm_b32", [&] { k_valu<0><<<blocks, 1024>>>(out, cyc, iters); }, 32);
    wall("ds_read_b32", [&] { k_lds<<<blocks, 1024>>>(out, cyc, iters); }, 16);
    wall("mix 16ds+32perm", [&] { k_mix<<<blocks, 1024>>>(out, cyc, iters); }, 48);
    for (int rep = 0; rep < 2; rep++) {
        k_valu<0><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[0], 32);
        k_valu<1><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[1], 32);
        k_valu<2><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[2], 32);
        k_valu<3><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[3], 32);
        k_valu<4><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[4], 32);
        k_valu<5><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[5], 32);
        k_valu<6><<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize(); if (rep) report(names[6], 32);
        k_lds<<<blocks, 1024>>>(out, cyc, iters); hipDeviceSynchronize();
        if (rep) {
            hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
            double avg = 0; for (int i = 0; i < blocks; i++) avg += h[i]; avg /= blocks;
            printf("%-22s %7.2f CU cycles per wave-instruction (16 waves/CU)\n", "ds_read_b32", avg / (iters * 16.0 * 16));
        }
    }
    // a lone wave per CU: wall time per wave-instruction (events) and shader
    // clocks per wave-instruction (s_memtime)
    const char *one[] = {"one wave: 32 indep add3", "one wave: 32-add3 chain", "one wave: chain + indep"};
    for (int k = 0; k < 3; k++) {
        auto launch = [&] {
            if (k == 0) k_one<0><<<blocks, 64>>>(out, cyc, iters);
            if (k == 1) k_one<1><<<blocks, 64>>>(out, cyc, iters);
            if (k == 2) k_one<2><<<blocks, 64>>>(out, cyc, iters);
        };
        launch(); hipDeviceSynchronize();
        hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
        double avg = 0; for (int i = 0; i < blocks; i++) avg += h[i]; avg /= blocks;
        printf("%-26s %.3f ns per wave-instr (wall), %.2f memtime ticks per wave-instr\n", one[k],
               ms * 1e6 / (iters * 32.0), avg / (iters * 32.0));
    }
    // the independent add3 stream with 1, 2, 4, 8, 16 waves per CU (one
    // workgroup per CU): each wave's time per instruction -- how many waves
    // the SIMDs give their single-wave issue rate before they share
    for (int w = 1; w <= 16; w *= 2) {
        auto launch = [&] { k_one<0><<<blocks, 64 * w>>>(out, cyc, iters); };
        launch(); hipDeviceSynchronize();
        hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%2d waves/CU: 32 indep add3 %.3f ns per wave-instr per wave (wall)\n", w, ms * 1e6 / (iters * 32.0));
    }
    hipError_t e = hipGetLastError();
    printf("status: %s\n", hipGetErrorString(e));
    return 0;
}
