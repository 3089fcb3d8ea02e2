// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the access
// pattern of the packet kernels (one lane per packet, 16-B loads/stores walking
// a 1200-B packet at a 1216-B slot stride) against a coalesced stream of the
// same bytes, and time each.  Run under `rocprofv3 --pmc FETCH_SIZE` and
// `--pmc WRITE_SIZE` (separate passes) plus `--kernel-trace --stats`.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#ifndef STRIDE
#define STRIDE 1216
#endif
constexpr int kN = 262144, kLen = 1200, kStride = STRIDE;

__global__ void k_stream_rd(const uint4 *src, size_t n16, uint32_t *out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_stream_rw(uint4 *buf, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 v = buf[i];
        v.x ^= 0x5a5a5a5au;
        buf[i] = v;
    }
}

// one lane per packet, 4 x 16 B per 64-B chunk (the k_protect pattern)
__global__ __launch_bounds__(1024) void k_lane_rd(const uint8_t *seg, uint32_t *out) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kN) return;
    const uint4 *q = reinterpret_cast<const uint4 *>(seg + (size_t)p * kStride);
    uint32_t acc = 0;
    for (int b = 0; b < kLen / 16; b++) {
        uint4 v = q[b];
        acc = (acc << 1 | acc >> 31) ^ v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(1024) void k_lane_rw(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kN) return;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 16; b++) {
        uint4 v = q[b];
        v.x ^= 0x5a5a5a5au ^ (uint32_t)b;
        q[b] = v;
    }
}

// one lane per packet, chunk-major: lanes of a wave walk their packets in
// lockstep 64 B at a time (same as k_lane_rw, but 4 loads in flight)
__global__ __launch_bounds__(1024) void k_lane_rw4(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kN) return;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 64; b++) {
        uint4 v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m] = q[4 * b + m];
#pragma unroll
        for (int m = 0; m < 4; m++) { v[m].y ^= 0xa5a5a5a5u; q[4 * b + m] = v[m]; }
    }
}

// 4x4 transpose of 16-B quads among lanes 4g..4g+3 (two DPP butterfly
// stages): afterwards lane 4g+k holds quad k of the packets of lanes 4g..4g+3,
// so store i writes 64 contiguous bytes of packet 4g+i per 4 lanes.
__device__ __forceinline__ uint32_t xlane(uint32_t v, int ctrl_x1) {
    return ctrl_x1 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xb1, 0xf, 0xf, false)   // quad_perm [1,0,3,2]
                   : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4e, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
}
__device__ __forceinline__ void quad_transpose(uint4 v[4]) {
    const int k = threadIdx.x & 3;
    // stage 1: exchange quads differing in bit 0 (lane ^1, quad ^1)
    for (int pair = 0; pair < 2; pair++) {
        uint4 &a = v[2 * pair], &b = v[2 * pair + 1];
        const bool hi = k & 1;
        uint4 send = hi ? a : b;
        uint4 got;
        got.x = xlane(send.x, 1); got.y = xlane(send.y, 1); got.z = xlane(send.z, 1); got.w = xlane(send.w, 1);
        if (hi) a = got; else b = got;
    }
    // stage 2: exchange quads differing in bit 1 (lane ^2, quad ^2)
    for (int q = 0; q < 2; q++) {
        uint4 &a = v[q], &b = v[q + 2];
        const bool hi = k & 2;
        uint4 send = hi ? a : b;
        uint4 got;
        got.x = xlane(send.x, 0); got.y = xlane(send.y, 0); got.z = xlane(send.z, 0); got.w = xlane(send.w, 0);
        if (hi) a = got; else b = got;
    }
}

__global__ __launch_bounds__(1024) void k_lane_rw4t(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t g0 = p & ~3u; const int k = threadIdx.x & 3;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 64; b++) {
        uint4 v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m] = q[4 * b + m];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m].y ^= 0xa5a5a5a5u;
        quad_transpose(v);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint4 *d = reinterpret_cast<uint4 *>(seg + (size_t)(g0 + i) * kStride);
            d[4 * b + k] = v[i];
        }
    }
}

__global__ __launch_bounds__(1024) void k_lane_rw8(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 128; b++) {
        uint4 v[8];
#pragma unroll
        for (int m = 0; m < 8; m++) v[m] = q[8 * b + m];
#pragma unroll
        for (int m = 0; m < 8; m++) { v[m].y ^= 0xa5a5a5a5u; q[8 * b + m] = v[m]; }
    }
}

__global__ __launch_bounds__(1024) void k_lane_w4(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 64; b++) {
#pragma unroll
        for (int m = 0; m < 4; m++) q[4 * b + m] = make_uint4(p, b, m, 7);
    }
}

__global__ __launch_bounds__(1024) void k_lane_rw4nt(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 64; b++) {
        uint4 v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m] = q[4 * b + m];
#pragma unroll
        for (int m = 0; m < 4; m++) {
            v[m].y ^= 0xa5a5a5a5u;
            __builtin_nontemporal_store(v[m].x, &q[4 * b + m].x); __builtin_nontemporal_store(v[m].y, &q[4 * b + m].y);
            __builtin_nontemporal_store(v[m].z, &q[4 * b + m].z); __builtin_nontemporal_store(v[m].w, &q[4 * b + m].w);
        }
    }
}

// half the lanes per CU: 512-thread groups holding 96 KB of LDS (one per CU)
__global__ __launch_bounds__(512) void k_lane_rw4_half(uint8_t *seg) {
    extern __shared__ uint32_t pad[];
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (threadIdx.x == 9999) pad[0] = 1;
    uint4 *q = reinterpret_cast<uint4 *>(seg + (size_t)p * kStride);
    for (int b = 0; b < kLen / 64; b++) {
        uint4 v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m] = q[4 * b + m];
#pragma unroll
        for (int m = 0; m < 4; m++) { v[m].y ^= 0xa5a5a5a5u; q[4 * b + m] = v[m]; }
    }
}

int main() {
    const size_t bytes = (size_t)kN * kStride;
    uint8_t *seg; uint32_t *out;
    hipMalloc(&seg, bytes); hipMalloc(&out, 64);
    hipMemset(seg, 1, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char *name, double payload, auto &&f) {
        for (int i = 0; i < 2; i++) f();
        hipEventRecord(e0);
        const int reps = 10;
        for (int i = 0; i < reps; i++) f();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        const double us = 1e3 * ms / reps;
        printf("%-12s %8.1f us  %7.1f GB/s (payload %.1f MB per launch)\n", name, us,
               payload / (us * 1e3), payload / 1e6);
    };
    const size_t n16 = bytes / 16;
    const double pay = (double)kN * kLen;
    run("stream_rd", (double)bytes, [&] { k_stream_rd<<<4096, 256>>>((const uint4 *)seg, n16, out); });
    run("stream_rw", 2.0 * bytes, [&] { k_stream_rw<<<4096, 256>>>((uint4 *)seg, n16); });
    run("lane_rd", pay, [&] { k_lane_rd<<<kN / 1024, 1024>>>(seg, out); });
    run("lane_rw", 2 * pay, [&] { k_lane_rw<<<kN / 1024, 1024>>>(seg); });
    run("lane_rw4", 2 * pay, [&] { k_lane_rw4<<<kN / 1024, 1024>>>(seg); });
    run("lane_rw4t", 2 * pay, [&] { k_lane_rw4t<<<kN / 1024, 1024>>>(seg); });
    run("lane_rw8", 2 * pay, [&] { k_lane_rw8<<<kN / 1024, 1024>>>(seg); });
    run("lane_w4", pay, [&] { k_lane_w4<<<kN / 1024, 1024>>>(seg); });
    run("lane_rw4nt", 2 * pay, [&] { k_lane_rw4nt<<<kN / 1024, 1024>>>(seg); });
    run("lane_rw4half", 2 * pay, [&] { k_lane_rw4_half<<<kN / 512, 512, 96 * 1024>>>(seg); });
    // transposed store correctness: after one rw4t pass every packet word 1 of each quad flipped once
    {
        hipMemset(seg, 0, bytes);
        k_lane_rw4t<<<kN / 1024, 1024>>>(seg);
        std::vector<uint32_t> h(bytes / 4);
        hipMemcpy(h.data(), seg, bytes, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t pk = 0; pk < kN; pk++)
            for (int w = 0; w < kStride / 4; w++) {
                const uint32_t want = (w < kLen / 64 * 16 && (w & 3) == 1) ? 0xa5a5a5a5u : 0u;
                if (h[pk * (kStride / 4) + w] != want) bad++;
            }
        printf("rw4t transpose check: %s (%zu bad words)\n", bad ? "FAIL" : "ok", bad);
    }
    hipDeviceSynchronize();
    printf("bytes: segment %zu, payload %.0f\n", bytes, pay);
    return 0;
}
