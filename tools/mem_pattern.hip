// mem_pattern.hip -- read-modify-write bandwidth of the packet access patterns
// the AES kernels can use (not product code).  2^18 packets of 1200 B at a
// 1216-B stride (the bench segment, 319 MB); each variant reads and writes
// every packet byte once (chunks 0..18 of 64 B; the last chunk is partial in
// the real kernel, whole here).
//   lane64   : one lane per packet, 4 x 16-B loads per 64-B chunk per step (today)
//   lane128  : one lane per packet, 8 x 16-B loads per 128-B step
//   quad     : four lanes per packet, 16 B each per 64-B chunk (4x the waves)
//   quad256  : four lanes per packet, 64 B each per 256-B step
//   stream   : contiguous 16-B per lane over the whole segment (upper bound)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

constexpr int kPackets = 1 << 18, kStride = 1216, kChunks = 19;

__global__ __launch_bounds__(1024) void lane64(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t *pkt = seg + (size_t)p * kStride;
    for (int b = 0; b < kChunks; b++) {
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 64 * b);
        uint4 v[4];
#pragma unroll
        for (int m = 0; m < 4; m++) v[m] = q[m];
#pragma unroll
        for (int m = 0; m < 4; m++) { v[m].x ^= 1u; q[m] = v[m]; }
    }
}

// one lane per packet, but each 16-B load instruction covers 16 whole chunks:
// lane m of a quad moves piece m of the quad's four packets (no transpose here)
__global__ __launch_bounds__(1024) void lane64q(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t qb = p & ~3u, m = p & 3u;
    for (int b = 0; b < kChunks; b++) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++)
            v[i] = *reinterpret_cast<uint4 *>(seg + (size_t)(qb + i) * kStride + 64 * b + 16 * m);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v[i].x ^= 1u;
            *reinterpret_cast<uint4 *>(seg + (size_t)(qb + i) * kStride + 64 * b + 16 * m) = v[i];
        }
    }
}

// lane64 with the next chunk's loads issued before this chunk's stores
__global__ __launch_bounds__(1024) void lane64pf(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t *pkt = seg + (size_t)p * kStride;
    uint4 cur[4], nxt[4];
#pragma unroll
    for (int m = 0; m < 4; m++) cur[m] = reinterpret_cast<uint4 *>(pkt)[m];
    for (int b = 0; b < kChunks; b++) {
        if (b + 1 < kChunks) {
#pragma unroll
            for (int m = 0; m < 4; m++) nxt[m] = reinterpret_cast<uint4 *>(pkt + 64 * (b + 1))[m];
        }
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 64 * b);
#pragma unroll
        for (int m = 0; m < 4; m++) { cur[m].x ^= 1u; q[m] = cur[m]; }
#pragma unroll
        for (int m = 0; m < 4; m++) cur[m] = nxt[m];
    }
}

__global__ __launch_bounds__(1024) void lane128(uint8_t *seg) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t *pkt = seg + (size_t)p * kStride;
    for (int b = 0; b < (kChunks + 1) / 2; b++) {
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 128 * b);
        const int nm = (128 * b + 128 <= 64 * kChunks) ? 8 : 4;
        uint4 v[8];
#pragma unroll
        for (int m = 0; m < 8; m++) if (m < nm) v[m] = q[m];
#pragma unroll
        for (int m = 0; m < 8; m++) if (m < nm) { v[m].x ^= 1u; q[m] = v[m]; }
    }
}

__global__ __launch_bounds__(1024) void quad(uint8_t *seg) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p = t >> 2, m = t & 3u;
    uint8_t *pkt = seg + (size_t)p * kStride;
    for (int b = 0; b < kChunks; b++) {
        uint4 *q = reinterpret_cast<uint4 *>(pkt + 64 * b + 16 * m);
        uint4 v = *q;
        v.x ^= 1u;
        *q = v;
    }
}

__global__ __launch_bounds__(1024) void quad256(uint8_t *seg) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t p = t >> 2, m = t & 3u;
    uint8_t *pkt = seg + (size_t)p * kStride;
    for (int b = 0; b < (kChunks + 3) / 4; b++) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int off = 256 * b + 64 * k + 16 * m;
            if (off < 64 * kChunks) v[k] = *reinterpret_cast<uint4 *>(pkt + off);
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int off = 256 * b + 64 * k + 16 * m;
            if (off < 64 * kChunks) { v[k].x ^= 1u; *reinterpret_cast<uint4 *>(pkt + off) = v[k]; }
        }
    }
}

__global__ __launch_bounds__(1024) void stream(uint8_t *seg, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        uint4 *q = reinterpret_cast<uint4 *>(seg) + i;
        uint4 v = *q;
        v.x ^= 1u;
        *q = v;
    }
}

int main() {
    const size_t bytes = (size_t)kPackets * kStride;
    uint8_t *seg;
    if (hipMalloc(&seg, bytes) != hipSuccess) return 1;
    (void)hipMemset(seg, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double moved = 2.0 * kPackets * 64.0 * kChunks; // read + write
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 3; w++) launch();
        (void)hipDeviceSynchronize();
        const int reps = 20;
        (void)hipEventRecord(e0);
        for (int r = 0; r < reps; r++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-8s %8.1f us  %6.2f TB/s (read+write of the packet bytes)\n", name, ms * 1e3,
               moved / (ms * 1e-3) / 1e12);
    };
    run("lane64", [&] { lane64<<<kPackets / 1024, 1024>>>(seg); });
    run("lane64q", [&] { lane64q<<<kPackets / 1024, 1024>>>(seg); });
    run("lane64pf", [&] { lane64pf<<<kPackets / 1024, 1024>>>(seg); });
    run("lane64/2", [&] { lane64<<<kPackets / 1024 / 2, 1024>>>(seg); }); // half the packets
    run("lane128", [&] { lane128<<<kPackets / 1024, 1024>>>(seg); });
    run("quad", [&] { quad<<<kPackets * 4 / 1024, 1024>>>(seg); });
    run("quad256", [&] { quad256<<<kPackets * 4 / 1024, 1024>>>(seg); });
    run("stream", [&] { stream<<<1024, 1024>>>(seg, bytes / 16); });
    printf("status: %s\n", hipGetErrorString(hipGetLastError()));
    (void)hipFree(seg);
    return 0;
}
