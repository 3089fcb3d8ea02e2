// Micro-benchmark: grouping 2^18 packets by context slot (18-bit keys), stable.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <rocprim/rocprim.hpp>
using OneSweep = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
#include <cstdio>
#include <vector>
#include <random>
struct alignas(16) Rec { uint32_t a, b, c, d; };
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
template <class F> float timeit(F f, int reps = 20) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); hipDeviceSynchronize();
    hipEventRecord(a); for (int i = 0; i < reps; i++) f(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); return ms / reps * 1000.f;
}
int main() {
    const int n = 1 << 18, bits = 18;
    std::vector<uint32_t> hk(n); std::mt19937 g(1);
    for (int i = 0; i < n; i++) hk[i] = g() % 131072u;
    uint32_t *k0, *k1, *v0, *v1; Rec *r0, *r1; uint64_t *q0, *q1;
    CK(hipMalloc(&k0, 4 * n)); CK(hipMalloc(&k1, 4 * n)); CK(hipMalloc(&v0, 4 * n)); CK(hipMalloc(&v1, 4 * n));
    CK(hipMalloc(&r0, 16 * n)); CK(hipMalloc(&r1, 16 * n)); CK(hipMalloc(&q0, 8 * n)); CK(hipMalloc(&q1, 8 * n));
    CK(hipMemcpy(k0, hk.data(), 4 * n, hipMemcpyHostToDevice));
    size_t t1 = 0, t2 = 0, t3 = 0; void *tmp;
    hipcub::DeviceRadixSort::SortPairs(nullptr, t1, k0, k1, r0, r1, n, 0, bits);
    hipcub::DeviceRadixSort::SortPairs(nullptr, t2, k0, k1, v0, v1, n, 0, bits);
    hipcub::DeviceRadixSort::SortKeys(nullptr, t3, q0, q1, n, 0, 32 + bits);
    CK(hipMalloc(&tmp, std::max(t1, std::max(t2, t3))));
    printf("pairs<u32,Rec16> %d bits: %.1f us\n", bits, timeit([&] { hipcub::DeviceRadixSort::SortPairs(tmp, t1, k0, k1, r0, r1, n, 0, bits); }));
    printf("pairs<u32,u32>   %d bits: %.1f us\n", bits, timeit([&] { hipcub::DeviceRadixSort::SortPairs(tmp, t2, k0, k1, v0, v1, n, 0, bits); }));
    printf("keys<u64>        %d bits: %.1f us\n", 32 + bits, timeit([&] { hipcub::DeviceRadixSort::SortKeys(tmp, t3, q0, q1, n, 0, 32 + bits); }));
    for (int b : {12, 15, 21}) {
        size_t t = 0; hipcub::DeviceRadixSort::SortPairs(nullptr, t, k0, k1, r0, r1, n, 0, b);
        printf("pairs<u32,Rec16> %d bits: %.1f us (temp %zu)\n", b, timeit([&] { hipcub::DeviceRadixSort::SortPairs(tmp, t1, k0, k1, r0, r1, n, 0, b); }), t);
    }
    for (int b : {14, 18, 21}) {
        size_t t = 0;
        rocprim::radix_sort_pairs<OneSweep>(nullptr, t, k0, k1, r0, r1, n, 0, b);
        void *tt; hipMalloc(&tt, t);
        printf("rocprim onesweep pairs<u32,Rec16> %d bits: %.1f us\n", b, timeit([&] { rocprim::radix_sort_pairs<OneSweep>(tt, t, k0, k1, r0, r1, n, 0, b); }));
        rocprim::radix_sort_pairs<OneSweep>(nullptr, t, k0, k1, v0, v1, n, 0, b);
        hipFree(tt); hipMalloc(&tt, t);
        printf("rocprim onesweep pairs<u32,u32>   %d bits: %.1f us\n", b, timeit([&] { rocprim::radix_sort_pairs<OneSweep>(tt, t, k0, k1, v0, v1, n, 0, b); }));
        hipFree(tt);
    }
    // correctness of one onesweep run (stable order within equal keys)
    {
        size_t t = 0; std::vector<uint32_t> idx(n); for (int i = 0; i < n; i++) idx[i] = i;
        hipMemcpy(v0, idx.data(), 4 * n, hipMemcpyHostToDevice);
        rocprim::radix_sort_pairs<OneSweep>(nullptr, t, k0, k1, v0, v1, n, 0, 18);
        void *tt; hipMalloc(&tt, t);
        rocprim::radix_sort_pairs<OneSweep>(tt, t, k0, k1, v0, v1, n, 0, 18);
        std::vector<uint32_t> ok(n), ov(n); hipMemcpy(ok.data(), k1, 4 * n, hipMemcpyDeviceToHost); hipMemcpy(ov.data(), v1, 4 * n, hipMemcpyDeviceToHost);
        bool good = true; for (int i = 1; i < n; i++) if (ok[i-1] > ok[i] || (ok[i-1] == ok[i] && ov[i-1] >= ov[i])) good = false;
        printf("onesweep stable & sorted: %s\n", good ? "yes" : "NO");
    }
    return 0;
}
