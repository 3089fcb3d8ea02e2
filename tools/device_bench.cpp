// device_bench.cpp -- bench.py's headline step without Python or torch:
// 2^18 RTP packets of 1200 B over 10k SSRCs (round robin) per bundle, a ring
// of bundles staged in HBM with advancing sequence numbers (every bundle
// fresh, checkReplay on), a sender engine protecting bundle i on its stream
// and a receiver engine unprotecting it on its own after a device-scope event
// (bench.py --pipe free --events device).  The HIP runtime is whichever
// libamdhip64.so.7 the loader finds: /opt/rocm's by default, torch's bundled
// one under LD_LIBRARY_PATH (profiles/r05/dispatch/hip_runtime/).  Prints one
// JSON line: packets/s per direction (= bench.py's value) and ms per step.
//
//   device_bench [steps] [warmup] [run-in steps]
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/srtp_mi355x.h"

namespace {
void check(int rc, const char *what) {
    if (rc != SRTP_OK) {
        fprintf(stderr, "%s failed: %d\n", what, rc);
        exit(1);
    }
}
void hcheck(hipError_t rc, const char *what) {
    if (rc != hipSuccess) {
        fprintf(stderr, "%s failed: %s\n", what, hipGetErrorString(rc));
        exit(1);
    }
}
double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
} // namespace

int main(int argc, char **argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 100;
    const int warmup = argc > 2 ? atoi(argv[2]) : 5;
    const int runin = argc > 3 ? atoi(argv[3]) : 40;
    const int ring = steps + warmup + runin; // no bundle is processed twice
    const uint32_t n = 1u << 18, L = 1200, nssrc = 10000;
    const uint32_t region = (L + 10 + 15) & ~15u;
    const size_t bytes = (size_t)n * region;
    size_t free_b = 0, total_b = 0;
    hcheck(hipMemGetInfo(&free_b, &total_b), "hipMemGetInfo");
    if ((size_t)ring * (bytes + 4 * (size_t)n) + (8ull << 30) > free_b) {
        fprintf(stderr, "ring of %d bundles does not fit in %zu free bytes\n", ring, free_b);
        return 1;
    }
    srtp_policy pol = {SRTP_AESCM_ENCRYPTION, 16, SRTP_HMACSHA1_AUTHENTICATION, 20, 10, 14};
    uint8_t key[16], salt[14];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(31 * i + 7);
    for (int i = 0; i < 14; i++) salt[i] = (uint8_t)(13 * i + 1);
    srtp_engine_opts o;
    srtp_engine_opts_default(&o);
    o.max_contexts = nssrc;
    o.max_factories = o.max_transformers = 64;
    o.max_batch = n;
    srtp_engine *es = nullptr, *er = nullptr;
    check(srtp_engine_create(&o, &es), "engine");
    check(srtp_engine_create(&o, &er), "engine");
    int32_t fs, fr, ts, tr;
    check(srtp_factory_create(es, 1, key, 16, salt, 14, &pol, &pol, &fs), "factory");
    check(srtp_factory_create(er, 0, key, 16, salt, 14, &pol, &pol, &fr), "factory");
    check(srtp_transformer_create(es, SRTP_KIND_RTP, fs, fs, &ts), "transformer");
    check(srtp_transformer_create(er, SRTP_KIND_RTP, fr, fr, &tr), "transformer");
    hipStream_t sa = (hipStream_t)srtp_engine_stream(es), sb = (hipStream_t)srtp_engine_stream(er);

    // host image of one bundle; each ring slot gets it with its own sequence numbers
    std::vector<uint8_t> h(bytes, 0);
    std::vector<uint32_t> off(n), len(n, L), cap(n, region);
    uint64_t rng = 0x9e3779b97f4a7c15ull;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *p = h.data() + (size_t)i * region;
        for (uint32_t k = 12; k < L; k++) {
            rng = rng * 6364136223846793005ull + 1442695040888963407ull;
            p[k] = (uint8_t)(rng >> 56);
        }
        const uint32_t ssrc = 0x30000000u + i % nssrc;
        p[0] = 0x80; p[1] = 96;
        p[8] = (uint8_t)(ssrc >> 24); p[9] = (uint8_t)(ssrc >> 16); p[10] = (uint8_t)(ssrc >> 8); p[11] = (uint8_t)ssrc;
        off[i] = i * region;
    }
    std::vector<uint16_t> seq(nssrc);
    for (uint32_t s = 0; s < nssrc; s++) seq[s] = (uint16_t)(s * 2654435761u >> 16);
    uint32_t *d_off, *d_cap;
    int32_t *d_st, *d_str;
    hcheck(hipMalloc((void **)&d_off, 4 * (size_t)n), "hipMalloc");
    hcheck(hipMalloc((void **)&d_cap, 4 * (size_t)n), "hipMalloc");
    hcheck(hipMalloc((void **)&d_st, 4 * (size_t)n), "hipMalloc");
    hcheck(hipMalloc((void **)&d_str, 4 * (size_t)n), "hipMalloc");
    hcheck(hipMemcpy(d_off, off.data(), 4 * (size_t)n, hipMemcpyHostToDevice), "H2D");
    hcheck(hipMemcpy(d_cap, cap.data(), 4 * (size_t)n, hipMemcpyHostToDevice), "H2D");
    std::vector<uint8_t *> segs(ring);
    std::vector<uint32_t *> lens(ring);
    for (int j = 0; j < ring; j++) {
        for (uint32_t i = 0; i < n; i++) {
            uint8_t *p = h.data() + (size_t)i * region;
            const uint16_t q = seq[i % nssrc]++;
            p[2] = (uint8_t)(q >> 8); p[3] = (uint8_t)q;
        }
        hcheck(hipMalloc((void **)&segs[j], bytes), "hipMalloc");
        hcheck(hipMalloc((void **)&lens[j], 4 * (size_t)n), "hipMalloc");
        hcheck(hipMemcpy(segs[j], h.data(), bytes, hipMemcpyHostToDevice), "H2D");
        hcheck(hipMemcpy(lens[j], len.data(), 4 * (size_t)n, hipMemcpyHostToDevice), "H2D");
    }
    hipEvent_t ev;
    hcheck(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventDisableSystemFence), "event");
    auto step = [&](int j) {
        check(srtp_transform_device(es, 0, nullptr, ts, segs[j], d_off, lens[j], d_cap, nullptr, d_st, n, sa),
              "protect");
        hcheck(hipEventRecord(ev, sa), "hipEventRecord");
        hcheck(hipStreamWaitEvent(sb, ev, 0), "hipStreamWaitEvent");
        check(srtp_transform_device(er, 1, nullptr, tr, segs[j], d_off, lens[j], d_cap, nullptr, d_str, n, sb),
              "unprotect");
    };
    int j = 0;
    for (int k = 0; k < runin + warmup; k++) step(j++);
    hcheck(hipDeviceSynchronize(), "sync");
    const double t0 = now_s();
    for (int k = 0; k < steps; k++) step(j++);
    hcheck(hipDeviceSynchronize(), "sync");
    const double dt = now_s() - t0;
    srtp_stats a, b;
    check(srtp_engine_stats(es, &a), "stats");
    check(srtp_engine_stats(er, &b), "stats");
    const bool ok = a.status[SRTP_STATUS_OK] == a.packets && b.status[SRTP_STATUS_OK] == b.packets &&
                    b.packets == (uint64_t)j * n;
    const char *hip = "?";
    FILE *f = fopen("/proc/self/maps", "r");
    static char line[1024], found[1024];
    while (f && fgets(line, sizeof line, f))
        if (strstr(line, "libamdhip64")) {
            char *p = strrchr(line, ' ');
            snprintf(found, sizeof found, "%s", p ? p + 1 : line);
            found[strcspn(found, "\n")] = 0;
            hip = found;
        }
    if (f) fclose(f);
    printf("{\"metric\": \"packets/s per direction\", \"value\": %.1f, \"ms_per_step\": %.4f, \"steps\": %d, "
           "\"warmup\": %d, \"run_in\": %d, \"all_ok\": %s, \"hip_runtime\": \"%s\"}\n",
           steps * (double)n / dt, dt / steps * 1e3, steps, warmup, runin, ok ? "true" : "false", hip);
    for (int k = 0; k < ring; k++) {
        (void)hipFree(segs[k]);
        (void)hipFree(lens[k]);
    }
    (void)hipFree(d_off); (void)hipFree(d_cap); (void)hipFree(d_st); (void)hipFree(d_str);
    (void)hipEventDestroy(ev);
    srtp_engine_destroy(es);
    srtp_engine_destroy(er);
    return ok ? 0 : 2;
}
