// dispatch_bench.cpp -- host bundles through the dispatcher
// (srtp_dispatch_transform_host, srtp_dispatch_submit_host / wait_host)
// without Python: 2^18 RTP packets of 1200 B over 10k SSRCs in engine-pinned
// memory (srtp_host_alloc: chunks move by DMA in place), protect then
// unprotect, synchronously or with two bundles in flight (two buffers,
// P(A) P(B) U(A) U(B) ..., each submit after the wait of the previous
// operation on its buffer).  Prints one JSON line per mode with packets/s per
// direction and the per-operation submit / wait times.
//
//   dispatch_bench [bundle-operations per mode] [shards on device 0]
#include <algorithm>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../include/srtp_mi355x.h"

namespace {
int check(int rc, const char *what) {
    if (rc != SRTP_OK) {
        fprintf(stderr, "%s failed: %d\n", what, rc);
        exit(1);
    }
    return rc;
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Bundle {
    uint8_t *seg = nullptr;
    size_t bytes = 0;
    std::vector<uint32_t> off, len, len0, cap;
    std::vector<int32_t> status;
};

void make_bundle(Bundle &b, uint32_t n, uint32_t L, uint32_t nssrc) {
    const uint32_t region = (L + 10 + 4 + 15) & ~15u; // room for the tag
    b.bytes = (size_t)n * region;
    check(srtp_host_alloc(b.bytes, (void **)&b.seg), "srtp_host_alloc");
    b.off.resize(n); b.len.resize(n); b.len0.resize(n); b.cap.resize(n); b.status.resize(n);
    uint64_t rng = 0x243f6a8885a308d3ull;
    std::vector<uint16_t> seq(nssrc);
    for (auto &q : seq) q = (uint16_t)(rng >> 40), rng = rng * 6364136223846793005ull + 1;
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *p = b.seg + (size_t)i * region;
        for (uint32_t k = 12; k < L; k++) {
            rng = rng * 6364136223846793005ull + 1442695040888963407ull;
            p[k] = (uint8_t)(rng >> 56);
        }
        const uint32_t s = i % nssrc, ssrc = 0x20000000u + s;
        const uint16_t q = seq[s]++;
        p[0] = 0x80; p[1] = 96; p[2] = (uint8_t)(q >> 8); p[3] = (uint8_t)q;
        p[4] = p[5] = p[6] = p[7] = 0;
        p[8] = (uint8_t)(ssrc >> 24); p[9] = (uint8_t)(ssrc >> 16); p[10] = (uint8_t)(ssrc >> 8); p[11] = (uint8_t)ssrc;
        b.off[i] = i * region;
        b.len[i] = b.len0[i] = L;
        b.cap[i] = region;
    }
}

double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
}
} // namespace

int main(int argc, char **argv) {
    const int ops = argc > 1 ? atoi(argv[1]) : 16;
    const int G = argc > 2 ? atoi(argv[2]) : 1;
    const uint32_t n = 1u << 18, L = 1200, nssrc = 10000;
    srtp_policy pol = {SRTP_AESCM_ENCRYPTION, 16, SRTP_HMACSHA1_AUTHENTICATION, 20, 10, 14};
    uint8_t key[16], salt[14];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(17 * i + 3);
    for (int i = 0; i < 14; i++) salt[i] = (uint8_t)(29 * i + 5);
    srtp_engine_opts o;
    srtp_engine_opts_default(&o);
    o.check_replay = 0; // the same bundles again and again
    o.max_contexts = 1u << 15;
    o.max_factories = 8;
    o.max_transformers = 8;
    std::vector<int32_t> devs((size_t)G, 0);
    srtp_dispatch *d = nullptr;
    check(srtp_dispatch_create(devs.data(), G, &o, &d), "dispatch");
    int32_t fs = -1, fr = -1, ts = -1, tr = -1;
    check(srtp_dispatch_factory_create(d, 1, key, 16, salt, 14, &pol, &pol, &fs), "factory");
    check(srtp_dispatch_factory_create(d, 0, key, 16, salt, 14, &pol, &pol, &fr), "factory");
    check(srtp_dispatch_transformer_create(d, SRTP_KIND_RTP, fs, fs, &ts), "transformer");
    check(srtp_dispatch_transformer_create(d, SRTP_KIND_RTP, fr, fr, &tr), "transformer");
    Bundle bu[2];
    make_bundle(bu[0], n, L, nssrc);
    make_bundle(bu[1], n, L, nssrc);
    auto run_sync = [&](Bundle &b, int32_t rev) {
        check(srtp_dispatch_transform_host(d, rev, nullptr, rev ? tr : ts, b.seg, b.bytes, b.off.data(),
                                           b.len.data(), b.cap.data(), nullptr, b.status.data(), n),
              "transform_host");
        for (int32_t s : b.status)
            if (s != SRTP_STATUS_OK) { fprintf(stderr, "status %d\n", s); exit(1); }
    };
    for (int w = 0; w < 2; w++) { // warm: both buffers through both directions
        run_sync(bu[0], 0); run_sync(bu[0], 1);
        run_sync(bu[1], 0); run_sync(bu[1], 1);
    }
    // synchronous: P(A) U(A) P(A) U(A) ...
    {
        std::vector<double> t_op;
        const double t0 = now_s();
        for (int k = 0; k < ops; k++) {
            const double a = now_s();
            run_sync(bu[0], k & 1);
            t_op.push_back(now_s() - a);
        }
        const double dt = now_s() - t0;
        printf("{\"mode\": \"sync\", \"shards\": %d, \"ops\": %d, \"pps_per_direction\": %.1f, \"ms_per_op\": %.3f, "
               "\"op_ms_p50\": %.3f, \"op_ms_max\": %.3f}\n",
               G, ops, (double)ops * n / dt, dt / ops * 1e3, pct(t_op, 0.5) * 1e3, pct(t_op, 1.0) * 1e3);
    }
    // two in flight: P(A) P(B) U(A) U(B) ...
    {
        std::vector<double> t_sub, t_wait;
        uint64_t pend[2] = {0, 0};
        int np = 0, head = 0;
        Bundle *owner[2] = {nullptr, nullptr};
        const double t0 = now_s();
        for (int k = 0; k < ops; k++) {
            const int32_t rev = (k >> 1) & 1;
            Bundle &b = bu[k & 1];
            if (np == 2) {
                const double a = now_s();
                check(srtp_dispatch_wait_host(d, pend[head]), "wait_host");
                t_wait.push_back(now_s() - a);
                for (int32_t s : owner[head]->status)
                    if (s != SRTP_STATUS_OK) { fprintf(stderr, "async status %d\n", s); exit(1); }
                head ^= 1;
                np--;
            }
            const int slot = (head + np) & 1;
            const double a = now_s();
            check(srtp_dispatch_submit_host(d, rev, nullptr, rev ? tr : ts, b.seg, b.bytes, b.off.data(),
                                            b.len.data(), b.cap.data(), nullptr, b.status.data(), n, &pend[slot]),
                  "submit_host");
            t_sub.push_back(now_s() - a);
            owner[slot] = &b;
            np++;
        }
        while (np) {
            check(srtp_dispatch_wait_host(d, pend[head]), "wait_host");
            head ^= 1;
            np--;
        }
        const double dt = now_s() - t0;
        printf("{\"mode\": \"async2\", \"shards\": %d, \"ops\": %d, \"pps_per_direction\": %.1f, \"ms_per_op\": %.3f, "
               "\"submit_ms_p50\": %.3f, \"submit_ms_max\": %.3f, \"wait_ms_p50\": %.3f, \"wait_ms_max\": %.3f}\n",
               G, ops, (double)ops * n / dt, dt / ops * 1e3, pct(t_sub, 0.5) * 1e3, pct(t_sub, 1.0) * 1e3,
               pct(t_wait, 0.5) * 1e3, pct(t_wait, 1.0) * 1e3);
    }
    srtp_dispatch_destroy(d);
    srtp_host_free(bu[0].seg);
    srtp_host_free(bu[1].seg);
    return 0;
}
