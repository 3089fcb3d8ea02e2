// agg_bench.cpp -- throughput of the per-packet aggregator (srtp_aggregator_*)
// with P producer threads, on one engine or over a G-shard dispatcher (all
// shards on device 0 of a one-GPU box, or devices 0..G-1): the deployment path
// of the reference's connectors, which hand the transform chain one packet at
// a time (RTPConnectorOutputStream.java:268-300,652-830).  Each producer
// protects its own SSRCs' 1200-B RTP packets (fresh sequence numbers), the
// callback counts completions; prints one JSON line per (G, P).
//
//   agg_bench [seconds-per-point] [devices: 0 = all shards on device 0]
//             [shards: only this count, 0 = one engine] [producers: only this count]
#include <atomic>
#include <chrono>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <vector>

#include "../include/srtp_mi355x.h"

namespace {
std::atomic<uint64_t> g_done{0}, g_bad{0};

void on_packet(void *, uint64_t, int32_t status, const uint8_t *, uint32_t) {
    g_done.fetch_add(1, std::memory_order_relaxed);
    if (status != SRTP_STATUS_OK) g_bad.fetch_add(1, std::memory_order_relaxed);
}

struct Producer {
    uint32_t ssrc0;
    int n_ssrc;
};

void fill_packet(uint8_t *p, uint32_t len, uint32_t ssrc, uint16_t seq, uint64_t &rng) {
    for (uint32_t i = 12; i < len; i++) {
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        p[i] = (uint8_t)(rng >> 56);
    }
    p[0] = 0x80; p[1] = 96;
    p[2] = (uint8_t)(seq >> 8); p[3] = (uint8_t)seq;
    p[4] = p[5] = p[6] = p[7] = 0;
    p[8] = (uint8_t)(ssrc >> 24); p[9] = (uint8_t)(ssrc >> 16); p[10] = (uint8_t)(ssrc >> 8); p[11] = (uint8_t)ssrc;
}

int check(int rc, const char *what) {
    if (rc != SRTP_OK) {
        fprintf(stderr, "%s failed: %d\n", what, rc);
        exit(1);
    }
    return rc;
}
} // namespace

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
    const int distinct_devices = argc > 2 ? atoi(argv[2]) : 0;
    const uint32_t L = 1200;
    std::vector<int> shard_counts = {0, 1, 4, 8}; // 0: one engine without a dispatcher
    std::vector<int> producer_counts = {1, 4, 16};
    if (argc > 3) shard_counts = {atoi(argv[3])};
    if (argc > 4) producer_counts = {atoi(argv[4])};
    srtp_policy pol = {SRTP_AESCM_ENCRYPTION, 16, SRTP_HMACSHA1_AUTHENTICATION, 20, 10, 14};
    uint8_t key[16], salt[14];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(17 * i + 3);
    for (int i = 0; i < 14; i++) salt[i] = (uint8_t)(29 * i + 5);
    for (int G : shard_counts) {
        srtp_engine_opts o;
        srtp_engine_opts_default(&o);
        o.abort_on_error = 0;
        o.max_contexts = 1u << 16;
        o.max_factories = 16;
        o.max_transformers = 16;
        srtp_engine *e = nullptr;
        srtp_dispatch *d = nullptr;
        int32_t f = -1, t = -1;
        if (G == 0) {
            check(srtp_engine_create(&o, &e), "engine");
            check(srtp_factory_create(e, 1, key, 16, salt, 14, &pol, &pol, &f), "factory");
        } else {
            std::vector<int32_t> devs((size_t)G);
            for (int s = 0; s < G; s++) devs[(size_t)s] = distinct_devices ? s : 0;
            check(srtp_dispatch_create(devs.data(), G, &o, &d), "dispatch");
            check(srtp_dispatch_factory_create(d, 1, key, 16, salt, 14, &pol, &pol, &f), "factory");
        }
        for (int P : producer_counts) {
            // a fresh sender transformer per point: the SSRCs and sequence
            // numbers of the producers repeat from point to point, and the
            // sender's replay check (SRTPCryptoContext.java:279-323) would drop
            // them in a transformer that has seen them
            check(d ? srtp_dispatch_transformer_create(d, SRTP_KIND_RTP, f, f, &t)
                    : srtp_transformer_create(e, SRTP_KIND_RTP, f, f, &t), "transformer");
            srtp_aggregator_opts ao;
            srtp_aggregator_opts_default(&ao);
            srtp_aggregator *a = nullptr;
            check(d ? srtp_aggregator_create_dispatch(d, &ao, on_packet, nullptr, &a)
                    : srtp_aggregator_create(e, &ao, on_packet, nullptr, &a), "aggregator");
            g_done = 0;
            g_bad = 0;
            std::atomic<bool> stop{false};
            std::atomic<uint64_t> submitted{0};
            std::vector<std::thread> th;
            const auto t0 = std::chrono::steady_clock::now();
            for (int k = 0; k < P; k++) {
                th.emplace_back([&, k] {
                    // 64 SSRCs per producer, each its own sequence; a pool of
                    // pre-made packets whose seq / SSRC are rewritten per submit
                    const int n_ssrc = 64;
                    std::vector<uint16_t> seq((size_t)n_ssrc);
                    uint64_t rng = 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1) + (uint64_t)G * 131;
                    for (auto &x : seq) x = (uint16_t)(rng >> 48), rng = rng * 6364136223846793005ull + 1;
                    std::vector<uint8_t> pkt(L);
                    fill_packet(pkt.data(), L, 0, 0, rng);
                    uint64_t n = 0;
                    while (!stop.load(std::memory_order_relaxed)) {
                        const int s = (int)(n % (uint64_t)n_ssrc);
                        const uint32_t ssrc = 0x10000000u + (uint32_t)k * 1000u + (uint32_t)s;
                        const uint16_t q = seq[(size_t)s]++;
                        pkt[2] = (uint8_t)(q >> 8); pkt[3] = (uint8_t)q;
                        pkt[8] = (uint8_t)(ssrc >> 24); pkt[9] = (uint8_t)(ssrc >> 16);
                        pkt[10] = (uint8_t)(ssrc >> 8); pkt[11] = (uint8_t)ssrc;
                        if (srtp_aggregator_submit(a, 0, t, pkt.data(), L, 0, n) != SRTP_OK) break;
                        n++;
                    }
                    submitted.fetch_add(n);
                });
            }
            std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
            stop = true;
            for (auto &x : th) x.join();
            check(srtp_aggregator_flush(a), "flush");
            const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            uint64_t acc = 0, comp = 0, bundles = 0;
            srtp_aggregator_stats(a, &acc, &comp, &bundles);
            srtp_aggregator_destroy(a);
            printf("{\"shards\": %d, \"dispatcher\": %s, \"producers\": %d, \"pkt_len\": %u, "
                   "\"packets\": %llu, \"seconds\": %.3f, \"pps\": %.1f, \"gbps_in\": %.3f, "
                   "\"bundles\": %llu, \"packets_per_bundle\": %.1f, \"not_ok\": %llu}\n",
                   G ? G : 1, G ? "true" : "false", P, L, (unsigned long long)comp, dt, comp / dt,
                   comp * (double)L / dt / 1e9, (unsigned long long)bundles,
                   bundles ? (double)comp / bundles : 0.0, (unsigned long long)g_bad.load());
            fflush(stdout);
        }
        if (d) srtp_dispatch_destroy(d);
        if (e) srtp_engine_destroy(e);
    }
    return 0;
}
