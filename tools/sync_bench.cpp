// sync_bench.cpp -- latency and throughput of the per-packet drop-in path:
// T threads, each calling SinglePacketTransformer.transform(RawPacket) as the
// reference's callers do (one packet per call: RTPConnectorOutputStream.java
// :268-300, DtlsPacketTransformer.java:1544-1564), on 50 transformers.
//
//   path "one":   srtp_rawpacket_transform_one -- the calls of all threads
//                 coalesce into shared bundles (srtp_aggregator_transform,
//                 SRTP_AGG_SEAL_IDLE)
//   path "array": srtp_rawpacket_transform with a 1-element array on the
//                 thread's own batch -- one GPU round trip per call (the
//                 round-3 drop-in)
//   path "arrayq": as "array", the batch routed through the aggregator
//                 (srtp_rawpacket_batch_set_aggregator: what the JNI shim's
//                 transformPackets does for arrays that cannot throw)
//   path "queue": the asynchronous call (GpuPacketQueue): each thread owns a
//                 completion queue and keeps SYNC_DEPTH (default 64) packets in
//                 flight -- srtp_rawpacket_submit, srtp_queue_reap, and
//                 srtp_rawpacket_complete + a copy of each result back into its
//                 buffer (the shim's SetByteArrayRegion); with "rt" each
//                 protected packet is then submitted for unprotect before its
//                 buffer takes the next packet
//
// over one engine or a G-shard dispatcher (all shards on device 0 of a one-GPU
// box).  1200-B RTP packets, AES_CM_128_HMAC_SHA1_80 protect, each thread its
// own SSRCs.  Prints one JSON line per (path, shards, threads): calls/s and
// the per-call latency percentiles.  With "rt" each protected packet is then
// unprotected by a receiving transformer of the same keys (the
// reverseTransform call of the receive side), timed on its own: calls count
// both calls, "lat_us" the protect calls and "lat_unprotect_us" the unprotect
// calls.
//
//   sync_bench [seconds-per-point] [path shards threads [rt]]   (one point: e.g. "one 0 1")
//
// The latency of a queued call runs from its submit to its reap.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <vector>
#include <unistd.h>

#include "../include/srtp_mi355x.h"

namespace {
using Clock = std::chrono::steady_clock;

int check(int rc, const char *what) {
    if (rc != SRTP_OK) {
        fprintf(stderr, "%s failed: %d\n", what, rc);
        fflush(stderr);
        _exit(1); // not exit(): other threads may be inside the library
    }
    return rc;
}

void fill_packet(uint8_t *p, uint32_t len, uint64_t &rng) {
    for (uint32_t i = 12; i < len; i++) {
        rng = rng * 6364136223846793005ull + 1442695040888963407ull;
        p[i] = (uint8_t)(rng >> 56);
    }
    p[0] = 0x80;
    p[1] = 96;
}

uint32_t ns_since(Clock::time_point t0) {
    return (uint32_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - t0).count();
}

// One thread of the "queue" path (see the file comment).
struct QueueWorker {
    srtp_aggregator *a;
    const std::vector<int32_t> &tr, &trr;
    int k, n_tr;
    uint32_t L, BUF, depth;
    bool rt;
    bool stagger; // rts: half the buffers start one protect ahead (below)
    std::atomic<bool> &stop;
    std::vector<uint32_t> &lat, &latu;
    uint64_t &bad;

    struct Buf {
        std::vector<uint8_t> b;
        uint32_t len = 0;
        int s = 0;
        Clock::time_point t0;
    };

    void run() {
        srtp_queue *q = nullptr;
        check(srtp_queue_create(a, depth, &q), "queue");
        std::vector<Buf> bufs(depth);
        std::vector<srtp_completion> comps(depth);
        std::deque<std::pair<uint32_t, int32_t>> pend; // (buffer, reverse) to submit, in order
        uint64_t rng = 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1);
        const int n_ssrc = 3;
        uint16_t seq[n_ssrc];
        for (auto &x : seq) x = (uint16_t)(rng >> 40), rng = rng * 6364136223846793005ull + 1;
        uint64_t n = 0;
        auto next_packet = [&](uint32_t i) {
            Buf &bf = bufs[i];
            const int s = (int)(n++ % n_ssrc);
            const uint32_t ssrc = 0x20000000u + (uint32_t)k * 16u + (uint32_t)s;
            const uint16_t sq = seq[s]++;
            uint8_t *p = bf.b.data();
            p[2] = (uint8_t)(sq >> 8); p[3] = (uint8_t)sq;
            p[8] = (uint8_t)(ssrc >> 24); p[9] = (uint8_t)(ssrc >> 16); p[10] = (uint8_t)(ssrc >> 8); p[11] = (uint8_t)ssrc;
            bf.len = L;
            bf.s = s;
            pend.emplace_back(i, 0);
        };
        for (uint32_t i = 0; i < depth; i++) {
            bufs[i].b.resize(BUF);
            fill_packet(bufs[i].b.data(), L, rng);
            next_packet(i);
        }
        // rts: the odd buffers are protected once before the loop, so that
        // half of a thread's packets are in their protect step and half in
        // their unprotect step -- as a sender and a receiver of independent
        // streams -- instead of all 64 moving through the two directions in
        // lockstep (rt), one direction's bundle at a time
        if (rt && stagger) {
            std::deque<std::pair<uint32_t, int32_t>> keep;
            uint32_t ahead = 0;
            for (const auto &pr : pend) {
                if (pr.first & 1u) {
                    Buf &bf = bufs[pr.first];
                    const int ti = (k * n_ssrc + bf.s) % n_tr;
                    check(srtp_rawpacket_submit(q, 0, tr[(size_t)ti], bf.b.data(), BUF, 0, bf.len, 0, pr.first),
                          "submit");
                    ahead++;
                } else {
                    keep.push_back(pr);
                }
            }
            pend.swap(keep);
            while (ahead) {
                const int m = srtp_queue_reap(q, comps.data(), depth, 1);
                if (m < 0) check(m, "reap");
                for (int j = 0; j < m; j++) {
                    const srtp_completion &c = comps[(size_t)j];
                    const uint32_t i = (uint32_t)c.cookie;
                    uint32_t copy = 0, need = 0;
                    check(srtp_rawpacket_complete(q, &c, BUF, &copy, &need), "complete");
                    if (!need && copy) memcpy(bufs[i].b.data(), c.data, copy);
                    bufs[i].len = c.len;
                    pend.emplace_back(i, 1);
                    ahead--;
                }
                srtp_queue_release(q);
            }
        }
        for (;;) {
            const bool stopping = stop.load(std::memory_order_relaxed);
            while (!stopping && !pend.empty()) {
                const auto [i, rev] = pend.front();
                Buf &bf = bufs[i];
                const int ti = (k * n_ssrc + bf.s) % n_tr;
                const int rc = srtp_rawpacket_submit(q, rev, rev ? trr[(size_t)ti] : tr[(size_t)ti], bf.b.data(), BUF, 0,
                                                     bf.len, 0, ((uint64_t)rev << 32) | i);
                if (rc == SRTP_EAGAIN) break;
                check(rc, "submit");
                bf.t0 = Clock::now();
                pend.pop_front();
            }
            if (srtp_queue_outstanding(q) == 0) {
                if (stopping) break;
                continue;
            }
            const int m = srtp_queue_reap(q, comps.data(), depth, 1);
            if (m < 0) check(m, "reap");
            for (int j = 0; j < m; j++) {
                const srtp_completion &c = comps[(size_t)j];
                const uint32_t i = (uint32_t)c.cookie;
                Buf &bf = bufs[i];
                (c.reverse ? latu : lat).push_back(ns_since(bf.t0));
                uint32_t copy = 0, need = 0;
                check(srtp_rawpacket_complete(q, &c, BUF, &copy, &need), "complete");
                if (need || c.status != SRTP_STATUS_OK || c.len != (c.reverse ? L : L + 10)) bad++;
                if (!need && copy) memcpy(bf.b.data(), c.data, copy); // SetByteArrayRegion
                bf.len = c.len;
                if (stopping) continue;
                if (!c.reverse && rt) pend.emplace_back(i, 1);
                else next_packet(i);
            }
            srtp_queue_release(q); // written back

        }
        srtp_queue_destroy(q);
    }
};

double pct(std::vector<uint32_t> &v, double q) {
    if (v.empty()) return 0.0;
    const size_t k = std::min(v.size() - 1, (size_t)(q * (double)v.size()));
    std::nth_element(v.begin(), v.begin() + (long)k, v.end());
    return v[k] / 1000.0;
}
} // namespace

int main(int argc, char **argv) {
    const double seconds = argc > 1 ? atof(argv[1]) : 2.0;
    // packet length: 1200 B, or SYNC_LEN (the per-block cost of the MAC chain)
    const uint32_t L = getenv("SYNC_LEN") ? (uint32_t)atoi(getenv("SYNC_LEN")) : 1200u;
    const uint32_t BUF = L + 16; // room behind the packet: the tag is appended in place
    const int n_tr = 50;
    srtp_policy pol = {SRTP_AESCM_ENCRYPTION, 16, SRTP_HMACSHA1_AUTHENTICATION, 20, 10, 14};
    const bool one_point = argc > 4;
    // a point's own shard and thread counts (any), else the sweep's
    const std::vector<int> shard_counts = one_point ? std::vector<int>{atoi(argv[3])} : std::vector<int>{0, 8};
    const std::vector<int> thread_counts = one_point ? std::vector<int>{atoi(argv[4])} : std::vector<int>{1, 8, 64};
    const int p_only = one_point ? (strcmp(argv[2], "one") == 0 ? 0 : strcmp(argv[2], "array") == 0 ? 1
                                    : strcmp(argv[2], "queue") == 0 ? 2 : 3) : -1;
    const uint32_t depth = getenv("SYNC_DEPTH") ? (uint32_t)atoi(getenv("SYNC_DEPTH")) : 64u;
    const int g_only = one_point ? atoi(argv[3]) : -1, t_only = one_point ? atoi(argv[4]) : -1;
    const bool rt = argc > 5 && (strcmp(argv[5], "rt") == 0 || strcmp(argv[5], "rts") == 0);
    const bool stagger = argc > 5 && strcmp(argv[5], "rts") == 0;
    for (int path = 0; path < 4; path++) {
        for (int G : shard_counts) {
            for (int T : thread_counts) {
                if (one_point) {
                    if (path != p_only || G != g_only || T != t_only) continue;
                } else if (((path == 1 || path == 3) && T == 64 && G == 8) || (path == 2 && T == 1)) {
                    continue; // 64 pinned batches x 8 shards: skip
                }
                srtp_engine_opts o;
                srtp_engine_opts_default(&o);
                o.max_contexts = 1u << 16;
                o.max_factories = 128;
                o.max_transformers = 128;
                srtp_engine *e = nullptr;
                srtp_dispatch *d = nullptr;
                std::vector<int32_t> tr((size_t)n_tr), trr((size_t)n_tr);
                if (G == 0) check(srtp_engine_create(&o, &e), "engine");
                else {
                    std::vector<int32_t> devs((size_t)G, 0);
                    check(srtp_dispatch_create(devs.data(), G, &o, &d), "dispatch");
                }
                for (int t = 0; t < n_tr; t++) {
                    uint8_t key[16], salt[14];
                    for (int i = 0; i < 16; i++) key[i] = (uint8_t)(17 * i + 3 + t);
                    for (int i = 0; i < 14; i++) salt[i] = (uint8_t)(29 * i + 5 + t);
                    int32_t f = -1;
                    check(d ? srtp_dispatch_factory_create(d, 1, key, 16, salt, 14, &pol, &pol, &f)
                            : srtp_factory_create(e, 1, key, 16, salt, 14, &pol, &pol, &f), "factory");
                    check(d ? srtp_dispatch_transformer_create(d, SRTP_KIND_RTP, f, f, &tr[(size_t)t])
                            : srtp_transformer_create(e, SRTP_KIND_RTP, f, f, &tr[(size_t)t]), "transformer");
                    if (!rt) continue;
                    int32_t fr = -1;
                    check(d ? srtp_dispatch_factory_create(d, 0, key, 16, salt, 14, &pol, &pol, &fr)
                            : srtp_factory_create(e, 0, key, 16, salt, 14, &pol, &pol, &fr), "factory");
                    check(d ? srtp_dispatch_transformer_create(d, SRTP_KIND_RTP, fr, fr, &trr[(size_t)t])
                            : srtp_transformer_create(e, SRTP_KIND_RTP, fr, fr, &trr[(size_t)t]), "transformer");
                }
                // SYNC_DEBUG=<flags>: srtp_engine_set_debug on every engine (A/B of
                // the engine's paths, e.g. 4 = SRTP_DEBUG_NO_WIDE)
                if (const char *dbg = getenv("SYNC_DEBUG")) {
                    const uint32_t f = (uint32_t)strtoul(dbg, nullptr, 0);
                    if (e) check(srtp_engine_set_debug(e, f), "debug");
                    for (int s2 = 0; d && s2 < G; s2++) check(srtp_engine_set_debug(srtp_dispatch_engine(d, s2), f), "debug");
                }
                srtp_aggregator *a = nullptr;
                if (path != 1) {
                    srtp_aggregator_opts ao;
                    srtp_aggregator_opts_default(&ao);
                    ao.max_packets = 4096;
                    ao.max_bytes = 8u << 20;
                    if (path != 0) ao.depth = 6; // as the JNI shim's aggregator
                    // SYNC_AGG="packets,MB,depth": other bundle sizes / slot counts
                    if (const char *g = getenv("SYNC_AGG")) {
                        unsigned pk = 0, mb = 0, dp = 0;
                        if (sscanf(g, "%u,%u,%u", &pk, &mb, &dp) == 3) {
                            ao.max_packets = pk;
                            ao.max_bytes = (size_t)mb << 20;
                            ao.depth = (int32_t)dp;
                        }
                    }
                    check(d ? srtp_aggregator_create_dispatch(d, &ao, nullptr, nullptr, &a)
                            : srtp_aggregator_create(e, &ao, nullptr, nullptr, &a), "aggregator");
                }
                std::atomic<bool> stop{false};
                std::atomic<int> started{0};
                std::vector<std::vector<uint32_t>> lat((size_t)T), latu((size_t)T);
                std::vector<uint64_t> bad((size_t)T, 0);
                std::vector<std::thread> th;
                for (int k = 0; k < T; k++) {
                    th.emplace_back([&, k] {
                        if (path == 2) {
                            started++;
                            QueueWorker{a, tr, trr, k, n_tr, L, BUF, depth, rt, stagger, stop, lat[(size_t)k], latu[(size_t)k],
                                        bad[(size_t)k]}.run();
                            return;
                        }
                        srtp_rawpacket_batch *b = nullptr;
                        if (path == 1 || path == 3)
                            check(d ? srtp_rawpacket_batch_create_dispatch(d, &b) : srtp_rawpacket_batch_create(e, &b),
                                  "batch");
                        if (path == 3) check(srtp_rawpacket_batch_set_aggregator(b, a), "batch agg");
                        std::vector<uint8_t> buf(BUF), grow(65535 + 16);
                        uint64_t rng = 0x9e3779b97f4a7c15ull * (uint64_t)(k + 1);
                        fill_packet(buf.data(), L, rng);
                        const int n_ssrc = 3;
                        uint16_t seq[n_ssrc];
                        for (auto &x : seq) x = (uint16_t)(rng >> 40), rng = rng * 6364136223846793005ull + 1;
                        std::vector<uint32_t> &mine = lat[(size_t)k], &mineu = latu[(size_t)k];
                        mine.reserve(1u << 20);
                        if (rt) mineu.reserve(1u << 20);
                        started++;
                        uint64_t n = 0;
                        while (!stop.load(std::memory_order_relaxed)) {
                            const int s = (int)(n % n_ssrc);
                            const uint32_t ssrc = 0x20000000u + (uint32_t)k * 16u + (uint32_t)s;
                            const int ti = (k * n_ssrc + s) % n_tr;
                            const int32_t t = tr[(size_t)ti];
                            const uint16_t q = seq[s]++;
                            buf[2] = (uint8_t)(q >> 8); buf[3] = (uint8_t)q;
                            buf[8] = (uint8_t)(ssrc >> 24); buf[9] = (uint8_t)(ssrc >> 16);
                            buf[10] = (uint8_t)(ssrc >> 8); buf[11] = (uint8_t)ssrc;
                            uint32_t len = L, need = 0;
                            int32_t st = -1;
                            const auto t0 = Clock::now();
                            if (path == 0) {
                                check(srtp_rawpacket_transform_one(a, 0, t, buf.data(), BUF, 0, &len, 0, &st, &need,
                                                                   grow.data(), (uint32_t)grow.size()), "one");
                            } else {
                                uint8_t *bp = buf.data();
                                uint32_t bl = BUF, off = 0, fl = 0;
                                int32_t thrown = -1;
                                check(srtp_rawpacket_transform(b, 0, nullptr, t, &bp, &bl, &off, &len, &fl, &st, &need, 1,
                                                               &thrown), "array");
                            }
                            const auto t1 = Clock::now();
                            mine.push_back((uint32_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
                            if (st != SRTP_STATUS_OK || len != L + 10) bad[(size_t)k]++;
                            n++;
                            if (!rt) continue;
                            // the receive side: reverseTransform of the packet just protected
                            const int32_t tu = trr[(size_t)ti];
                            const uint32_t plen = len;
                            const auto u0 = Clock::now();
                            if (path == 0) {
                                check(srtp_rawpacket_transform_one(a, 1, tu, buf.data(), BUF, 0, &len, 0, &st, &need,
                                                                   grow.data(), (uint32_t)grow.size()), "one");
                            } else {
                                uint8_t *bp = buf.data();
                                uint32_t bl = BUF, off = 0, fl = 0;
                                int32_t thrown = -1;
                                check(srtp_rawpacket_transform(b, 1, nullptr, tu, &bp, &bl, &off, &len, &fl, &st, &need, 1,
                                                               &thrown), "array");
                            }
                            const auto u1 = Clock::now();
                            mineu.push_back((uint32_t)std::chrono::duration_cast<std::chrono::nanoseconds>(u1 - u0).count());
                            if (st != SRTP_STATUS_OK || len != plen - 10) bad[(size_t)k]++;
                        }
                        if (b) srtp_rawpacket_batch_destroy(b);
                    });
                }
                while (started.load() < T) std::this_thread::yield();
                const auto t0 = Clock::now();
                std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
                stop = true;
                for (auto &x : th) x.join();
                const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
                std::vector<uint32_t> all, allu;
                uint64_t nbad = 0;
                for (int k = 0; k < T; k++) {
                    all.insert(all.end(), lat[(size_t)k].begin(), lat[(size_t)k].end());
                    allu.insert(allu.end(), latu[(size_t)k].begin(), latu[(size_t)k].end());
                    nbad += bad[(size_t)k];
                }
                uint64_t acc = 0, comp = 0, bundles = 0;
                if (a) {
                    srtp_aggregator_stats(a, &acc, &comp, &bundles);
                    srtp_aggregator_destroy(a);
                }
                double mean = 0;
                for (uint32_t x : all) mean += x;
                mean = all.empty() ? 0 : mean / all.size() / 1000.0;
                const size_t calls = all.size() + allu.size();
                char ul[160] = "";
                if (rt)
                    snprintf(ul, sizeof ul, "\"lat_unprotect_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"p999\": %.1f}, ",
                             pct(allu, 0.5), pct(allu, 0.9), pct(allu, 0.99), pct(allu, 0.999));
                printf("{\"path\": \"%s\", \"shards\": %d, \"dispatcher\": %s, \"threads\": %d, \"transformers\": %d, "
                       "\"pkt_len\": %u, \"calls\": %zu, \"seconds\": %.3f, \"calls_per_s\": %.1f, "
                       "\"lat_us\": {\"mean\": %.1f, \"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"p999\": %.1f}, "
                       "%s\"bundles\": %llu, \"packets_per_bundle\": %.1f, \"not_ok\": %llu}\n",
                       path == 0 ? "one" : path == 1 ? "array" : path == 2 ? "queue" : "arrayq", G ? G : 1, G ? "true" : "false", T, n_tr, L, calls, dt,
                       calls / dt, mean, pct(all, 0.5), pct(all, 0.9), pct(all, 0.99), pct(all, 0.999), ul,
                       (unsigned long long)bundles, bundles ? (double)comp / bundles : 0.0,
                       (unsigned long long)nbad);
                fflush(stdout);
                if (d) srtp_dispatch_destroy(d);
                if (e) srtp_engine_destroy(e);
            }
        }
    }
    return 0;
}
