/*
 * oracle_bench.c -- CPU baseline timing loop over the oracle (TEST / BENCH
 * INFRASTRUCTURE ONLY: bench.py's cpu_baseline leg; see srtp_oracle.h).
 *
 * The reference's hot path is one SRTPTransformer call per packet per
 * direction (SinglePacketTransformer.java:121-216 -> SRTPCryptoContext
 * transformPacket :658-705 / reverseTransformPacket :572-642), one thread per
 * stream.  Here `threads` POSIX threads, each pinned to one CPU of the
 * process's affinity set, each own a sender and a receiver transformer pair
 * and a 4096-packet bundle of its share of the SSRCs, and loop protect ->
 * unprotect -> advance every sequence number, for `seconds`.  The loop is
 * pure C (no interpreter between calls).  mode = ORC_MODE_REF (the
 * reference's call structure: one 16-B AES call per keystream block, HMAC
 * re-keyed per packet) or ORC_MODE_TUNED (one EVP CTR call per packet,
 * pre-keyed HMAC copied per packet).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "srtp_oracle.h"

enum { kBundle = 4096 };

typedef struct {
    int mode, cpu, pkt_len, ssrcs;
    uint32_t seed;
    volatile int *stop;
    int64_t done;
    int ok;
} worker_arg;

static uint64_t splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *worker(void *p) {
    worker_arg *w = (worker_arg *)p;
    if (w->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(w->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    uint64_t rs = w->seed;
    uint8_t key[16], salt[14];
    for (int i = 0; i < 16; i++) key[i] = (uint8_t)splitmix64(&rs);
    for (int i = 0; i < 14; i++) salt[i] = (uint8_t)splitmix64(&rs);
    const orc_policy pol = {ORC_AESCM_ENCRYPTION, 16, ORC_HMACSHA1_AUTHENTICATION, 20, 10, 14};
    orc_factory *fs = orc_factory_new(1, key, 16, salt, 14, &pol, &pol, w->mode);
    orc_factory *fr = orc_factory_new(0, key, 16, salt, 14, &pol, &pol, w->mode);
    orc_transformer *ts = orc_transformer_new(ORC_KIND_RTP, fs, fs);
    orc_transformer *tr = orc_transformer_new(ORC_KIND_RTP, fr, fr);
    const int L = w->pkt_len, cap = (L + 16 + 15) & ~15, ns = w->ssrcs > 0 ? w->ssrcs : 1;
    uint8_t *seg = (uint8_t *)malloc((size_t)cap * kBundle);
    uint32_t *off = (uint32_t *)malloc(sizeof(uint32_t) * kBundle);
    uint32_t *len = (uint32_t *)malloc(sizeof(uint32_t) * kBundle);
    uint32_t *cp = (uint32_t *)malloc(sizeof(uint32_t) * kBundle);
    uint32_t *fl = (uint32_t *)calloc(kBundle, sizeof(uint32_t));
    int32_t *st = (int32_t *)malloc(sizeof(int32_t) * kBundle);
    uint32_t *ssrc = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)ns);
    uint16_t *seq = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)ns);
    w->ok = seg && off && len && cp && fl && st && ssrc && seq && ts && tr;
    if (w->ok) {
        for (int s = 0; s < ns; s++) {
            ssrc[s] = (uint32_t)splitmix64(&rs) | 1u;
            seq[s] = (uint16_t)splitmix64(&rs);
        }
        for (int i = 0; i < kBundle; i++) {
            uint8_t *b = seg + (size_t)i * cap;
            off[i] = (uint32_t)((size_t)i * cap);
            cp[i] = (uint32_t)cap;
            for (int j = 0; j < L; j++) b[j] = (uint8_t)splitmix64(&rs);
            b[0] = 0x80;
            b[1] = 96;
            const uint32_t x = ssrc[i % ns];
            b[8] = (uint8_t)(x >> 24); b[9] = (uint8_t)(x >> 16); b[10] = (uint8_t)(x >> 8); b[11] = (uint8_t)x;
        }
    }
    while (w->ok && !*w->stop) {
        /* packet i of SSRC i % ns carries that SSRC's next sequence number */
        for (int i = 0; i < kBundle; i++) {
            uint8_t *b = seg + off[i];
            const uint16_t q = seq[i % ns]++;
            b[2] = (uint8_t)(q >> 8);
            b[3] = (uint8_t)q;
            len[i] = (uint32_t)L;
        }
        orc_process(&ts, 0, 0, seg, off, len, cp, fl, st, kBundle, 1);
        for (int i = 0; i < kBundle && w->ok; i++) w->ok = st[i] == ORC_OK;
        orc_process(&tr, 0, 1, seg, off, len, cp, fl, st, kBundle, 1);
        for (int i = 0; i < kBundle && w->ok; i++) w->ok = st[i] == ORC_OK && len[i] == (uint32_t)L;
        w->done += kBundle;
    }
    free(seg); free(off); free(len); free(cp); free(fl); free(st); free(ssrc); free(seq);
    if (ts) { orc_transformer_close(ts); orc_transformer_free(ts); }
    if (tr) { orc_transformer_close(tr); orc_transformer_free(tr); }
    return NULL;
}

/* Packets protected AND unprotected by `threads` pinned threads in about
 * `seconds`; *elapsed receives the wall time.  Returns -1 if a packet was
 * rejected (the loop is expected to accept everything). */
int64_t orc_bench_round_trips(int mode, int threads, double seconds, int pkt_len, int ssrcs,
                              uint32_t seed, double *elapsed) {
    if (threads < 1 || pkt_len < 12 || pkt_len > 8192) return -1;
    cpu_set_t allowed;
    int cpus[1024], ncpu = 0;
    if (sched_getaffinity(0, sizeof allowed, &allowed) == 0)
        for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; c++)
            if (CPU_ISSET(c, &allowed)) cpus[ncpu++] = c;
    volatile int stop = 0;
    worker_arg *args = (worker_arg *)calloc((size_t)threads, sizeof(worker_arg));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!args || !th) { free(args); free(th); return -1; }
    const int per = ssrcs / threads > 0 ? ssrcs / threads : 1;
    const double t0 = now_s();
    for (int t = 0; t < threads; t++) {
        args[t].mode = mode;
        args[t].cpu = ncpu ? cpus[t % ncpu] : -1;
        args[t].pkt_len = pkt_len;
        args[t].ssrcs = per;
        args[t].seed = seed + 7919u * (uint32_t)t;
        args[t].stop = &stop;
        pthread_create(&th[t], NULL, worker, &args[t]);
    }
    struct timespec nap = {(time_t)seconds, (long)((seconds - (double)(time_t)seconds) * 1e9)};
    nanosleep(&nap, NULL);
    stop = 1;
    int64_t total = 0;
    int ok = 1;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        total += args[t].done;
        ok &= args[t].ok;
    }
    if (elapsed) *elapsed = now_s() - t0;
    free(args);
    free(th);
    return ok ? total : -1;
}
