// dispatch.cpp -- in-process multi-GPU front end of the SRTP engine
// (SURVEY.md 8b engine_create(devices, opts), 8e SSRC sharding).
//
// A libjitsi JVM is one process; it hands RawPacket[] bundles to the engine
// through one JNI shim.  srtp_dispatch owns one engine per shard (one shard per
// GPU, or several on one GPU for testing) and splits each host bundle by
// shard = mix32(SSRC) % shards.  SRTP state is per (transformer, SSRC) context
// (SRTPTransformer.java:62,152-175 keeps one context per SSRC, nothing else is
// shared but the read-only factory keys), so a shard owns its SSRCs' contexts
// and no data moves between GPUs.  Factories and transformers are replicated
// to every shard with identical ids.
//
// Order and abort semantics.  Each shard receives its packets in bundle
// order, which is all the per-context state machine needs.  The one
// cross-shard dependency is SinglePacketTransformer's rethrow
// (SinglePacketTransformer.java:134-155,190-210): a packet that throws aborts
// the later packets of the same transformer's array, on every shard.  The
// whole bundle runs on every shard at once; when a packet of transformer t
// came back ERR_MALFORMED, t's packets after the first such packet e_t (in
// bundle order, over all shards) are rolled back: they get NOT_PROCESSED and
// their original bytes and length, and every context they touched is reset to
// its state before the bundle (srtp_contexts_save before the run,
// srtp_contexts_restore after it; contexts they created are removed) and
// then re-run with t's packets up to e_t -- which gives exactly the state one
// engine leaves, because those packets see the same state and bytes as in the
// first run.  Only transformers with a packet that could throw (a superset of
// the engine's throws: RawPacket.getHeaderLength / SRTPCipherCTR.process /
// RawPacket.getSRTCPIndex bounds, see may_throw) are snapshotted and stashed.
// A bundle therefore costs at most two runs on each shard plus two context
// copies, however many packets throw or could throw; without abort_on_error,
// or without any packet that could throw (the normal case), one run.
//
// Data path per shard: a worker thread packs its packets into pinned slots of
// an srtp_pipeline on its engine (H2D, kernels and D2H of consecutive chunks
// overlap), then scatters statuses, lengths and packet bytes back.  The packet
// copies of a chunk are split over the worker and a pool of copy helpers
// shared by the shards (one host thread copies ~12 GB/s, below the PCIe rate).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <sched.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/srtp_mi355x.h"

namespace {

constexpr int32_t kHdrThrow = (int32_t)0x80000000; // getHeaderLength would throw
constexpr uint32_t kChunkPackets = 1u << 15;       // packets per pipeline slot
constexpr size_t kChunkBytes = (size_t)48 << 20;   // segment bytes per pipeline slot
constexpr size_t kGatherMax = 32768;               // packets per gathered chunk (srtp_pipeline_submit_gather)
constexpr int kDepth = 8;                          // pipeline slots per shard
constexpr size_t kMaxInflight = 64;                // host bundles submitted and not yet waited for

uint32_t mix32(uint32_t x) { // murmur3 fmix32 (libjitsi_amd/dispatch.py mix32)
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// RawPacket.getHeaderLength (RawPacket.java:602-614) with the signed extension
// length (:544-556); kHdrThrow when the extension length lies outside cap.
int32_t rtp_header_len(const uint8_t *pkt, uint32_t cap) {
    const uint32_t b0 = pkt[0];
    const int cc = (int)(b0 & 0x0fu);
    int32_t h = 12 + 4 * cc;
    if (b0 & 0x10u) {
        const int idx = 12 + cc * 4 + 2;
        if (idx + 1 >= (int)cap) return kHdrThrow;
        const int ext = ((int)(int8_t)pkt[idx] * 256) | (int)pkt[idx + 1];
        h += 4 + ext * 4;
    }
    return h;
}

// SRTPCipherCTR.process would throw on region [h, h + plen) (:99-120); the
// AES-F8 (SRTPCipherF8.process :97-128) and NULL ciphers throw on a subset.
bool cipher_may_throw(int32_t h, int32_t plen) {
    if (h == kHdrThrow) return true;
    if (plen < 0) return (plen % 16) != 0;
    return plen > 0 && h < 0;
}

// Whether the reference could throw on a valid packet (12 <= L <= C): a
// superset of its throws (RawPacket.getHeaderLength, SRTPCipherCTR.process /
// SRTPCipherF8.process bounds, RawPacket.getSRTCPIndex).  t_max: the largest
// tag length in tag_mask.
bool may_throw_one(bool rtp, int32_t reverse, const uint8_t *pkt, uint32_t L, uint32_t C, uint32_t fl,
                   uint32_t tag_mask, int t_max) {
    if (rtp) {
        const int32_t h = rtp_header_len(pkt, C);
        if (!reverse) return cipher_may_throw(h, (int32_t)L - (h == kHdrThrow ? 0 : h));
        if (!(fl & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE)) || h == kHdrThrow) {
            for (int T = 0; T < 32; T++) {
                if (!(tag_mask & (1u << T))) continue;
                const int32_t newL = (int32_t)L - T > 0 ? (int32_t)L - T : 0;
                if (cipher_may_throw(h, newL - (h == kHdrThrow ? 0 : h))) return true;
            }
        }
        return false;
    }
    // getSRTCPIndex at length - 4 - tag, decryption from byte 8
    // (SRTCPCryptoContext.reverseTransformPacket :315-374)
    return reverse && (int32_t)L < 12 + t_max;
}

} // namespace

// Plan of one bundle: the shard of each packet and whether it could throw
// (see the file comment).  kinds[t] is transformer t's kind; tag_mask bit T
// is set when some policy of the dispatcher has tag length T (0 for NULL
// authentication).  Packets that need no engine (SKIP flag, bad transformer
// id) get shard -1.  Returns 2 if some packet could throw, else 1.
static int32_t plan_bundle(int32_t n_shards, int32_t abort_on_error, int32_t reverse,
                           const int32_t *kinds, int32_t n_transformers, uint32_t tag_mask,
                           const int32_t *tids, int32_t tid, const uint8_t *seg, const uint32_t *off,
                           const uint32_t *len, const uint32_t *cap, const uint32_t *flags, uint32_t n,
                           int32_t *shard, int32_t *may_throw) {
    int t_max = 0;
    for (int T = 0; T < 32; T++)
        if (tag_mask & (1u << T)) t_max = T;
    int32_t any = 0;
    for (uint32_t i = 0; i < n; i++) {
        const int32_t t = tids ? tids[i] : tid;
        const uint32_t fl = flags ? flags[i] : 0u;
        if (i + 16 < n) __builtin_prefetch(seg + off[i + 16]); // the loop is bound by these misses
        may_throw[i] = 0;
        if ((fl & SRTP_PKT_FLAG_SKIP) || t < 0 || t >= n_transformers) {
            shard[i] = -1;
            continue;
        }
        const uint32_t L = len[i], C = cap[i];
        const bool invalid = L < 12 || L > C || C > 65535u; // RawPacket.isInvalid :903-909
        const uint8_t *pkt = seg + off[i];
        const bool rtp = kinds[t] == SRTP_KIND_RTP;
        shard[i] = invalid ? 0
                           : (int32_t)(mix32(be32(pkt + (rtp ? 8 : 4))) % (uint32_t)n_shards);
        const bool mt = abort_on_error && !invalid && may_throw_one(rtp, reverse, pkt, L, C, fl, tag_mask, t_max);
        may_throw[i] = mt ? 1 : 0;
        any |= may_throw[i];
    }
    return any ? 2 : 1;
}

namespace {
// A FIFO mutex: callers get the dispatcher in the order they asked.  With a
// plain std::mutex, eight threads each calling srtp_dispatch_transform_host
// in a loop took the lock back-to-back from one another unevenly: p999 of a
// call was 183 ms against a p50 of 92 us (profiles/r05/).
class FairMutex {
  public:
    void lock() {
        std::unique_lock<std::mutex> lk(m_);
        const uint64_t t = next_++;
        cv_.wait(lk, [&] { return serving_ == t; });
    }
    void unlock() {
        {
            std::lock_guard<std::mutex> lk(m_);
            serving_++;
        }
        cv_.notify_all();
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    uint64_t next_ = 0, serving_ = 0;
};

// Fork-join helpers for the packet copies (pack / scatter).  run(parts, f)
// calls f(0..parts-1): the caller takes parts itself while helpers take the
// rest from the queue, so it never waits on a busy pool.
class CopyPool {
  public:
    explicit CopyPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    void run(int parts, const std::function<void(int)> &f) {
        if (parts <= 1 || th_.empty()) {
            for (int i = 0; i < parts; i++) f(i);
            return;
        }
        struct Job {
            std::atomic<int> next{0}, done{0};
        };
        auto job = std::make_shared<Job>();
        auto body = [job, parts, &f] {
            int i;
            while ((i = job->next.fetch_add(1)) < parts) {
                f(i);
                job->done.fetch_add(1);
            }
        };
        const int helpers = std::min(parts - 1, (int)th_.size());
        {
            std::lock_guard<std::mutex> lk(m_);
            for (int h = 0; h < helpers; h++) q_.push_back(body);
        }
        cv_.notify_all();
        body();
        while (job->done.load() < parts) std::this_thread::yield();
    }

  private:
    void loop() {
        for (;;) {
            std::function<void()> t;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                t = std::move(q_.front());
                q_.pop_front();
            }
            t();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
};

// copy helpers: the CPUs this process may run on beyond one per shard
// worker, at most 8
int copy_threads(int n_shards) {
    cpu_set_t cs;
    int ncpu = 4;
    if (sched_getaffinity(0, sizeof cs, &cs) == 0) ncpu = CPU_COUNT(&cs);
    return std::max(0, std::min(8, ncpu - n_shards));
}
} // namespace

// A host bundle (srtp_dispatch_submit_host): the caller's arrays, valid
// until its wait returns, and the shards' share of it.  Its chunks pass
// through the shards' pipeline slots; a chunk is drained (results back into
// the caller's arrays) when its slot is needed again -- by this bundle or
// the next one -- or by a wait.
struct HostBundle {
    uint64_t ticket = 0;
    int32_t reverse = 0;
    const int32_t *tids = nullptr;
    int32_t tid = -1;
    uint8_t *seg = nullptr;
    const uint32_t *off = nullptr, *cap = nullptr, *flags = nullptr;
    uint32_t *len = nullptr;
    int32_t *status = nullptr;
    bool registered = false; // the segment lies in registered memory (srtp_host_register)
    size_t seg_bytes = 0;
    std::vector<std::vector<uint32_t>> per_shard;
    std::atomic<int> chunks_out{0}; // chunks in slots, not yet drained
    std::atomic<int> rc{SRTP_OK};
};

// A shard's pipeline slots, in use across bundles: slot k holds the packets
// ch[0, n) of owner (null: free) -- a stretch of the index list the chunk was
// cut from, which lives as long as the chunk is in flight; k is the next slot
// to fill.
struct ShardRing {
    int k = 0;
    std::shared_ptr<HostBundle> owner[kDepth];
    const uint32_t *ch[kDepth] = {};
    size_t n[kDepth] = {};
    bool direct[kDepth] = {}; // the chunk runs in place in the caller's registered segment
};

struct srtp_dispatch {
    std::unique_ptr<CopyPool> pool;
    std::vector<srtp_engine *> engines;
    std::vector<srtp_pipeline *> pipes; // per shard, made by the first host bundle (nullptr until then)
    std::vector<char> shared;           // the shard's device hosts other shards too
    std::vector<int32_t> kinds;  // transformer kinds (replicated ids); written under mu and kmu
    uint32_t tag_mask = 0;
    int32_t abort_on_error = 1;
    FairMutex mu;                // control calls and host bundles, in arrival order
    std::mutex kmu;              // kinds (the vector)
    // transformer kinds for srtp_dispatch_route, read without a lock (it is
    // called once per packet by the aggregator's producers): -1 = no such id
    std::unique_ptr<std::atomic<int32_t>[]> route_kind;
    uint32_t n_route_kind = 0;
    // host time per phase of a bundle, summed over shards (srtp_dispatch_host_times)
    std::atomic<uint64_t> t_plan{0}, t_pack{0}, t_wait{0}, t_scatter{0}, t_total{0}, n_calls{0};
    std::string last_error;

    // worker threads, one per shard.  A job is a bundle's chunks on that shard
    // (idx: its packets; drain_all: then drain every slot, the synchronous
    // call and the rollback's runs), or -- b null -- a drain of the slots whose
    // bundles have tickets up to `upto` (a wait).
    struct Job {
        std::shared_ptr<HostBundle> b;
        const std::vector<uint32_t> *idx = nullptr;
        bool drain_all = false;
        uint64_t upto = 0;
        int32_t rc = SRTP_OK;
    };
    std::vector<std::thread> workers;
    std::vector<Job> jobs;
    std::vector<ShardRing> rings;
    std::mutex wmu;
    std::condition_variable cv_go, cv_done;
    uint64_t generation = 0;
    int pending = 0;
    bool stop = false;
    // bundles submitted and not yet waited for, in ticket order (under mu)
    std::deque<std::shared_ptr<HostBundle>> inflight;
    uint64_t next_ticket = 1;
};

namespace {

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int dfail(srtp_dispatch *d, int code, const std::string &msg) {
    d->last_error = msg;
    return code;
}

size_t region(uint32_t cap) { return ((size_t)cap + 15) & ~(size_t)15; }

// Copies packets [j0, j1) of a chunk (ch: their bundle indices) between a
// pipeline slot and the caller's segment, one memcpy per run of packets that
// lie back to back in both (the slot's are by construction; a one-shard
// bundle is then a single run): a call per 1.2-KB packet costs as much as its
// bytes.
template <bool ToSlot>
void copy_runs(const HostBundle &b, const srtp_pipeline_slot &sl, const uint32_t *ch, size_t j0, size_t j1) {
    for (size_t j = j0; j < j1;) {
        const uint32_t i = ch[j];
        size_t bytes = region(b.cap[i]);
        size_t e = j + 1;
        while (e < j1 && b.off[ch[e]] == b.off[ch[e - 1]] + region(b.cap[ch[e - 1]])) {
            bytes += region(b.cap[ch[e]]);
            e++;
        }
        uint8_t *slot = sl.seg + sl.off[j], *user = b.seg + b.off[i];
        if (ToSlot) memcpy(slot, user, bytes);
        else memcpy(user, slot, bytes);
        j = e;
    }
}

// Drains slot k of shard s: waits for its chunk and scatters statuses,
// lengths and (unless it ran in place) packet bytes back into its bundle.
void drain_slot(srtp_dispatch *d, int s, int k, const srtp_pipeline_slot &sl) {
    ShardRing &rg = d->rings[(size_t)s];
    std::shared_ptr<HostBundle> ob = std::move(rg.owner[k]);
    if (!ob) return;
    HostBundle &b = *ob;
    const uint64_t tw = now_ns();
    const int rc = srtp_pipeline_wait(d->pipes[(size_t)s], k);
    const uint64_t ts = now_ns();
    d->t_wait += ts - tw;
    const uint32_t *ch = rg.ch[k];
    const size_t nch = rg.n[k];
    if (rc != SRTP_OK) {
        int ok = SRTP_OK;
        b.rc.compare_exchange_strong(ok, rc);
        for (size_t j = 0; j < nch; j++) b.status[ch[j]] = SRTP_STATUS_ERR_INTERNAL;
    } else {
        const bool direct = rg.direct[k];
        const int parts = (int)std::min<size_t>((size_t)d->pool->size() + 1, (nch + 1023) / 1024);
        d->pool->run(parts, [&](int q) {
            const size_t j0 = nch * q / parts, j1 = nch * (q + 1) / parts;
            for (size_t j = j0; j < j1; j++) {
                const uint32_t i = ch[j];
                b.status[i] = sl.status[j];
                b.len[i] = sl.len[j];
            }
            if (!direct) copy_runs<false>(b, sl, ch, j0, j1);
        });
        d->t_scatter += now_ns() - ts;
    }
    b.chunks_out.fetch_sub(1, std::memory_order_acq_rel);
}

// Shard s's share of bundle b (its packets idx) through the shard's pipeline
// slots, after the chunks of earlier bundles still in them: each slot is
// drained when it is needed again.  The last chunks stay in flight unless
// drain_all, so that the caller's next bundle overlaps them.
int run_shard(srtp_dispatch *d, int s, HostBundle &b, const std::shared_ptr<HostBundle> &bp,
              const std::vector<uint32_t> &idx, bool drain_all) {
    srtp_pipeline *pl = d->pipes[(size_t)s];
    ShardRing &rg = d->rings[(size_t)s];
    srtp_pipeline_slot sl[kDepth];
    for (int k = 0; k < kDepth; k++) {
        int rc = srtp_pipeline_slot_get(pl, k, &sl[k]);
        if (rc != SRTP_OK) return rc;
    }
    int rc_all = SRTP_OK;
    size_t pos = 0;
    std::vector<uint32_t> src; // a gathered chunk's packet offsets in the caller's segment
    while (pos < idx.size()) {
        const int k = rg.k;
        drain_slot(d, s, k, sl[k]);
        const uint64_t tp = now_ns();
        // the chunk's extent and layout (offsets only: one pass over the caps)
        const uint32_t *ch = idx.data() + pos;
        const size_t room = std::min<size_t>(idx.size() - pos, sl[k].max_packets);
        size_t bytes = 0, nch = 0;
        bool contig = true; // the chunk's packets lie back to back in the caller's segment
        for (; nch < room; nch++) {
            const uint32_t i = ch[nch];
            const size_t r = region(b.cap[i]);
            if (bytes + r > sl[k].seg_cap) break;
            if (nch && b.off[i] != b.off[ch[nch - 1]] + region(b.cap[ch[nch - 1]])) contig = false;
            sl[k].off[nch] = (uint32_t)bytes;
            bytes += r;
        }
        if (nch == 0) { // a packet larger than a slot (cannot happen: cap <= 65535)
            rc_all = SRTP_EINVAL;
            break;
        }
        // a registered segment whose chunk is one run: the DMA reads and
        // writes the caller's bytes in place; else the packet bytes go
        // through the slot.  Either way the per-packet arrays, and the copies,
        // are split over the copy helpers.
        // a registered segment whose chunk is scattered over it (a shard's
        // share of an interleaved bundle): the GPU gathers the packets over
        // PCIe and writes them back (srtp_pipeline_submit_gather) -- no host
        // copy of their bytes either (round 6; was two memcpy passes)
        const bool direct = b.registered && contig;
        const bool gather = b.registered && !contig && nch <= kGatherMax;
        if (gather) src.resize(nch);
        {
            const int parts = (int)std::min<size_t>((size_t)d->pool->size() + 1, (nch + 1023) / 1024);
            d->pool->run(parts, [&](int q) {
                const size_t j0 = nch * q / parts, j1 = nch * (q + 1) / parts;
                for (size_t j = j0; j < j1; j++) {
                    const uint32_t i = ch[j];
                    sl[k].len[j] = b.len[i];
                    sl[k].cap[j] = b.cap[i];
                    sl[k].flags[j] = b.flags ? b.flags[i] : 0u;
                    sl[k].tids[j] = b.tids ? b.tids[i] : b.tid;
                    if (gather) src[j] = b.off[i];
                }
                if (!direct && !gather) copy_runs<true>(b, sl[k], ch, j0, j1);
            });
        }
        const int rc = direct ? srtp_pipeline_submit_host(pl, k, b.reverse, 1, -1, 1, (uint32_t)nch, bytes, -1,
                                                          b.seg + b.off[ch[0]])
                       : gather ? srtp_pipeline_submit_gather(pl, k, b.reverse, 1, -1, 1, (uint32_t)nch, bytes, -1,
                                                              b.seg, b.seg_bytes, src.data())
                              : srtp_pipeline_submit(pl, k, b.reverse, 1, -1, 1, (uint32_t)nch, bytes);
        d->t_pack += now_ns() - tp; // the enqueue of the chunk's copies and kernels included
        if (rc != SRTP_OK) {
            rc_all = rc;
            break;
        }
        rg.owner[k] = bp;
        rg.ch[k] = ch;
        rg.n[k] = nch;
        rg.direct[k] = direct || gather;
        b.chunks_out.fetch_add(1, std::memory_order_acq_rel);
        pos += nch;
        rg.k = (k + 1) % kDepth;
    }
    // packets never submitted (an error) get an explicit status; every chunk
    // in flight still comes back, its results the caller's
    for (size_t q = pos; q < idx.size(); q++) b.status[idx[q]] = SRTP_STATUS_ERR_INTERNAL;
    if (drain_all || rc_all != SRTP_OK)
        for (int q = 0; q < kDepth; q++) {
            const int k = (rg.k + q) % kDepth;
            drain_slot(d, s, k, sl[k]);
        }
    return rc_all;
}

// Drains, oldest first, the slots of shard s whose bundles have tickets up
// to `upto` (a wait for one of them).
int drain_upto(srtp_dispatch *d, int s, uint64_t upto) {
    srtp_pipeline *pl = d->pipes[(size_t)s];
    if (!pl) return SRTP_OK;
    ShardRing &rg = d->rings[(size_t)s];
    for (int q = 0; q < kDepth; q++) {
        const int k = (rg.k + q) % kDepth;
        if (!rg.owner[k] || rg.owner[k]->ticket > upto) continue;
        srtp_pipeline_slot sl;
        const int rc = srtp_pipeline_slot_get(pl, k, &sl);
        if (rc != SRTP_OK) return rc;
        drain_slot(d, s, k, sl);
    }
    return SRTP_OK;
}

void worker_main(srtp_dispatch *d, int s) {
    uint64_t seen = 0;
    for (;;) {
        std::unique_lock<std::mutex> lk(d->wmu);
        d->cv_go.wait(lk, [&] { return d->stop || d->generation != seen; });
        if (d->stop) return;
        seen = d->generation;
        srtp_dispatch::Job job = d->jobs[(size_t)s];
        lk.unlock();
        int rc = SRTP_OK;
        if (!job.b) rc = drain_upto(d, s, job.upto);
        else if (job.idx && !job.idx->empty()) rc = run_shard(d, s, *job.b, job.b, *job.idx, job.drain_all);
        job = srtp_dispatch::Job{}; // drop the bundle reference before reporting
        lk.lock();
        d->jobs[(size_t)s].rc = rc;
        if (--d->pending == 0) d->cv_done.notify_all();
    }
}

// Runs one phase on every shard at once; returns the first error.  b null:
// drain the slots of the bundles with tickets up to `upto`.
int run_phase(srtp_dispatch *d, const std::shared_ptr<HostBundle> &b,
              const std::vector<std::vector<uint32_t>> *per_shard, bool drain_all, uint64_t upto = 0) {
    std::unique_lock<std::mutex> lk(d->wmu);
    for (size_t s = 0; s < d->engines.size(); s++) {
        d->jobs[s].b = b;
        d->jobs[s].idx = per_shard ? &(*per_shard)[s] : nullptr;
        d->jobs[s].drain_all = drain_all;
        d->jobs[s].upto = upto;
        d->jobs[s].rc = SRTP_OK;
    }
    d->pending = (int)d->engines.size();
    d->generation++;
    d->cv_go.notify_all();
    d->cv_done.wait(lk, [&] { return d->pending == 0; });
    int rc = SRTP_OK;
    for (auto &j : d->jobs) {
        if (j.rc != SRTP_OK && rc == SRTP_OK) rc = j.rc;
        j.b.reset();
    }
    return rc;
}

// Calls f(engine) on every shard; fails unless every shard returns the same id.
int replicate(srtp_dispatch *d, const std::function<int(srtp_engine *, int32_t *)> &f, int32_t *out) {
    int32_t id0 = -1;
    for (size_t s = 0; s < d->engines.size(); s++) {
        int32_t id = -1;
        const int rc = f(d->engines[s], &id);
        if (rc != SRTP_OK)
            return dfail(d, rc, std::string("shard ") + std::to_string(s) + ": " +
                                    srtp_engine_last_error(d->engines[s]));
        if (s == 0) id0 = id;
        else if (id != id0) return dfail(d, SRTP_EINVAL, "shard ids diverged");
    }
    if (out) *out = id0;
    return SRTP_OK;
}

int each(srtp_dispatch *d, const std::function<int(srtp_engine *)> &f) {
    for (size_t s = 0; s < d->engines.size(); s++) {
        const int rc = f(d->engines[s]);
        if (rc != SRTP_OK)
            return dfail(d, rc, std::string("shard ") + std::to_string(s) + ": " +
                                    srtp_engine_last_error(d->engines[s]));
    }
    return SRTP_OK;
}

} // namespace

extern "C" {

int32_t srtp_shard_of(uint32_t ssrc, int32_t n_shards) {
    return n_shards > 0 ? (int32_t)(mix32(ssrc) % (uint32_t)n_shards) : -1;
}

int32_t srtp_dispatch_route(srtp_dispatch *d, int32_t tid, const uint8_t *pkt, uint32_t len) {
    if (!d || (!pkt && len)) return -1;
    if (tid < 0 || (uint32_t)tid >= d->n_route_kind) return -1;
    const int32_t kind = d->route_kind[(size_t)tid].load(std::memory_order_acquire);
    if (kind < 0) return -1;
    if (len < 12) return 0; // RawPacket.isInvalid: shard 0 reports it (DROP_INVALID)
    return (int32_t)(mix32(be32(pkt + (kind == SRTP_KIND_RTP ? 8 : 4))) % (uint32_t)d->engines.size());
}

int32_t srtp_dispatch_plan(int32_t n_shards, int32_t abort_on_error, int32_t reverse,
                           const int32_t *kinds, int32_t n_transformers, uint32_t tag_mask,
                           const int32_t *tids, int32_t tid, const uint8_t *seg, size_t seg_bytes,
                           const uint32_t *off, const uint32_t *len, const uint32_t *cap,
                           const uint32_t *flags, uint32_t n, int32_t *shard, int32_t *may_throw) {
    if (n_shards < 1 || !kinds || n_transformers < 0 || (n && (!seg || !off || !len || !cap ||
                                                               !shard || !may_throw)))
        return SRTP_EINVAL;
    for (uint32_t i = 0; i < n; i++)
        if (off[i] % 16 != 0 || cap[i] > 65535u || (uint64_t)off[i] + region(cap[i]) > seg_bytes)
            return SRTP_EINVAL;
    return plan_bundle(n_shards, abort_on_error, reverse, kinds, n_transformers, tag_mask, tids, tid,
                       seg, off, len, cap, flags, n, shard, may_throw);
}

int32_t srtp_packet_may_throw(int32_t kind, int32_t reverse, const uint8_t *pkt, uint32_t len, uint32_t cap,
                              uint32_t flags, uint32_t tag_mask) {
    if (!pkt || (flags & SRTP_PKT_FLAG_SKIP) || len < 12 || len > cap || cap > 65535u) return 0;
    int t_max = 0;
    for (int T = 0; T < 32; T++)
        if (tag_mask & (1u << T)) t_max = T;
    return may_throw_one(kind == SRTP_KIND_RTP, reverse, pkt, len, cap, flags, tag_mask, t_max) ? 1 : 0;
}

void srtp_dispatch_destroy(srtp_dispatch *d) {
    if (!d) return;
    if (!d->workers.empty() && !d->inflight.empty()) { // bundles never waited for: their results first
        std::lock_guard<FairMutex> g(d->mu);
        (void)run_phase(d, nullptr, nullptr, false, UINT64_MAX);
        d->inflight.clear();
    }
    {
        std::lock_guard<std::mutex> lk(d->wmu);
        d->stop = true;
    }
    d->cv_go.notify_all();
    for (auto &w : d->workers)
        if (w.joinable()) w.join();
    d->pool.reset();
    for (auto *p : d->pipes)
        if (p) srtp_pipeline_destroy(p);
    for (auto *e : d->engines) srtp_engine_destroy(e);
    delete d;
}

int srtp_dispatch_create(const int32_t *devices, int32_t n_shards, const srtp_engine_opts *opts,
                         srtp_dispatch **out) {
    if (!devices || n_shards < 1 || n_shards > 256 || !out) return SRTP_EINVAL;
    *out = nullptr;
    srtp_dispatch *d = new (std::nothrow) srtp_dispatch();
    if (!d) return SRTP_ENOMEM;
    srtp_engine_opts o;
    if (opts) o = *opts;
    else srtp_engine_opts_default(&o);
    d->abort_on_error = o.abort_on_error;
    d->n_route_kind = o.max_transformers;
    d->route_kind.reset(new (std::nothrow) std::atomic<int32_t>[o.max_transformers]);
    if (!d->route_kind) {
        delete d;
        return SRTP_ENOMEM;
    }
    for (uint32_t t = 0; t < o.max_transformers; t++) d->route_kind[t].store(-1);
    int rc = SRTP_OK;
    try {
        d->pool.reset(new CopyPool(copy_threads(n_shards)));
    } catch (...) {
        rc = SRTP_ENOMEM;
    }
    for (int32_t s = 0; s < n_shards && rc == SRTP_OK; s++) {
        srtp_engine_opts os = o;
        os.device = devices[s];
        srtp_engine *e = nullptr;
        rc = srtp_engine_create(&os, &e);
        if (rc != SRTP_OK) break;
        d->engines.push_back(e);
        // the shard's pipeline (pinned chunk slots, copy streams) is made by
        // the first host bundle (srtp_dispatch_transform_host): a process that
        // only uses the aggregator over the dispatcher never holds its 192 MB
        // of pinned memory per shard, nor its two streams (which shared the
        // device's few hardware queues with the aggregator lanes' streams)
        d->pipes.push_back(nullptr);
        d->shared.push_back(std::count(devices, devices + n_shards, devices[s]) > 1);
    }
    if (rc == SRTP_OK) {
        d->jobs.resize((size_t)n_shards);
        d->rings.resize((size_t)n_shards);
        try {
            for (int32_t s = 0; s < n_shards; s++) d->workers.emplace_back(worker_main, d, (int)s);
        } catch (...) {
            rc = SRTP_ENOMEM;
        }
    }
    if (rc != SRTP_OK) {
        srtp_dispatch_destroy(d);
        return rc;
    }
    *out = d;
    return SRTP_OK;
}

const char *srtp_dispatch_last_error(srtp_dispatch *d) { return d ? d->last_error.c_str() : ""; }

int32_t srtp_dispatch_num_shards(srtp_dispatch *d) { return d ? (int32_t)d->engines.size() : 0; }

srtp_engine *srtp_dispatch_engine(srtp_dispatch *d, int32_t shard) {
    if (!d || shard < 0 || (size_t)shard >= d->engines.size()) return nullptr;
    return d->engines[(size_t)shard];
}

int srtp_dispatch_factory_create(srtp_dispatch *d, int32_t sender, const uint8_t *master_key,
                                 int32_t key_len, const uint8_t *master_salt, int32_t salt_len,
                                 const srtp_policy *srtp, const srtp_policy *srtcp, int32_t *out) {
    if (!d || !srtp || !srtcp) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    const int rc = replicate(d, [&](srtp_engine *e, int32_t *id) {
        return srtp_factory_create(e, sender, master_key, key_len, master_salt, salt_len, srtp, srtcp, id);
    }, out);
    if (rc != SRTP_OK) return rc;
    for (const srtp_policy *p : {srtp, srtcp}) {
        const int T = p->auth_type == SRTP_NULL_AUTHENTICATION ? 0 : p->auth_tag_len;
        if (T >= 0 && T < 32) d->tag_mask |= 1u << T;
    }
    return SRTP_OK;
}

int srtp_dispatch_factory_close(srtp_dispatch *d, int32_t factory) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return each(d, [&](srtp_engine *e) { return srtp_factory_close(e, factory); });
}

int srtp_dispatch_transformer_create(srtp_dispatch *d, int32_t kind, int32_t fwd, int32_t rev,
                                     int32_t *out) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    int32_t id = -1;
    const int rc = replicate(d, [&](srtp_engine *e, int32_t *x) {
        return srtp_transformer_create(e, kind, fwd, rev, x);
    }, &id);
    if (rc != SRTP_OK) return rc;
    std::lock_guard<std::mutex> kg(d->kmu);
    if ((size_t)id >= d->kinds.size()) d->kinds.resize((size_t)id + 1, SRTP_KIND_RTP);
    d->kinds[(size_t)id] = kind;
    if ((uint32_t)id < d->n_route_kind) d->route_kind[(size_t)id].store(kind, std::memory_order_release);
    if (out) *out = id;
    return SRTP_OK;
}

int srtp_dispatch_transformer_set_factory(srtp_dispatch *d, int32_t t, int32_t f, int32_t forward) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return each(d, [&](srtp_engine *e) { return srtp_transformer_set_factory(e, t, f, forward); });
}

int srtp_dispatch_transformer_close(srtp_dispatch *d, int32_t t) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return each(d, [&](srtp_engine *e) { return srtp_transformer_close(e, t); });
}

namespace {
// One host bundle, under d->mu.  Synchronous (ticket null): returns when its
// results are in the caller's arrays.  Asynchronous: returns once every chunk
// is on its way, the last ones still in flight, with the bundle's ticket for
// srtp_dispatch_wait_host.  A bundle that may throw (the rollback below) runs
// synchronously either way.
int submit_locked(srtp_dispatch *d, int32_t reverse, const int32_t *tids, int32_t tid, uint8_t *seg,
                  size_t seg_bytes, const uint32_t *off, uint32_t *len, const uint32_t *cap,
                  const uint32_t *flags, int32_t *status, uint32_t n, uint64_t *ticket) {
    const bool async = ticket != nullptr;
    auto bp = std::make_shared<HostBundle>();
    bp->ticket = d->next_ticket++;
    auto finish = [&](int rc) { // the bundle's outcome: async callers get it from the wait
        if (async && rc == SRTP_OK) {
            d->inflight.push_back(bp);
            *ticket = bp->ticket;
        }
        return rc;
    };
    if (n == 0) return finish(SRTP_OK);
    if (!seg || !off || !len || !cap || !status) return dfail(d, SRTP_EINVAL, "null buffer");
    const uint64_t t0 = now_ns();
    struct Done { // the call's total host time, however it returns
        srtp_dispatch *d;
        uint64_t t0;
        ~Done() {
            d->t_total += now_ns() - t0;
            d->n_calls++;
        }
    } done{d, t0};
    const int32_t nt = (int32_t)d->kinds.size();
    if (!tids && (tid < 0 || tid >= nt)) return dfail(d, SRTP_EINVAL, "bad transformer id");
    const size_t ns = d->engines.size();
    std::vector<int32_t> shard(n), mt(n);
    // The plan (srtp_dispatch_plan: region checks, each packet's shard and
    // may-throw mark) and the per-shard index lists, split over the copy
    // helpers: each part plans its range and counts its packets per shard, and
    // then fills its stretch of each shard's list (bundle order kept).
    const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)d->pool->size() + 1, (n + 16383) / 16384));
    std::vector<int32_t> plan_p((size_t)parts, 1);
    std::vector<uint32_t> cnt((size_t)parts * ns, 0u);
    // a throw aborts its transformer's later packets across the shard's
    // chunks only through the plan's rollback; one chunk needs no plan
    const bool fast1 = ns == 1 && (!d->abort_on_error || (n <= kChunkPackets && seg_bytes <= kChunkBytes));
    d->pool->run(parts, [&](int q) {
        const uint32_t lo = (uint32_t)((uint64_t)n * q / parts), hi = (uint32_t)((uint64_t)n * (q + 1) / parts);
        if (fast1) {
            // one shard and one chunk (or no abort-on-throw): the engine applies
            // abort-on-throw itself, so no packet needs reading -- only the
            // region checks and which packets run
            int32_t r = 1;
            for (uint32_t i = lo; i < hi; i++) {
                if (off[i] % 16 != 0 || cap[i] > 65535u || (uint64_t)off[i] + region(cap[i]) > seg_bytes) r = SRTP_EINVAL;
                const int32_t t = tids ? tids[i] : tid;
                shard[i] = ((flags && (flags[i] & SRTP_PKT_FLAG_SKIP)) || t < 0 || t >= nt) ? -1 : 0;
                mt[i] = 0;
            }
            plan_p[(size_t)q] = r;
        } else {
            plan_p[(size_t)q] = srtp_dispatch_plan((int32_t)ns, d->abort_on_error, reverse, d->kinds.data(), nt,
                                                   d->tag_mask, tids ? tids + lo : nullptr, tid, seg, seg_bytes,
                                                   off + lo, len + lo, cap + lo, flags ? flags + lo : nullptr,
                                                   hi - lo, shard.data() + lo, mt.data() + lo);
        }
        uint32_t *c = cnt.data() + (size_t)q * ns;
        for (uint32_t i = lo; i < hi; i++)
            if (shard[i] >= 0) c[shard[i]]++;
    });
    int32_t plan = 1;
    for (int32_t x : plan_p) {
        if (x < 0) return dfail(d, x, "packet region outside the segment");
        plan = std::max(plan, x);
    }
    HostBundle &b = *bp;
    b.reverse = reverse;
    b.tids = tids; b.tid = tid; b.seg = seg; b.off = off; b.len = len;
    b.cap = cap; b.flags = flags; b.status = status;
    b.registered = srtp_host_is_registered(seg, seg_bytes) != 0;
    b.seg_bytes = seg_bytes;
    for (size_t s = 0; s < ns; s++) {
        if (d->pipes[s]) continue;
        // shards sharing a GPU: one stream each (SRTP_PIPE_ONE_STREAM); the
        // other shards' chunks keep that GPU's copy engines and CUs busy
        const int rc = srtp_pipeline_create_ex(d->engines[s], kChunkPackets, kChunkBytes, kDepth,
                                               d->shared[s] ? SRTP_PIPE_ONE_STREAM : 0u, &d->pipes[s]);
        if (rc != SRTP_OK) return dfail(d, rc, "shard pipeline");
    }
    auto tid_of = [&](uint32_t i) { return tids ? tids[i] : tid; };
    std::vector<std::vector<uint32_t>> &per_shard = b.per_shard;
    per_shard.resize(ns);
    std::vector<uint32_t> at((size_t)parts * ns);
    for (size_t s = 0; s < ns; s++) {
        uint32_t acc = 0;
        for (int q = 0; q < parts; q++) {
            at[(size_t)q * ns + s] = acc;
            acc += cnt[(size_t)q * ns + s];
        }
        per_shard[s].resize(acc);
    }
    d->pool->run(parts, [&](int q) {
        const uint32_t lo = (uint32_t)((uint64_t)n * q / parts), hi = (uint32_t)((uint64_t)n * (q + 1) / parts);
        uint32_t *a = at.data() + (size_t)q * ns;
        for (uint32_t i = lo; i < hi; i++) {
            if (shard[i] < 0) status[i] = SRTP_STATUS_SKIPPED; // SKIP flag or no such transformer
            else per_shard[(size_t)shard[i]][a[shard[i]]++] = i;
        }
    });
    d->t_plan += now_ns() - t0;
    if (plan == 1) { // nothing can throw: one run
        int rc = run_phase(d, bp, &per_shard, !async);
        if (rc == SRTP_OK && !async) rc = b.rc.load();
        if (rc != SRTP_OK && async) // no ticket: nothing of this bundle may stay in flight
            (void)run_phase(d, nullptr, nullptr, false, bp->ticket);
        return rc == SRTP_OK ? finish(SRTP_OK) : dfail(d, rc, "shard bundle failed");
    }
    // The rollback needs every earlier bundle's results and this one's whole
    // run: the bundles in flight come back first.
    {
        const int rc = run_phase(d, nullptr, nullptr, false, UINT64_MAX);
        if (rc != SRTP_OK) return dfail(d, rc, "shard bundle failed");
    }
    // Transformers that could throw: their contexts in this bundle are
    // snapshotted per shard and their packets' input bytes stashed.
    std::vector<char> risky((size_t)nt, 0);
    for (uint32_t i = 0; i < n; i++)
        if (mt[i]) risky[(size_t)tid_of(i)] = 1;
    // RawPacket.isInvalid of the packet as handed in (the lengths change in the run)
    std::vector<char> valid0(n);
    for (uint32_t i = 0; i < n; i++) valid0[i] = len[i] >= 12 && len[i] <= cap[i];
    auto valid = [&](uint32_t i) { return valid0[i] != 0; };
    auto ssrc_of = [&](uint32_t i) {
        return be32(seg + off[i] + (d->kinds[(size_t)tid_of(i)] == SRTP_KIND_RTP ? 8 : 4));
    };
    auto key_of = [&](uint32_t i) { return ((uint64_t)(uint32_t)tid_of(i) << 32) | ssrc_of(i); };
    struct Snap {
        std::vector<uint64_t> keys;
        std::vector<srtp_ctx_raw> st;
        std::vector<int32_t> present;
    };
    std::vector<Snap> snap(ns);
    std::vector<uint8_t> stash;
    std::vector<size_t> stash_at(n, SIZE_MAX);
    std::vector<uint32_t> stash_len(n, 0);
    for (size_t sh = 0; sh < ns; sh++) {
        Snap &sn = snap[sh];
        for (uint32_t i : per_shard[sh]) {
            if (!risky[(size_t)tid_of(i)]) continue;
            stash_at[i] = stash.size();
            stash_len[i] = len[i];
            stash.insert(stash.end(), seg + off[i], seg + off[i] + region(cap[i]));
            if (valid(i)) sn.keys.push_back(key_of(i));
        }
        std::sort(sn.keys.begin(), sn.keys.end());
        sn.keys.erase(std::unique(sn.keys.begin(), sn.keys.end()), sn.keys.end());
        if (sn.keys.empty()) continue;
        std::vector<int32_t> kt(sn.keys.size());
        std::vector<uint32_t> ks(sn.keys.size());
        for (size_t q = 0; q < sn.keys.size(); q++) {
            kt[q] = (int32_t)(sn.keys[q] >> 32);
            ks[q] = (uint32_t)sn.keys[q];
        }
        sn.st.resize(sn.keys.size());
        sn.present.resize(sn.keys.size());
        const int rc = srtp_contexts_save(d->engines[sh], (uint32_t)kt.size(), kt.data(), ks.data(),
                                          sn.st.data(), sn.present.data());
        if (rc != SRTP_OK)
            return dfail(d, rc, std::string("shard ") + std::to_string(sh) + ": " +
                                    srtp_engine_last_error(d->engines[sh]));
    }
    int rc = run_phase(d, bp, &per_shard, true);
    if (rc == SRTP_OK) rc = b.rc.load();
    if (rc != SRTP_OK) return dfail(d, rc, "shard bundle failed");
    // e_t: each risky transformer's first throw over all shards
    std::vector<int64_t> e_first((size_t)nt, -1);
    for (uint32_t i = 0; i < n; i++)
        if (shard[i] >= 0 && status[i] == SRTP_STATUS_ERR_MALFORMED && e_first[(size_t)tid_of(i)] < 0)
            e_first[(size_t)tid_of(i)] = i;
    // t's packets after e_t are rolled back; the contexts they touched are
    // dirty.  Everything the rollback needs is checked before anything is
    // changed, so a failure (a throw the plan did not foresee: cannot happen
    // by construction) returns the bundle as the run left it -- packets and
    // contexts consistent with each other -- never half rolled back.
    std::vector<std::vector<uint64_t>> dirty(ns);
    std::vector<uint32_t> undo;
    for (uint32_t i = 0; i < n; i++) {
        if (shard[i] < 0) continue;
        const int64_t e = e_first[(size_t)tid_of(i)];
        if (e < 0 || (int64_t)i <= e) continue;
        if (stash_at[i] == SIZE_MAX) return dfail(d, SRTP_EINVAL, "rollback: a throw the plan did not foresee");
        if (status[i] != SRTP_STATUS_NOT_PROCESSED && valid(i)) dirty[(size_t)shard[i]].push_back(key_of(i));
        undo.push_back(i);
    }
    // the snapshot entries of the dirty contexts, per shard
    std::vector<std::vector<size_t>> snap_at(ns);
    bool any_dirty = false;
    for (size_t sh = 0; sh < ns; sh++) {
        std::vector<uint64_t> &dk = dirty[sh];
        std::sort(dk.begin(), dk.end());
        dk.erase(std::unique(dk.begin(), dk.end()), dk.end());
        const Snap &sn = snap[sh];
        for (uint64_t k : dk) {
            const size_t q = (size_t)(std::lower_bound(sn.keys.begin(), sn.keys.end(), k) - sn.keys.begin());
            if (q >= sn.keys.size() || sn.keys[q] != k)
                return dfail(d, SRTP_EINVAL, "rollback: context not in the snapshot");
            snap_at[sh].push_back(q);
            any_dirty = true;
        }
    }
    for (uint32_t i : undo) {
        status[i] = SRTP_STATUS_NOT_PROCESSED;
        memcpy(seg + off[i], stash.data() + stash_at[i], region(cap[i]));
        len[i] = stash_len[i];
    }
    if (!any_dirty) return finish(SRTP_OK);
    // Reset the dirty contexts, then re-run t's packets up to e_t on them.
    std::vector<std::vector<uint32_t>> rerun(ns);
    for (size_t sh = 0; sh < ns; sh++) {
        std::vector<uint64_t> &dk = dirty[sh];
        if (dk.empty()) continue;
        const Snap &sn = snap[sh];
        std::vector<int32_t> kt, pr;
        std::vector<uint32_t> ks;
        std::vector<srtp_ctx_raw> st;
        for (size_t j = 0; j < dk.size(); j++) {
            const uint64_t k = dk[j];
            const size_t q = snap_at[sh][j];
            kt.push_back((int32_t)(k >> 32));
            ks.push_back((uint32_t)k);
            st.push_back(sn.st[q]);
            pr.push_back(sn.present[q]);
        }
        rc = srtp_contexts_restore(d->engines[sh], (uint32_t)kt.size(), kt.data(), ks.data(), st.data(),
                                   pr.data());
        if (rc != SRTP_OK)
            return dfail(d, rc, std::string("shard ") + std::to_string(sh) + ": " +
                                    srtp_engine_last_error(d->engines[sh]));
        for (uint32_t i : per_shard[sh]) {
            const int64_t e = e_first[(size_t)tid_of(i)];
            if (e < 0 || (int64_t)i > e || !valid(i)) continue;
            if (!std::binary_search(dk.begin(), dk.end(), key_of(i))) continue;
            memcpy(seg + off[i], stash.data() + stash_at[i], region(cap[i]));
            len[i] = stash_len[i];
            rerun[sh].push_back(i);
        }
    }
    rc = run_phase(d, bp, &rerun, true);
    if (rc == SRTP_OK) rc = b.rc.load();
    return rc == SRTP_OK ? finish(SRTP_OK) : dfail(d, rc, "shard bundle failed (rollback re-run)");
}
} // namespace

int srtp_dispatch_transform_host(srtp_dispatch *d, int32_t reverse, const int32_t *tids, int32_t tid,
                                 uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                                 const uint32_t *cap, const uint32_t *flags, int32_t *status,
                                 uint32_t n) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return submit_locked(d, reverse, tids, tid, seg, seg_bytes, off, len, cap, flags, status, n, nullptr);
}

int srtp_dispatch_submit_host(srtp_dispatch *d, int32_t reverse, const int32_t *tids, int32_t tid,
                              uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                              const uint32_t *cap, const uint32_t *flags, int32_t *status, uint32_t n,
                              uint64_t *ticket) {
    if (!d || !ticket) return SRTP_EINVAL;
    *ticket = 0;
    std::lock_guard<FairMutex> g(d->mu);
    if (d->inflight.size() >= kMaxInflight) return dfail(d, SRTP_EAGAIN, "too many host bundles in flight");
    return submit_locked(d, reverse, tids, tid, seg, seg_bytes, off, len, cap, flags, status, n, ticket);
}

int srtp_dispatch_wait_host(srtp_dispatch *d, uint64_t ticket) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    auto it = std::find_if(d->inflight.begin(), d->inflight.end(),
                           [&](const std::shared_ptr<HostBundle> &b) { return b->ticket == ticket; });
    if (it == d->inflight.end()) return dfail(d, SRTP_EINVAL, "no such host bundle in flight");
    const std::shared_ptr<HostBundle> b = *it;
    if (b->chunks_out.load(std::memory_order_acquire) != 0) {
        // drains this bundle's slots and those of the bundles before it
        const int rc = run_phase(d, nullptr, nullptr, false, ticket);
        if (rc != SRTP_OK) return dfail(d, rc, "shard bundle failed");
    }
    d->inflight.erase(std::find(d->inflight.begin(), d->inflight.end(), b));
    const int rc = b->rc.load();
    return rc == SRTP_OK ? SRTP_OK : dfail(d, rc, "shard bundle failed");
}

int srtp_dispatch_host_times(srtp_dispatch *d, uint64_t ns[6]) {
    if (!d || !ns) return SRTP_EINVAL;
    ns[0] = d->t_plan; ns[1] = d->t_pack; ns[2] = d->t_wait; ns[3] = d->t_scatter;
    ns[4] = d->t_total; ns[5] = d->n_calls;
    return SRTP_OK;
}

int srtp_dispatch_get_context_state(srtp_dispatch *d, int32_t t, uint32_t ssrc, srtp_ctx_state *out) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return srtp_get_context_state(d->engines[(size_t)srtp_shard_of(ssrc, (int32_t)d->engines.size())], t,
                                  ssrc, out);
}

int srtp_dispatch_set_context_state(srtp_dispatch *d, int32_t t, uint32_t ssrc, int32_t forward,
                                    const srtp_ctx_state *st) {
    if (!d) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    return srtp_set_context_state(d->engines[(size_t)srtp_shard_of(ssrc, (int32_t)d->engines.size())], t,
                                  ssrc, forward, st);
}

int srtp_dispatch_stats(srtp_dispatch *d, srtp_stats *out) {
    if (!d || !out) return SRTP_EINVAL;
    std::lock_guard<FairMutex> g(d->mu);
    memset(out, 0, sizeof *out);
    return each(d, [&](srtp_engine *e) {
        srtp_stats s;
        const int rc = srtp_engine_stats(e, &s);
        if (rc != SRTP_OK) return rc;
        uint64_t *dst = reinterpret_cast<uint64_t *>(out);
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&s);
        for (size_t k = 0; k < sizeof s / sizeof(uint64_t); k++) dst[k] += src[k];
        return SRTP_OK;
    });
}

} // extern "C"
