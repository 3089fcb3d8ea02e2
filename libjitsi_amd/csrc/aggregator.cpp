// aggregator.cpp -- bundle aggregator over srtp_pipeline_* (SURVEY.md 8f.2).
//
// The reference moves packets one at a time: RTPConnectorInputStream.read
// hands each received datagram to the transform chain as a 1-element array
// (RTPConnectorInputStream.java:425-452), and RTPConnectorOutputStream's
// send loop does the same per outgoing packet (RTPConnectorOutputStream.java
// :268-300,652-830), each through SinglePacketTransformer
// (SinglePacketTransformer.java:121-216).  The engine wants bundles.  This
// layer takes those per-packet calls from any number of threads
// (srtp_aggregator_submit), packs them into the pipeline's pinned slots, and
// seals a bundle when it is full (packets or bytes) or its oldest packet has
// waited `deadline_us`.  One dispatch thread submits sealed bundles in sealing
// order and, when each completes, calls the callback once per packet in
// bundle order -- so packets of one transformer (in fact all packets of one
// direction) complete in the order they were accepted.
//
// Per-packet semantics: each submitted packet is its own 1-element
// RawPacket[] in the reference, so one packet's exception must not stop
// later packets of the same transformer in the bundle.  The engine therefore
// has to run with abort_on_error = 0 (srtp_aggregator_create refuses
// otherwise); a packet the reference would throw on completes with
// SRTP_STATUS_ERR_MALFORMED.
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string.h>
#include <string>
#include <thread>
#include <vector>

#include "../../include/srtp_mi355x.h"

namespace {
using Clock = std::chrono::steady_clock;

enum SlotState { kFree, kOpen, kSealed, kInflight };

struct Slot {
    SlotState state = kFree;
    int32_t reverse = 0;
    uint32_t n = 0;
    size_t bytes = 0;
    Clock::time_point first;
    std::vector<uint64_t> cookies;
    srtp_pipeline_slot h{};
};
} // namespace

struct srtp_aggregator {
    srtp_engine *e = nullptr;
    srtp_pipeline *pl = nullptr;
    srtp_aggregator_opts opts{};
    srtp_aggregator_cb cb = nullptr;
    void *user = nullptr;

    std::mutex mu;
    std::condition_variable cv_work;  // dispatcher / flusher: something to do
    std::condition_variable cv_space; // producers: a slot became free
    std::condition_variable cv_idle;  // flush(): everything completed
    std::vector<Slot> slots;
    int open[2] = {-1, -1};           // open slot per direction
    std::deque<int> sealed, inflight;
    bool stop = false;
    uint64_t accepted = 0, completed = 0, bundles = 0;
    int error = SRTP_OK;
    std::string last_error;
    std::thread dispatcher, flusher;
};

namespace {

void seal_locked(srtp_aggregator *a, int dir) {
    const int s = a->open[dir];
    if (s < 0) return;
    a->open[dir] = -1;
    a->slots[(size_t)s].state = kSealed;
    a->sealed.push_back(s);
    a->cv_work.notify_all();
}

int free_slot_locked(srtp_aggregator *a) {
    for (size_t i = 0; i < a->slots.size(); i++)
        if (a->slots[i].state == kFree) return (int)i;
    return -1;
}

void dispatch_loop(srtp_aggregator *a) {
    std::unique_lock<std::mutex> lk(a->mu);
    for (;;) {
        a->cv_work.wait(lk, [&] { return a->stop || !a->sealed.empty() || !a->inflight.empty(); });
        if (a->stop && a->sealed.empty() && a->inflight.empty()) return;
        // keep up to depth - 2 bundles in flight (one slot per open direction)
        const size_t max_inflight = a->slots.size() > 2 ? a->slots.size() - 2 : 1;
        if (!a->sealed.empty() && a->inflight.size() < max_inflight) {
            const int s = a->sealed.front();
            a->sealed.pop_front();
            Slot &sl = a->slots[(size_t)s];
            sl.state = kInflight;
            a->inflight.push_back(s);
            const uint32_t n = sl.n;
            const size_t bytes = sl.bytes;
            const int32_t rev = sl.reverse;
            lk.unlock(); // the slot is ours: producers only touch open slots
            const int rc = srtp_pipeline_submit(a->pl, s, rev, 1, -1, 1, n, bytes);
            lk.lock();
            if (rc != SRTP_OK) {
                a->error = rc;
                a->last_error = srtp_engine_last_error(a->e);
                for (uint32_t i = 0; i < n; i++) sl.h.status[i] = -1; // reported below as failed
            }
            continue;
        }
        const int s = a->inflight.front();
        Slot &sl = a->slots[(size_t)s];
        lk.unlock();
        (void)srtp_pipeline_wait(a->pl, s);
        // callbacks outside the lock, in bundle order
        for (uint32_t i = 0; i < sl.n; i++) {
            const int32_t st = sl.h.status[i];
            a->cb(a->user, sl.cookies[i], st, sl.h.seg + sl.h.off[i], sl.h.len[i]);
        }
        lk.lock();
        a->inflight.pop_front();
        a->completed += sl.n;
        a->bundles++;
        sl.state = kFree;
        sl.n = 0;
        sl.bytes = 0;
        sl.cookies.clear();
        a->cv_space.notify_all();
        a->cv_idle.notify_all();
    }
}

void flush_loop(srtp_aggregator *a) {
    const auto deadline = std::chrono::microseconds(a->opts.deadline_us);
    std::unique_lock<std::mutex> lk(a->mu);
    while (!a->stop) {
        Clock::time_point wake = Clock::now() + std::chrono::milliseconds(50);
        for (int d = 0; d < 2; d++) {
            const int s = a->open[d];
            if (s < 0) continue;
            const Clock::time_point due = a->slots[(size_t)s].first + deadline;
            if (due <= Clock::now()) seal_locked(a, d);
            else if (due < wake) wake = due;
        }
        a->cv_work.wait_until(lk, wake);
    }
}

} // namespace

extern "C" {

int srtp_aggregator_opts_default(srtp_aggregator_opts *o) {
    if (!o) return SRTP_EINVAL;
    o->max_packets = 1u << 14;
    o->max_bytes = (size_t)24 << 20;
    o->deadline_us = 1000;
    o->depth = 4;
    return SRTP_OK;
}

int srtp_aggregator_create(srtp_engine *e, const srtp_aggregator_opts *opts, srtp_aggregator_cb cb,
                           void *user, srtp_aggregator **out) {
    if (!e || !cb || !out) return SRTP_EINVAL;
    *out = nullptr;
    srtp_aggregator_opts o;
    if (opts) o = *opts;
    else srtp_aggregator_opts_default(&o);
    if (o.max_packets == 0 || o.max_bytes < 64 || o.depth < 3 || o.depth > 16) return SRTP_EINVAL;
    srtp_engine_opts eo;
    if (srtp_engine_get_opts(e, &eo) != SRTP_OK || eo.abort_on_error) return SRTP_EINVAL;
    srtp_aggregator *a = new (std::nothrow) srtp_aggregator();
    if (!a) return SRTP_ENOMEM;
    a->e = e;
    a->opts = o;
    a->cb = cb;
    a->user = user;
    int rc = srtp_pipeline_create(e, o.max_packets, o.max_bytes, o.depth, &a->pl);
    if (rc != SRTP_OK) {
        delete a;
        return rc;
    }
    a->slots.resize((size_t)o.depth);
    for (int i = 0; i < o.depth; i++) {
        srtp_pipeline_slot_get(a->pl, i, &a->slots[(size_t)i].h);
        a->slots[(size_t)i].cookies.reserve(o.max_packets);
    }
    a->dispatcher = std::thread(dispatch_loop, a);
    a->flusher = std::thread(flush_loop, a);
    *out = a;
    return SRTP_OK;
}

int srtp_aggregator_submit(srtp_aggregator *a, int32_t reverse, int32_t tid, const uint8_t *pkt,
                           uint32_t len, uint32_t flags, uint64_t cookie) {
    if (!a || (!pkt && len) || len > 65535u - 16u) return SRTP_EINVAL;
    const int dir = reverse ? 1 : 0;
    // protect appends up to 16 bytes (SRTCP E|index + a 12-byte tag): the
    // in-place form of RawPacket.append / grow; unprotect only shrinks
    const uint32_t cap = reverse ? len : len + 16u;
    const size_t need = ((size_t)cap + 15u) & ~(size_t)15u;
    if (need > a->opts.max_bytes) return SRTP_EINVAL;
    std::unique_lock<std::mutex> lk(a->mu);
    if (a->stop) return SRTP_EINVAL;
    for (;;) {
        int s = a->open[dir];
        if (s >= 0) {
            Slot &sl = a->slots[(size_t)s];
            if (sl.n < a->opts.max_packets && sl.bytes + need <= a->opts.max_bytes) break;
            seal_locked(a, dir);
        }
        s = free_slot_locked(a);
        if (s >= 0) {
            Slot &sl = a->slots[(size_t)s];
            sl.state = kOpen;
            sl.reverse = reverse ? 1 : 0;
            sl.n = 0;
            sl.bytes = 0;
            sl.first = Clock::now();
            a->open[dir] = s;
            a->cv_work.notify_all(); // the flusher learns the new deadline
            break;
        }
        a->cv_space.wait(lk); // backpressure: every slot is sealed or in flight
        if (a->stop) return SRTP_EINVAL;
    }
    Slot &sl = a->slots[(size_t)a->open[dir]];
    const uint32_t i = sl.n;
    const uint32_t off = (uint32_t)sl.bytes;
    if (len) memcpy(sl.h.seg + off, pkt, len);
    if (need > len) memset(sl.h.seg + off + len, 0, need - len);
    sl.h.off[i] = off;
    sl.h.len[i] = len;
    sl.h.cap[i] = cap;
    sl.h.flags[i] = flags;
    sl.h.tids[i] = tid;
    sl.cookies.push_back(cookie);
    sl.n++;
    sl.bytes += need;
    a->accepted++;
    if (sl.n == a->opts.max_packets) seal_locked(a, dir);
    return SRTP_OK;
}

int srtp_aggregator_flush(srtp_aggregator *a) {
    if (!a) return SRTP_EINVAL;
    std::unique_lock<std::mutex> lk(a->mu);
    seal_locked(a, 0);
    seal_locked(a, 1);
    const uint64_t target = a->accepted;
    a->cv_idle.wait(lk, [&] { return a->completed >= target; });
    return a->error;
}

int srtp_aggregator_stats(srtp_aggregator *a, uint64_t *accepted, uint64_t *completed,
                          uint64_t *bundles) {
    if (!a) return SRTP_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    if (accepted) *accepted = a->accepted;
    if (completed) *completed = a->completed;
    if (bundles) *bundles = a->bundles;
    return a->error;
}

void srtp_aggregator_destroy(srtp_aggregator *a) {
    if (!a) return;
    {
        std::unique_lock<std::mutex> lk(a->mu);
        seal_locked(a, 0);
        seal_locked(a, 1);
        const uint64_t target = a->accepted;
        a->cv_idle.wait(lk, [&] { return a->completed >= target; });
        a->stop = true;
        a->cv_work.notify_all();
        a->cv_space.notify_all();
    }
    a->dispatcher.join();
    a->flusher.join();
    srtp_pipeline_destroy(a->pl);
    delete a;
}

} // extern "C"
