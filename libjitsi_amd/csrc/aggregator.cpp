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
// waited `deadline_us`.
//
// Lanes.  Over one engine there is one lane; over a dispatcher
// (srtp_aggregator_create_dispatch) one lane per shard, and a packet goes to
// the lane of its SSRC's shard (srtp_dispatch_route), so per-packet submits
// from one JVM reach every GPU.  Each lane has its own pinned slots and its
// own dispatch thread, which submits the lane's sealed bundles in sealing
// order and, when each completes, calls the callback once per packet in
// bundle order -- so packets of one lane (one shard, hence one context) and
// one direction complete in the order they were accepted.
//
// Concurrency.  A submit reserves its packet's place (slot, index, bytes)
// under the aggregator's lock and copies the packet outside it; a sealed
// slot is handed to the engine only when the copies into it have finished
// (Slot::writers).  Callbacks run on the lanes' dispatch threads.  A
// callback may submit (an SFU forwarding what it just received), but such a
// submit never waits for a free slot -- only the dispatch threads free slots,
// so waiting could deadlock -- and returns SRTP_EFULL instead; flush and
// destroy from a callback return SRTP_EINVAL.  So that callbacks rarely see
// SRTP_EFULL, producers leave one slot of each lane free: only a callback's
// submit opens a lane's last free slot.  A bundle holds at most max_packets
// packets, so the callbacks of one completed bundle can forward all of its
// packets (a bundle's worth fits the reserved slot, and the completed slot
// restores the reserve once its callbacks have run) unless the forwarded
// packets outgrow max_bytes.
//
// Per-packet semantics: each submitted packet is its own 1-element
// RawPacket[] in the reference, so one packet's exception must not stop
// later packets of the same transformer in the bundle.  The engines therefore
// run with abort_on_error = 0 (creation refuses otherwise); a packet the
// reference would throw on completes with SRTP_STATUS_ERR_MALFORMED.
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
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
    uint32_t n = 0;         // packets reserved
    size_t bytes = 0;       // segment bytes reserved
    uint32_t writers = 0;   // submits still copying into the slot
    Clock::time_point first;
    std::vector<uint64_t> cookies;
    srtp_pipeline_slot h{};
};

struct Lane {
    srtp_engine *e = nullptr;
    srtp_pipeline *pl = nullptr;
    std::vector<Slot> slots;
    int open[2] = {-1, -1}; // open slot per direction
    std::deque<int> sealed, inflight;
    std::condition_variable cv_work;  // the lane's dispatch thread: something to do
    std::condition_variable cv_space; // producers: a slot of this lane became free
    std::thread thread;
};

thread_local const void *tl_in_callback = nullptr; // the aggregator whose callback runs here
} // namespace

struct srtp_aggregator {
    srtp_dispatch *d = nullptr; // dispatch mode: lane = shard
    srtp_aggregator_opts opts{};
    srtp_aggregator_cb cb = nullptr;
    void *user = nullptr;

    std::mutex mu;
    std::condition_variable cv_flush; // the flusher: a new deadline
    std::condition_variable cv_idle;  // flush(): everything completed
    std::vector<std::unique_ptr<Lane>> lanes;
    bool stop = false;
    uint64_t accepted = 0, completed = 0, bundles = 0;
    int error = SRTP_OK;
    std::string last_error;
    std::thread flusher;
};

namespace {

void seal_locked(srtp_aggregator *a, Lane &ln, int dir) {
    const int s = ln.open[dir];
    if (s < 0) return;
    ln.open[dir] = -1;
    ln.slots[(size_t)s].state = kSealed;
    ln.sealed.push_back(s);
    ln.cv_work.notify_all();
    (void)a;
}

// a free slot of the lane; producers (not in a callback) only take one when
// another stays free for callbacks
int free_slot_locked(Lane &ln, bool in_cb) {
    int first = -1, n_free = 0;
    for (size_t i = 0; i < ln.slots.size(); i++)
        if (ln.slots[i].state == kFree) {
            if (first < 0) first = (int)i;
            n_free++;
        }
    return (in_cb ? n_free >= 1 : n_free >= 2) ? first : -1;
}

void lane_loop(srtp_aggregator *a, Lane *ln) {
    std::unique_lock<std::mutex> lk(a->mu);
    // keep up to depth - 2 bundles in flight (one slot per open direction)
    const size_t max_inflight = ln->slots.size() > 2 ? ln->slots.size() - 2 : 1;
    for (;;) {
        auto can_submit = [&] {
            return !ln->sealed.empty() && ln->inflight.size() < max_inflight &&
                   ln->slots[(size_t)ln->sealed.front()].writers == 0;
        };
        ln->cv_work.wait(lk, [&] { return a->stop || can_submit() || !ln->inflight.empty(); });
        if (a->stop && ln->sealed.empty() && ln->inflight.empty()) return;
        if (can_submit()) {
            const int s = ln->sealed.front();
            ln->sealed.pop_front();
            Slot &sl = ln->slots[(size_t)s];
            sl.state = kInflight;
            ln->inflight.push_back(s);
            const uint32_t n = sl.n;
            const size_t bytes = sl.bytes;
            const int32_t rev = sl.reverse;
            lk.unlock(); // the slot is ours: producers only touch open slots
            const int rc = srtp_pipeline_submit(ln->pl, s, rev, 1, -1, 1, n, bytes);
            lk.lock();
            if (rc != SRTP_OK) {
                a->error = rc;
                a->last_error = srtp_engine_last_error(ln->e);
                for (uint32_t i = 0; i < n; i++) sl.h.status[i] = -1; // reported below as failed
            }
            continue;
        }
        if (ln->inflight.empty()) continue; // stop requested with sealed slots still being written
        const int s = ln->inflight.front();
        Slot &sl = ln->slots[(size_t)s];
        lk.unlock();
        (void)srtp_pipeline_wait(ln->pl, s);
        // callbacks outside the lock, in bundle order
        tl_in_callback = a;
        for (uint32_t i = 0; i < sl.n; i++) {
            const int32_t st = sl.h.status[i];
            a->cb(a->user, sl.cookies[i], st, sl.h.seg + sl.h.off[i], sl.h.len[i]);
        }
        tl_in_callback = nullptr;
        lk.lock();
        ln->inflight.pop_front();
        a->completed += sl.n;
        a->bundles++;
        sl.state = kFree;
        sl.n = 0;
        sl.bytes = 0;
        ln->cv_space.notify_all();
        a->cv_idle.notify_all();
    }
}

void flush_loop(srtp_aggregator *a) {
    const auto deadline = std::chrono::microseconds(a->opts.deadline_us);
    std::unique_lock<std::mutex> lk(a->mu);
    while (!a->stop) {
        Clock::time_point wake = Clock::now() + std::chrono::milliseconds(50);
        for (auto &ln : a->lanes) {
            for (int d = 0; d < 2; d++) {
                const int s = ln->open[d];
                if (s < 0) continue;
                const Clock::time_point due = ln->slots[(size_t)s].first + deadline;
                if (due <= Clock::now()) seal_locked(a, *ln, d);
                else if (due < wake) wake = due;
            }
        }
        a->cv_flush.wait_until(lk, wake);
    }
}

void seal_all_locked(srtp_aggregator *a) {
    for (auto &ln : a->lanes) {
        seal_locked(a, *ln, 0);
        seal_locked(a, *ln, 1);
    }
}

void destroy_lanes(srtp_aggregator *a) {
    for (auto &ln : a->lanes)
        if (ln->pl) srtp_pipeline_destroy(ln->pl);
    a->lanes.clear();
}

int create(srtp_dispatch *d, srtp_engine *const *engines, size_t n_lanes, const srtp_aggregator_opts *opts,
           srtp_aggregator_cb cb, void *user, srtp_aggregator **out) {
    if (!cb || !out || n_lanes == 0) return SRTP_EINVAL;
    *out = nullptr;
    srtp_aggregator_opts o;
    if (opts) o = *opts;
    else srtp_aggregator_opts_default(&o);
    if (o.max_packets == 0 || o.max_bytes < 64 || o.depth < 3 || o.depth > 16) return SRTP_EINVAL;
    for (size_t l = 0; l < n_lanes; l++) {
        srtp_engine_opts eo;
        if (!engines[l] || srtp_engine_get_opts(engines[l], &eo) != SRTP_OK || eo.abort_on_error)
            return SRTP_EINVAL;
    }
    srtp_aggregator *a = new (std::nothrow) srtp_aggregator();
    if (!a) return SRTP_ENOMEM;
    a->d = d;
    a->opts = o;
    a->cb = cb;
    a->user = user;
    for (size_t l = 0; l < n_lanes; l++) {
        a->lanes.emplace_back(new Lane());
        Lane &ln = *a->lanes.back();
        ln.e = engines[l];
        const int rc = srtp_pipeline_create(ln.e, o.max_packets, o.max_bytes, o.depth, &ln.pl);
        if (rc != SRTP_OK) {
            destroy_lanes(a);
            delete a;
            return rc;
        }
        ln.slots.resize((size_t)o.depth);
        for (int i = 0; i < o.depth; i++) {
            srtp_pipeline_slot_get(ln.pl, i, &ln.slots[(size_t)i].h);
            ln.slots[(size_t)i].cookies.resize(o.max_packets);
        }
    }
    for (auto &ln : a->lanes) ln->thread = std::thread(lane_loop, a, ln.get());
    a->flusher = std::thread(flush_loop, a);
    *out = a;
    return SRTP_OK;
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
    if (!e) return SRTP_EINVAL;
    return create(nullptr, &e, 1, opts, cb, user, out);
}

int srtp_aggregator_create_dispatch(srtp_dispatch *d, const srtp_aggregator_opts *opts,
                                    srtp_aggregator_cb cb, void *user, srtp_aggregator **out) {
    if (!d) return SRTP_EINVAL;
    std::vector<srtp_engine *> es((size_t)srtp_dispatch_num_shards(d));
    for (size_t s = 0; s < es.size(); s++) es[s] = srtp_dispatch_engine(d, (int32_t)s);
    return create(d, es.data(), es.size(), opts, cb, user, out);
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
    size_t lane = 0;
    if (a->d) {
        const int32_t sh = srtp_dispatch_route(a->d, tid, pkt, len);
        lane = sh < 0 ? 0 : (size_t)sh; // an unknown transformer: the engine reports it SKIPPED
    }
    Lane &ln = *a->lanes[lane];
    const bool in_cb = tl_in_callback == a;
    std::unique_lock<std::mutex> lk(a->mu);
    if (a->stop) return SRTP_EINVAL;
    for (;;) {
        int s = ln.open[dir];
        if (s >= 0) {
            Slot &sl = ln.slots[(size_t)s];
            if (sl.n < a->opts.max_packets && sl.bytes + need <= a->opts.max_bytes) break;
            seal_locked(a, ln, dir);
        }
        s = free_slot_locked(ln, in_cb);
        if (s >= 0) {
            Slot &sl = ln.slots[(size_t)s];
            sl.state = kOpen;
            sl.reverse = reverse ? 1 : 0;
            sl.n = 0;
            sl.bytes = 0;
            sl.writers = 0;
            sl.first = Clock::now();
            ln.open[dir] = s;
            a->cv_flush.notify_all(); // the flusher learns the new deadline
            break;
        }
        if (in_cb) return SRTP_EFULL; // only the dispatch threads free slots: never wait on one
        ln.cv_space.wait(lk); // backpressure: every slot is sealed or in flight
        if (a->stop) return SRTP_EINVAL;
    }
    const int s = ln.open[dir];
    Slot &sl = ln.slots[(size_t)s];
    const uint32_t i = sl.n++;
    const size_t off = sl.bytes;
    sl.bytes += need;
    sl.writers++;
    a->accepted++;
    if (sl.n == a->opts.max_packets) seal_locked(a, ln, dir);
    lk.unlock();
    // the packet's place is reserved: copy it without the lock
    if (len) memcpy(sl.h.seg + off, pkt, len);
    if (need > len) memset(sl.h.seg + off + len, 0, need - len);
    sl.h.off[i] = (uint32_t)off;
    sl.h.len[i] = len;
    sl.h.cap[i] = cap;
    sl.h.flags[i] = flags;
    sl.h.tids[i] = tid;
    sl.cookies[i] = cookie;
    lk.lock();
    if (--sl.writers == 0 && sl.state == kSealed) ln.cv_work.notify_all();
    return SRTP_OK;
}

int srtp_aggregator_flush(srtp_aggregator *a) {
    if (!a) return SRTP_EINVAL;
    if (tl_in_callback == a) return SRTP_EINVAL; // would wait for its own callback
    std::unique_lock<std::mutex> lk(a->mu);
    seal_all_locked(a);
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
    if (!a || tl_in_callback == a) return; // from its own callback: refused (see the header)
    {
        std::unique_lock<std::mutex> lk(a->mu);
        seal_all_locked(a);
        const uint64_t target = a->accepted;
        a->cv_idle.wait(lk, [&] { return a->completed >= target; });
        a->stop = true;
        a->cv_flush.notify_all();
        for (auto &ln : a->lanes) {
            ln->cv_work.notify_all();
            ln->cv_space.notify_all();
        }
    }
    for (auto &ln : a->lanes) ln->thread.join();
    a->flusher.join();
    destroy_lanes(a);
    delete a;
}

} // extern "C"
