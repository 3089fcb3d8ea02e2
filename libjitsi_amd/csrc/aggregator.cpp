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
// Concurrency.  A submit reserves its packet's place (index, bytes) in the
// open slot of its lane and direction with one compare-and-swap on a packed
// reservation word -- no lock, and the only read-modify-write a submit makes
// on memory other threads write -- and copies the packet, storing its length
// last; only opening, sealing and freeing slots take the aggregator's lock
// (once per bundle, not per packet).  A sealed slot is handed to the engine
// once every reserved packet's length has been stored (lengths start as a
// sentinel).  Callbacks run on the lanes'
// dispatch threads.  A callback may submit (an SFU forwarding what it just
// received); such a submit never waits for a slot -- only the dispatch
// threads free slots, so waiting could deadlock.  When no slot is free it
// parks a copy of the packet in the lane's overflow queue, which the lane's
// thread moves into the first slot it frees, ahead of other producers, so a
// forwarded packet is never refused.  flush and destroy from a callback
// return SRTP_EINVAL.
//
// Per-packet semantics: each submitted packet is its own 1-element
// RawPacket[] in the reference, so one packet's exception must not stop
// later packets of the same transformer in the bundle.  The engines therefore
// run with abort_on_error = 0 (creation refuses otherwise); a packet the
// reference would throw on completes with SRTP_STATUS_ERR_MALFORMED.
#include <atomic>
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
constexpr uint32_t kNoLen = 0xffffffffu; // h.len[i] until packet i's copy has finished

// Reservation word of a lane direction's open slot: slot + 1 (0 = none) in
// bits 56-63, packets reserved in bits 32-55, segment bytes in bits 0-31.
constexpr uint64_t resv_pack(uint32_t slot1, uint32_t n, uint32_t bytes) {
    return ((uint64_t)slot1 << 56) | ((uint64_t)n << 32) | bytes;
}
constexpr uint32_t resv_slot1(uint64_t r) { return (uint32_t)(r >> 56); }
constexpr uint32_t resv_n(uint64_t r) { return (uint32_t)(r >> 32) & 0xffffffu; }
constexpr uint32_t resv_bytes(uint64_t r) { return (uint32_t)r; }

struct Slot {
    SlotState state = kFree;                 // under the aggregator's lock
    int32_t reverse = 0;
    uint32_t n = 0;                          // packets, final once sealed
    size_t bytes = 0;                        // segment bytes, final once sealed
    uint32_t ready = 0;                      // h.len[0 .. ready) seen stored (lane thread)
    Clock::time_point first;
    std::vector<uint64_t> cookies;
    srtp_pipeline_slot h{};
};

// a callback's packet parked until a slot frees (see the file comment)
struct Parked {
    int32_t reverse, tid;
    uint32_t flags;
    uint64_t cookie;
    std::vector<uint8_t> pkt;
};

struct Lane {
    srtp_engine *e = nullptr;
    srtp_pipeline *pl = nullptr;
    std::unique_ptr<Slot[]> slots;
    int n_slots = 0;
    std::atomic<uint64_t> resv[2] = {{0}, {0}}; // open slot per direction
    std::deque<int> sealed, inflight;
    std::deque<Parked> parked;
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
    uint64_t completed = 0, bundles = 0;
    int error = SRTP_OK;
    std::string last_error;
    std::thread flusher;
};

namespace {

// Seals direction dir's open slot of the lane (no more reservations); a slot
// nobody reserved in goes back to the free list.
void seal_locked(Lane &ln, int dir) {
    const uint64_t r = ln.resv[dir].exchange(0);
    if (!resv_slot1(r)) return;
    Slot &sl = ln.slots[resv_slot1(r) - 1];
    sl.n = resv_n(r);
    sl.bytes = resv_bytes(r);
    if (sl.n == 0) {
        sl.state = kFree;
        ln.cv_space.notify_all();
        return;
    }
    sl.state = kSealed;
    sl.ready = 0;
    ln.sealed.push_back(resv_slot1(r) - 1);
    ln.cv_work.notify_all();
}

// A free slot of the lane; producers (not in a callback) only take one when
// another stays free, so a callback's submit usually finds a slot at once.
int free_slot_locked(Lane &ln, bool in_cb) {
    int first = -1, n_free = 0;
    for (int i = 0; i < ln.n_slots; i++)
        if (ln.slots[i].state == kFree) {
            if (first < 0) first = i;
            n_free++;
        }
    return (in_cb ? n_free >= 1 : n_free >= 2) ? first : -1;
}

void open_locked(srtp_aggregator *a, Lane &ln, int dir, int s) {
    Slot &sl = ln.slots[s];
    sl.state = kOpen;
    sl.reverse = dir;
    sl.n = 0;
    sl.bytes = 0;
    sl.first = Clock::now();
    ln.resv[dir].store(resv_pack((uint32_t)s + 1u, 0, 0));
    a->cv_flush.notify_all(); // the flusher learns the new deadline
}

// Fast path: reserve (index, offset) in the open slot of direction dir.
// False when there is none or it has no room.
bool try_reserve(const srtp_aggregator *a, Lane &ln, int dir, size_t need, int &s, uint32_t &i,
                 size_t &off) {
    uint64_t r = ln.resv[dir].load();
    for (;;) {
        const uint32_t s1 = resv_slot1(r);
        if (!s1 || resv_n(r) >= a->opts.max_packets || resv_bytes(r) + need > a->opts.max_bytes)
            return false;
        const uint64_t nr = resv_pack(s1, resv_n(r) + 1u, resv_bytes(r) + (uint32_t)need);
        if (ln.resv[dir].compare_exchange_weak(r, nr)) {
            s = (int)s1 - 1;
            i = resv_n(r);
            off = resv_bytes(r);
            return true;
        }
    }
}

// Copies the packet into its reserved place; its length, stored last, marks
// it complete for the lane's thread.
void fill(Lane &ln, int s, uint32_t i, size_t off, int32_t tid, const uint8_t *pkt, uint32_t len, uint32_t cap,
          size_t need, uint32_t flags, uint64_t cookie) {
    Slot &sl = ln.slots[s];
    if (len) memcpy(sl.h.seg + off, pkt, len);
    if (need > len) memset(sl.h.seg + off + len, 0, need - len);
    sl.h.off[i] = (uint32_t)off;
    sl.h.cap[i] = cap;
    sl.h.flags[i] = flags;
    sl.h.tids[i] = tid;
    sl.cookies[i] = cookie;
    __atomic_store_n(&sl.h.len[i], len, __ATOMIC_RELEASE);
}

// True when every packet reserved in sealed slot sl has been copied.
bool slot_ready(Slot &sl) {
    while (sl.ready < sl.n && __atomic_load_n(&sl.h.len[sl.ready], __ATOMIC_ACQUIRE) != kNoLen) sl.ready++;
    return sl.ready == sl.n;
}

// Packets accepted and not yet completed (under the lock).
uint64_t pending_locked(const srtp_aggregator *a) {
    uint64_t n = 0;
    for (const auto &ln : a->lanes) {
        for (int s = 0; s < ln->n_slots; s++)
            if (ln->slots[s].state == kSealed || ln->slots[s].state == kInflight) n += ln->slots[s].n;
        for (int d = 0; d < 2; d++) n += resv_n(ln->resv[d].load());
        n += ln->parked.size();
    }
    return n;
}

size_t need_of(uint32_t cap) { return ((size_t)cap + 15u) & ~(size_t)15u; }

// Places parked callback packets into slots (the lane's thread, after it
// freed one); stops when no slot is left.
void place_parked_locked(srtp_aggregator *a, Lane &ln) {
    while (!ln.parked.empty()) {
        Parked &pk = ln.parked.front();
        const int dir = pk.reverse ? 1 : 0;
        const uint32_t len = (uint32_t)pk.pkt.size();
        const uint32_t cap = pk.reverse ? len : len + 16u;
        const size_t need = need_of(cap);
        int s;
        uint32_t i;
        size_t off;
        if (!try_reserve(a, ln, dir, need, s, i, off)) {
            seal_locked(ln, dir);
            const int f = free_slot_locked(ln, true);
            if (f < 0) return;
            open_locked(a, ln, dir, f);
            if (!try_reserve(a, ln, dir, need, s, i, off)) return; // cannot happen: need <= max_bytes
        }
        fill(ln, s, i, off, pk.tid, pk.pkt.data(), len, cap, need, pk.flags, pk.cookie);
        if (i + 1u == a->opts.max_packets) seal_locked(ln, dir);
        ln.parked.pop_front();
    }
}

void lane_loop(srtp_aggregator *a, Lane *ln) {
    std::unique_lock<std::mutex> lk(a->mu);
    // keep up to depth - 2 bundles in flight (one slot per open direction)
    const size_t max_inflight = ln->n_slots > 2 ? (size_t)ln->n_slots - 2 : 1;
    for (;;) {
        bool straggler = false; // a sealed slot still being copied into
        auto can_submit = [&] {
            straggler = false;
            if (ln->sealed.empty() || ln->inflight.size() >= max_inflight) return false;
            straggler = !slot_ready(ln->slots[ln->sealed.front()]);
            return !straggler;
        };
        auto go = [&] { return a->stop || can_submit() || !ln->inflight.empty(); };
        while (!go()) {
            if (straggler) ln->cv_work.wait_for(lk, std::chrono::microseconds(20)); // copies take ~0.1 us
            else ln->cv_work.wait(lk);
        }
        if (a->stop && ln->sealed.empty() && ln->inflight.empty() && ln->parked.empty()) return;
        if (can_submit()) {
            const int s = ln->sealed.front();
            ln->sealed.pop_front();
            Slot &sl = ln->slots[s];
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
        Slot &sl = ln->slots[s];
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
        for (uint32_t i = 0; i < sl.n; i++) sl.h.len[i] = kNoLen;
        sl.state = kFree;
        sl.n = 0;
        sl.bytes = 0;
        place_parked_locked(a, *ln);
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
                const uint32_t s1 = resv_slot1(ln->resv[d].load());
                if (!s1) continue;
                const Clock::time_point due = ln->slots[s1 - 1].first + deadline;
                if (due <= Clock::now()) seal_locked(*ln, d);
                else if (due < wake) wake = due;
            }
        }
        a->cv_flush.wait_until(lk, wake);
    }
}

void seal_all_locked(srtp_aggregator *a) {
    for (auto &ln : a->lanes) {
        seal_locked(*ln, 0);
        seal_locked(*ln, 1);
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
    // the reservation word holds 24 bits of packets and 32 of bytes
    if (o.max_packets == 0 || o.max_packets > 0xffffffu || o.max_bytes < 64 ||
        o.max_bytes > 0xffffffffull || o.depth < 3 || o.depth > 16)
        return SRTP_EINVAL;
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
        ln.n_slots = o.depth;
        ln.slots.reset(new Slot[(size_t)o.depth]);
        for (int i = 0; i < o.depth; i++) {
            srtp_pipeline_slot_get(ln.pl, i, &ln.slots[i].h);
            ln.slots[i].cookies.resize(o.max_packets);
            for (uint32_t k = 0; k < o.max_packets; k++) ln.slots[i].h.len[k] = kNoLen;
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
    const size_t need = need_of(cap);
    if (need > a->opts.max_bytes) return SRTP_EINVAL;
    size_t lane = 0;
    if (a->d) {
        const int32_t sh = srtp_dispatch_route(a->d, tid, pkt, len);
        lane = sh < 0 ? 0 : (size_t)sh; // an unknown transformer: the engine reports it SKIPPED
    }
    Lane &ln = *a->lanes[lane];
    const bool in_cb = tl_in_callback == a;
    int s;
    uint32_t i;
    size_t off;
    if (!try_reserve(a, ln, dir, need, s, i, off)) {
        std::unique_lock<std::mutex> lk(a->mu);
        for (;;) {
            if (a->stop) return SRTP_EINVAL;
            if (try_reserve(a, ln, dir, need, s, i, off)) break;
            seal_locked(ln, dir); // full (or none open)
            const int f = free_slot_locked(ln, in_cb);
            if (f >= 0) {
                open_locked(a, ln, dir, f);
                continue;
            }
            if (in_cb) { // never wait for a slot from a callback: park the packet
                ln.parked.push_back(Parked{dir, tid, flags, cookie, std::vector<uint8_t>(pkt, pkt + len)});
                return SRTP_OK;
            }
            ln.cv_space.wait(lk); // backpressure: every slot is sealed or in flight
        }
    }
    fill(ln, s, i, off, tid, pkt, len, cap, need, flags, cookie);
    if (i + 1u == a->opts.max_packets) { // the reservation that filled the slot seals it
        std::lock_guard<std::mutex> lk(a->mu);
        const uint64_t r = ln.resv[dir].load();
        if (resv_slot1(r) == (uint32_t)s + 1u && resv_n(r) == a->opts.max_packets) seal_locked(ln, dir);
    }
    return SRTP_OK;
}

int srtp_aggregator_flush(srtp_aggregator *a) {
    if (!a) return SRTP_EINVAL;
    if (tl_in_callback == a) return SRTP_EINVAL; // would wait for its own callback
    std::unique_lock<std::mutex> lk(a->mu);
    seal_all_locked(a);
    const uint64_t target = a->completed + pending_locked(a);
    a->cv_idle.wait(lk, [&] {
        if (a->completed >= target) return true;
        seal_all_locked(a); // parked callback packets placed since then
        return false;
    });
    return a->error;
}

int srtp_aggregator_stats(srtp_aggregator *a, uint64_t *accepted, uint64_t *completed,
                          uint64_t *bundles) {
    if (!a) return SRTP_EINVAL;
    std::lock_guard<std::mutex> lk(a->mu);
    if (accepted) *accepted = a->completed + pending_locked(a);
    if (completed) *completed = a->completed;
    if (bundles) *bundles = a->bundles;
    return a->error;
}

void srtp_aggregator_destroy(srtp_aggregator *a) {
    if (!a || tl_in_callback == a) return; // from its own callback: refused (see the header)
    {
        std::unique_lock<std::mutex> lk(a->mu);
        seal_all_locked(a);
        const uint64_t target = a->completed + pending_locked(a);
        a->cv_idle.wait(lk, [&] {
            if (a->completed >= target) return true;
            seal_all_locked(a);
            return false;
        });
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
