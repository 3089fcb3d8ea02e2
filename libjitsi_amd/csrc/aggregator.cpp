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
// Concurrency.  Each producer thread fills blocks of 16 consecutive packet
// entries of the open slot of its lane and direction (with a byte range of
// the segment): it takes a block with one compare-and-swap on the slot's
// reservation word, then claims the block's entries one at a time with a
// compare-and-swap on the block's own cache line, which no other thread
// touches until the slot is sealed.  So producers share no written cache
// line per packet (the entries' metadata of a block fill whole lines), and
// the aggregator's lock is taken only to open, seal and free slots.  A packet
// is copied with its length stored last; a sealed slot goes to the engine once
// every claimed entry's length has been stored (lengths start as a
// sentinel).  Sealing closes every block: entries nobody claimed become holes
// (SRTP_PKT_FLAG_SKIP, no callback), at most 15 per producer per bundle.
// Callbacks run on the lanes' dispatch threads.  A callback may submit (an SFU
// forwarding what it just received); such a submit never waits for a slot --
// only the dispatch threads free slots, so waiting could deadlock.  When no
// slot is free it parks a copy of the packet in the lane's overflow queue,
// which the lane's thread moves into the first slot it frees, ahead of other
// producers, so a forwarded packet is never refused.  flush and destroy from
// a callback return SRTP_EINVAL.
//
// Per-packet semantics: each submitted packet is its own 1-element
// RawPacket[] in the reference, so one packet's exception must not stop
// later packets of the same transformer in the bundle.  The lanes therefore
// submit their bundles without abort-on-throw (srtp_pipeline_submit_ex with
// abort_on_error = 0), whatever the engines' option -- so the same engines
// (contexts) also serve srtp_rawpacket_transform's RawPacket[] calls, which
// keep it; a packet the reference would throw on completes with
// SRTP_STATUS_ERR_MALFORMED.
//
// Adaptive sealing (SRTP_AGG_SEAL_IDLE).  A lane with no bundle in flight
// seals its open bundle as soon as a packet lands in it; while a bundle is in
// flight the next one fills, and is sealed when the one in flight completes.
// So a lone packet waits one GPU round trip, not the deadline, and under load
// bundles grow to what arrives during a round trip -- the group commit of a
// database log.  Pipelined (round 5): with one bundle in flight, the lane
// thread does not block on it at once; half an average round trip after its
// submit it seals what has arrived meanwhile and submits that too, so two
// bundles are in flight and one's copies run beside the other's kernels (a
// lone bundle's GPU round trip is mostly copies and latency-bound kernels; the
// GPU idled a third of the time between bundles).  The lane thread and the producers meet through `idle`:
// the lane stores idle = 1 and then looks at its open slot, a producer
// reserves its entry and then looks at idle, both sequentially consistent,
// so at least one of them sees the other and seals.
//
// Synchronous calls (srtp_aggregator_transform) do not reserve entries: a
// caller pushes its request (packet pointer, lengths, where the result goes)
// on its lane's lock-free stack and sleeps on a futex.  The lane thread pops
// the stack, copies the requests' packets into a free slot itself and submits
// it -- so a caller preempted between reserving and filling an entry can never
// hold a bundle back (64 callers on 16 cores made that the common case) -- and
// when the bundle completes it copies each result back and wakes its caller.
// While the lane has a bundle in flight the requests pile up on the stack and
// go out together when it returns: bundles grow with the number of callers.
// Before it places them the lane seals its open bundle of that direction, so a
// thread's earlier submits run before its later synchronous call.
//
// Completion queues (srtp_queue_*): the asynchronous form of the per-packet
// call for a thread that keeps many packets in flight (a connector's send
// thread draining its queue, a receive loop).  A queue submit reserves and
// fills an entry exactly like srtp_aggregator_submit, but the entry carries a
// pointer to the queue's ring entry instead of a callback cookie.  When the
// bundle completes, the lane thread only publishes each such entry's status,
// length and a pointer to its bytes in the pinned slot (a few stores, no copy
// and no upcall) and wakes the queue's owner if it sleeps; the owner reaps the
// entries in submission order and copies the bytes out itself.  The slot stays
// held (kHeld) until every reaped entry of it has been released (by
// srtp_queue_release or the owner's next reap), so a completed packet's bytes
// never move.  A submit that finds no free slot waits for one only until its
// queue's oldest packet completes, then returns SRTP_EAGAIN (the owner reaps,
// which releases slots) -- after at most kHeldWait once its oldest packet has
// completed, so a thread never waits long on slots that only it can free.
#include <algorithm>
#include <atomic>
#include <climits>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <stdio.h>
#include <string.h>
#include <string>
#include <thread>
#include <vector>

#include <linux/futex.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include "../../include/srtp_mi355x.h"

namespace {
using Clock = std::chrono::steady_clock;

enum SlotState { kFree, kOpen, kSealed, kInflight, kHeld };
constexpr uint32_t kNoLen = 0xffffffffu; // h.len[i] until packet i's copy has finished
constexpr uint32_t kBlock = 16;          // entries per producer block (a cache line of u32s)
// how long a queue's submit keeps waiting for a slot after its own oldest
// packet has completed (see submit_entry)
constexpr std::chrono::microseconds kHeldWait{500};

// Reservation word of a lane direction's open slot: slot + 1 (0 = none) in
// bits 56-63, blocks handed out in bits 32-55, segment bytes in bits 0-31.
constexpr uint64_t resv_pack(uint32_t slot1, uint32_t n, uint32_t bytes) {
    return ((uint64_t)slot1 << 56) | ((uint64_t)n << 32) | bytes;
}
constexpr uint32_t resv_slot1(uint64_t r) { return (uint32_t)(r >> 56); }
constexpr uint32_t resv_n(uint64_t r) { return (uint32_t)(r >> 32) & 0xffffffu; }
constexpr uint32_t resv_bytes(uint64_t r) { return (uint32_t)r; }

// Claim word of a block: entries claimed in bits 0-7, bytes used in bits
// 8-39, the slot's generation (mod 2^23) in bits 40-62, closed (sealed) in bit
// 63.  The generation keeps a thread that cached a block from claiming in a
// later opening of the same slot.
constexpr uint64_t kClosed = 1ull << 63;
constexpr uint32_t blk_used(uint64_t w) { return (uint32_t)(w & 0xffu); }
constexpr uint32_t blk_bytes(uint64_t w) { return (uint32_t)(w >> 8); }
constexpr uint64_t blk_tag(uint32_t gen) { return (uint64_t)(gen & 0x7fffffu) << 40; }
constexpr uint64_t kTagMask = 0x7fffffull << 40;

// A synchronous caller waiting for its packet (srtp_aggregator_transform).
struct Waiter {
    std::atomic<uint32_t> done{0};
    int32_t status = 0;
    uint32_t len = 0;
    uint8_t *out = nullptr;
};

// Its request, on the caller's stack until it is woken.
struct SyncReq {
    SyncReq *next = nullptr;
    const uint8_t *pkt = nullptr;
    uint32_t copy_len = 0, len = 0, cap = 0, flags = 0;
    int32_t tid = -1, reverse = 0;
    Waiter w;
};

struct Slot;
struct Lane;

// A queue's ring entry (srtp_queue_submit .. srtp_queue_reap).
struct QEntry {
    std::atomic<uint32_t> ready{0}; // published by the lane thread (release)
    srtp_completion c{};            // cookie / in_len / avail / reverse / tid at submit, the rest at completion
    srtp_queue *q = nullptr;
    Slot *slot = nullptr;           // held until released (nullptr: completed at submit)
    Lane *lane = nullptr;
};

void futex_wait(std::atomic<uint32_t> *w, uint32_t v) {
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
void futex_wake(std::atomic<uint32_t> *w) {
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr, 0);
}

struct alignas(64) Block {
    std::atomic<uint64_t> w{0};
    uint32_t b0 = 0, size = 0; // byte range (written by the block's owner)
};

struct Slot {
    SlotState state = kFree;                 // under the aggregator's lock
    int idx = 0;
    std::atomic<uint32_t> holds{0};          // kHeld: reaped-or-not queue entries + the lane's own
    std::atomic<uint32_t> gen{0};            // opened how often (producers' cached blocks)
    int32_t reverse = 0;
    uint32_t n = 0;                          // entries (with holes), final once sealed
    uint32_t n_real = 0;                     // packets, final once sealed
    size_t bytes = 0;                        // segment bytes, final once sealed
    uint32_t ready = 0;                      // h.len[0 .. ready) seen stored (lane thread)
    Clock::time_point first;
    std::unique_ptr<Block[]> blocks;
    std::vector<uint8_t> hole;
    std::vector<uint64_t> cookies;
    std::vector<Waiter *> waiters;           // non-null: a synchronous caller's entry
    std::vector<QEntry *> qents;             // non-null: a completion queue's entry
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
    uint32_t idx = 0;
    srtp_engine *e = nullptr;
    srtp_pipeline *pl = nullptr;
    std::unique_ptr<Slot[]> slots;
    int n_slots = 0;
    std::atomic<uint64_t> resv[2] = {{0}, {0}}; // open slot per direction
    std::deque<int> sealed, inflight;
    std::deque<Parked> parked;
    std::condition_variable cv_work;  // the lane's dispatch thread: something to do
    std::condition_variable cv_space; // producers: a slot of this lane became free
    std::atomic<int> idle{1};         // SRTP_AGG_SEAL_IDLE: nothing sealed or in flight
    std::atomic<SyncReq *> sync_head{nullptr}; // synchronous requests, newest first
    std::deque<SyncReq *> sync_pending;        // popped, not yet placed (lane thread, in order)
    std::atomic<int> sleeping{0};              // the lane thread waits on cv_work
    std::thread thread;
};

thread_local const void *tl_in_callback = nullptr; // the aggregator whose callback runs here

// The block a thread is filling, per (aggregator, lane, direction).
struct TlBlock {
    uint64_t a = 0; // srtp_aggregator::id (0: unused)
    uint32_t lane = 0, dir = 0, slot = 0, gen = 0, blk = 0;
};
constexpr int kTlBlocks = 8;
thread_local TlBlock tl_blocks[kTlBlocks];
thread_local unsigned tl_victim = 0;
std::atomic<uint64_t> g_next_id{1};
} // namespace

// Fork-join helpers for a completed bundle's synchronous callers: each one's
// result copy and its futex wake-up.  A lane thread that copied and woke 169
// sleeping callers one after the other spent ~2.4 us per packet -- a syscall
// and a reschedule each -- and that, not the GPU, set the bundle rate of 256
// and more callers (profiles/r06/sync/).  run(parts, f) calls f(0..parts-1),
// the caller taking parts itself.
class WakePool {
  public:
    explicit WakePool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this] { loop(); });
    }
    ~WakePool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    template <class F> void run(int parts, const F &f) {
        if (parts <= 1 || th_.empty()) {
            for (int i = 0; i < parts; i++) f(i);
            return;
        }
        struct Job {
            std::atomic<int> next{0}, done{0};
        };
        auto job = std::make_shared<Job>();
        std::function<void()> body = [job, parts, &f] {
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

struct srtp_aggregator {
    srtp_dispatch *d = nullptr; // dispatch mode: lane = shard
    srtp_aggregator_opts opts{};
    srtp_aggregator_cb cb = nullptr;
    void *user = nullptr;
    uint64_t id = g_next_id.fetch_add(1); // keys the threads' cached blocks (never reused)
    uint32_t blk = kBlock;      // entries per block (max_packets if smaller)
    uint32_t n_blk = 0;         // blocks per slot
    uint32_t blk_bytes = 0;     // default byte range of a block

    std::mutex mu;
    std::condition_variable cv_flush; // the flusher: a new deadline
    std::condition_variable cv_idle;  // flush(): everything completed
    std::vector<std::unique_ptr<Lane>> lanes;
    std::atomic<bool> closing{false}; // destroy has begun: submits are refused
    std::atomic<int> sync_callers{0}; // srtp_aggregator_transform calls inside (destroy waits)
    std::atomic<int> queues{0};       // live srtp_queue objects (destroy waits)
    bool stop = false;
    // transformer kinds, read without a lock (-2: not looked up yet)
    std::unique_ptr<std::atomic<int32_t>[]> kinds;
    uint32_t n_kinds = 0;
    uint64_t completed = 0, bundles = 0;
    int error = SRTP_OK;
    std::string last_error;
    std::thread flusher;
    std::unique_ptr<WakePool> wakers; // helpers for the synchronous callers' wake-ups (may be empty)
};

// A completion queue: one owner thread (or externally serialised callers).
struct srtp_queue {
    srtp_aggregator *a = nullptr;
    uint32_t cap = 0;                  // ring entries: packets submitted and not yet reaped
    std::unique_ptr<QEntry[]> ring;
    uint64_t head = 0, tail = 0;       // next to reap, next to submit
    uint64_t rel_from = 0, rel_to = 0; // the last reap's entries, released at the next
    std::atomic<uint32_t> wake{0};     // futex word: bumped by a lane that saw `waiting`
    std::atomic<uint32_t> waiting{0};  // the owner sleeps (or is about to) in srtp_queue_reap
    std::atomic<uint32_t> lane_refs{0}; // lane threads between publishing entries and their wake-up
};

namespace {

// Seals direction dir's open slot of the lane: no more blocks, every block
// closed, unclaimed entries become holes.  A slot without packets goes back
// to the free list.
void seal_locked(srtp_aggregator *a, Lane &ln, int dir) {
    const uint64_t r = ln.resv[dir].exchange(0);
    if (!resv_slot1(r)) return;
    Slot &sl = ln.slots[resv_slot1(r) - 1];
    const uint32_t nb = resv_n(r);
    uint32_t real = 0;
    for (uint32_t k = 0; k < nb; k++) {
        const uint32_t u = blk_used(sl.blocks[k].w.fetch_or(kClosed));
        real += u;
        for (uint32_t i = k * a->blk + u; i < (k + 1) * a->blk; i++) {
            sl.hole[i] = 1;
            sl.h.off[i] = 0;
            sl.h.cap[i] = 0;
            sl.h.flags[i] = SRTP_PKT_FLAG_SKIP;
            sl.h.tids[i] = -1;
            sl.h.len[i] = 0;
        }
    }
    sl.n = nb * a->blk;
    sl.n_real = real;
    sl.bytes = resv_bytes(r);
    if (real == 0) {
        for (uint32_t i = 0; i < sl.n; i++) {
            sl.h.len[i] = kNoLen;
            sl.hole[i] = 0;
        }
        sl.n = 0;
        sl.state = kFree;
        ln.cv_space.notify_all();
        return;
    }
    sl.state = kSealed;
    sl.ready = 0;
    ln.sealed.push_back(resv_slot1(r) - 1);
    ln.idle.store(0);
    ln.cv_work.notify_all();
}

// SRTP_AGG_SEAL_IDLE, the lane thread's side (see the file comment): with
// nothing sealed or in flight, mark the lane idle, then seal an open bundle
// that has packets (which clears idle again).
void seal_if_idle_locked(srtp_aggregator *a, Lane &ln) {
    if (!(a->opts.flags & SRTP_AGG_SEAL_IDLE) || !ln.sealed.empty() || !ln.inflight.empty()) return;
    ln.idle.store(1);
    for (int d = 0; d < 2; d++)
        if (resv_n(ln.resv[d].load()) > 0) seal_locked(a, ln, d);
}

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
    sl.n = sl.n_real = 0;
    sl.bytes = 0;
    sl.first = Clock::now();
    const uint32_t g = sl.gen.load() + 1u;
    for (uint32_t k = 0; k < a->n_blk; k++) sl.blocks[k].w.store(blk_tag(g), std::memory_order_relaxed);
    sl.gen.store(g, std::memory_order_release);
    ln.resv[dir].store(resv_pack((uint32_t)s + 1u, 0, 0));
    a->cv_flush.notify_all(); // the flusher learns the new deadline
}

// Fast path: an entry (index, offset) in the calling thread's block of the
// open slot of direction dir, taking a new block when it has none or its
// block is full or closed.  False when the slot has no room (or none is open).
bool try_reserve(srtp_aggregator *a, Lane &ln, uint32_t lane, int dir, size_t need, int &s, uint32_t &i,
                 size_t &off) {
    TlBlock *tb = nullptr;
    for (auto &t : tl_blocks)
        if (t.a == a->id && t.lane == lane && t.dir == (uint32_t)dir) tb = &t;
    if (tb) {
        Slot &sl = ln.slots[tb->slot];
        Block &bk = sl.blocks[tb->blk];
        uint64_t w = bk.w.load(std::memory_order_acquire);
        if ((w & kTagMask) == blk_tag(tb->gen)) {
            // (b0 and size are this thread's own writes when the tag matches)
            while (!(w & kClosed) && blk_used(w) < a->blk && blk_bytes(w) + need <= bk.size) {
                const uint64_t nw = blk_tag(tb->gen) | ((uint64_t)(blk_bytes(w) + need) << 8) | (blk_used(w) + 1u);
                if (bk.w.compare_exchange_weak(w, nw, std::memory_order_acq_rel)) {
                    s = (int)tb->slot;
                    i = tb->blk * a->blk + blk_used(w);
                    off = bk.b0 + blk_bytes(w);
                    return true;
                }
            }
        }
    } else {
        tb = &tl_blocks[tl_victim++ % kTlBlocks];
        tb->a = a->id;
        tb->lane = lane;
        tb->dir = (uint32_t)dir;
    }
    // a new block
    uint64_t r = ln.resv[dir].load();
    for (;;) {
        const uint32_t s1 = resv_slot1(r);
        const size_t size = need > a->blk_bytes ? need : a->blk_bytes;
        if (!s1 || resv_n(r) >= a->n_blk || resv_bytes(r) + size > a->opts.max_bytes) {
            tb->a = 0;
            return false;
        }
        Slot &sl = ln.slots[s1 - 1];
        const uint32_t g = sl.gen.load(std::memory_order_acquire); // before the CAS (see below)
        const uint64_t nr = resv_pack(s1, resv_n(r) + 1u, resv_bytes(r) + (uint32_t)size);
        if (!ln.resv[dir].compare_exchange_weak(r, nr)) continue;
        const uint32_t k = resv_n(r);
        Block &bk = sl.blocks[k];
        // The first entry -- unless the slot was sealed meanwhile (closed), or
        // sealed and reopened between reading g and the CAS (tag of a later
        // generation: the block is then a run of holes in that opening).
        uint64_t w = blk_tag(g);
        if (!bk.w.compare_exchange_strong(w, blk_tag(g) | ((uint64_t)need << 8) | 1u, std::memory_order_acq_rel)) {
            r = ln.resv[dir].load();
            continue;
        }
        bk.b0 = resv_bytes(r);
        bk.size = (uint32_t)size;
        tb->slot = s1 - 1;
        tb->gen = g;
        tb->blk = k;
        s = (int)(s1 - 1);
        i = k * a->blk;
        off = bk.b0;
        return true;
    }
}

// Copies the packet into its reserved place; its length, stored last, marks
// it complete for the lane's thread.
void fill(Lane &ln, int s, uint32_t i, size_t off, int32_t tid, const uint8_t *pkt, uint32_t len, uint32_t cap,
          size_t need, uint32_t flags, uint64_t cookie, uint32_t copy_len) {
    Slot &sl = ln.slots[s];
    if (copy_len) memcpy(sl.h.seg + off, pkt, copy_len);
    if (need > copy_len) memset(sl.h.seg + off + copy_len, 0, need - copy_len);
    sl.h.off[i] = (uint32_t)off;
    sl.h.cap[i] = cap;
    sl.h.flags[i] = flags;
    sl.h.tids[i] = tid;
    sl.cookies[i] = cookie;
    __atomic_store_n(&sl.h.len[i], len, __ATOMIC_RELEASE);
}

// SRTP_AGG_SEAL_IDLE, the producer's side: after its entry is reserved (and
// filled), an idle lane's open bundle is sealed by the producer.
void producer_seal_if_idle(srtp_aggregator *a, Lane &ln, int dir) {
    if (!(a->opts.flags & SRTP_AGG_SEAL_IDLE) || !ln.idle.load()) return;
    std::lock_guard<std::mutex> lk(a->mu);
    if (ln.idle.load() && ln.sealed.empty() && ln.inflight.empty()) seal_locked(a, ln, dir);
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
            if (ln->slots[s].state == kSealed || ln->slots[s].state == kInflight) n += ln->slots[s].n_real;
        for (int d = 0; d < 2; d++) {
            const uint64_t r = ln->resv[d].load();
            if (!resv_slot1(r)) continue;
            const Slot &sl = ln->slots[resv_slot1(r) - 1];
            for (uint32_t k = 0; k < resv_n(r); k++) n += blk_used(sl.blocks[k].w.load());
        }
        n += ln->parked.size() + ln->sync_pending.size() + (ln->sync_head.load() ? 1 : 0);
    }
    return n;
}

size_t need_of(uint32_t cap) { return ((size_t)cap + 15u) & ~(size_t)15u; }

// Places parked callback packets into slots (the lane's thread, after it
// freed one); stops when no slot is left.
void place_parked_locked(srtp_aggregator *a, Lane &ln, uint32_t lane) {
    while (!ln.parked.empty()) {
        Parked &pk = ln.parked.front();
        const int dir = pk.reverse ? 1 : 0;
        const uint32_t len = (uint32_t)pk.pkt.size();
        const uint32_t cap = pk.reverse ? len : len + 16u;
        const size_t need = need_of(cap);
        int s;
        uint32_t i;
        size_t off;
        if (!try_reserve(a, ln, lane, dir, need, s, i, off)) {
            seal_locked(a, ln, dir);
            const int f = free_slot_locked(ln, true);
            if (f < 0) return;
            open_locked(a, ln, dir, f);
            if (!try_reserve(a, ln, lane, dir, need, s, i, off)) return; // cannot happen: need <= max_bytes
        }
        ln.slots[s].waiters[i] = nullptr;
        ln.slots[s].qents[i] = nullptr;
        fill(ln, s, i, off, pk.tid, pk.pkt.data(), len, cap, need, pk.flags, pk.cookie, len);
        ln.parked.pop_front();
    }
}

// A completed slot none of whose queue entries is still held goes back to the
// free list (under the lock): parked callback packets are placed first, then
// an idle lane's open bundle is sealed.
void slot_free_locked(srtp_aggregator *a, Lane &ln, Slot &sl) {
    for (uint32_t i = 0; i < sl.n; i++) {
        sl.h.len[i] = kNoLen;
        sl.hole[i] = 0;
    }
    sl.state = kFree;
    sl.n = sl.n_real = 0;
    sl.bytes = 0;
    place_parked_locked(a, ln, ln.idx);
    seal_if_idle_locked(a, ln);
    ln.cv_space.notify_all();
    ln.cv_work.notify_all(); // synchronous requests may wait for a free slot
    a->cv_idle.notify_all();
}

#ifndef SRTP_AGG_SYNC_CAP
#define SRTP_AGG_SYNC_CAP 2
#endif
// Synchronous requests may be placed: some are waiting, a slot is free and
// fewer than SRTP_AGG_SYNC_CAP (two) bundles are sealed or in flight.
bool sync_placeable_locked(const Lane &ln) {
    if (!ln.sync_head.load() && ln.sync_pending.empty()) return false;
    if (ln.sealed.size() + ln.inflight.size() >= (size_t)SRTP_AGG_SYNC_CAP) return false;
    for (int i = 0; i < ln.n_slots; i++)
        if (ln.slots[i].state == kFree) return true;
    return false;
}

// Copies waiting synchronous requests of one direction (the oldest request's)
// into a free slot, in arrival order, and seals it.
void place_sync_locked(srtp_aggregator *a, Lane &ln) {
    SyncReq *h = ln.sync_head.exchange(nullptr);
    SyncReq *rev = nullptr; // the stack is newest first
    while (h) {
        SyncReq *nx = h->next;
        h->next = rev;
        rev = h;
        h = nx;
    }
    for (; rev; rev = rev->next) ln.sync_pending.push_back(rev);
    int s = -1;
    for (int i = 0; i < ln.n_slots && s < 0; i++)
        if (ln.slots[i].state == kFree) s = i;
    if (s < 0 || ln.sync_pending.empty()) return;
    Slot &sl = ln.slots[s];
    const int32_t dir = ln.sync_pending.front()->reverse;
    // packets a caller submitted before its synchronous call go first
    seal_locked(a, ln, dir);
    uint32_t n = 0;
    size_t pos = 0;
    for (auto it = ln.sync_pending.begin(); it != ln.sync_pending.end();) {
        SyncReq *r = *it;
        const size_t need = need_of(r->cap);
        if (r->reverse != dir) { ++it; continue; }
        if (n == a->opts.max_packets || pos + need > a->opts.max_bytes) break;
        if (r->copy_len) memcpy(sl.h.seg + pos, r->pkt, r->copy_len);
        if (need > r->copy_len) memset(sl.h.seg + pos + r->copy_len, 0, need - r->copy_len);
        sl.h.off[n] = (uint32_t)pos;
        sl.h.len[n] = r->len;
        sl.h.cap[n] = r->cap;
        sl.h.flags[n] = r->flags;
        sl.h.tids[n] = r->tid;
        sl.cookies[n] = r->len; // the submitted length (see the completion loop)
        sl.waiters[n] = &r->w;
        sl.qents[n] = nullptr;
        sl.hole[n] = 0;
        pos += need;
        n++;
        it = ln.sync_pending.erase(it);
    }
    sl.state = kSealed;
    sl.reverse = dir;
    sl.n = sl.n_real = n;
    sl.bytes = pos;
    sl.ready = n; // every entry is complete
    ln.sealed.push_back(s);
    ln.idle.store(0);
}

// The lane thread polls its bundle in flight (hipEventQuery) between waits on
// its condition variable, every kPollUs; with Linux's default 50-us timer
// slack each such wait would oversleep by up to 50 us -- most of a lone
// call's host time -- so lane threads run with 1 us of slack.
#ifndef SRTP_AGG_POLL_US
#define SRTP_AGG_POLL_US 5
#endif
constexpr long kPollUs = SRTP_AGG_POLL_US;

#ifndef SRTP_AGG_PIPE
#define SRTP_AGG_PIPE 2
#endif
constexpr size_t kPipe = SRTP_AGG_PIPE; // bundles a lane keeps in flight under load (SRTP_AGG_SEAL_IDLE)

#ifdef SRTP_AGG_TRACE
// diagnostic builds only (tools/build_agg_variant.sh NAME -DSRTP_AGG_TRACE):
// the lane's submits, timed seals, waits and completions with their times,
// printed to stderr when the lane ends (profiles/r06/small/queue64_lane_trace.txt)
struct TraceEv { char k; int slot; uint32_t n; int dir; double us; size_t sealed, inflight; };
#define AGG_TRACE(vec, k, s, n, d)                                                                         \
    vec.push_back(TraceEv{k, s, n, d, std::chrono::duration<double, std::micro>(Clock::now().time_since_epoch()).count(), \
                          ln->sealed.size(), ln->inflight.size()})
#else
#define AGG_TRACE(vec, k, s, n, d) do {} while (0)
#endif

void lane_loop(srtp_aggregator *a, Lane *ln, uint32_t lane) {
    (void)lane;
#ifdef SRTP_AGG_TRACE
    std::vector<TraceEv> trace;
    trace.reserve(1 << 16);
    struct Dump {
        std::vector<TraceEv> &t;
        ~Dump() {
            for (size_t i = 0; i < t.size() && i < 4000; i++)
                fprintf(stderr, "AGGTRACE %c slot %d n %u dir %d t %.1f sealed %zu inflight %zu\n", t[i].k, t[i].slot,
                        t[i].n, t[i].dir, t[i].us, t[i].sealed, t[i].inflight);
        }
    } dump{trace};
#endif
    prctl(PR_SET_TIMERSLACK, 1000UL); // ns (see kPollUs)
    std::vector<srtp_queue *> touched; // queues with entries in the completed bundle
    std::vector<uint32_t> waiters;     // its synchronous callers' entries
    std::unique_lock<std::mutex> lk(a->mu);
    // keep up to depth - 2 bundles in flight (one slot per open direction)
    const size_t max_inflight = ln->n_slots > 2 ? (size_t)ln->n_slots - 2 : 1;
    // submit time per slot and the average round trip (EWMA, us)
    std::vector<Clock::time_point> t_sub((size_t)ln->n_slots);
    double rt_us = 200.0;
    for (;;) {
        bool straggler = false; // a sealed slot still being copied into
        auto can_submit = [&] {
            straggler = false;
            if (ln->sealed.empty() || ln->inflight.size() >= max_inflight) return false;
            straggler = !slot_ready(ln->slots[ln->sealed.front()]);
            return !straggler;
        };
        auto go = [&] {
            return a->stop || sync_placeable_locked(*ln) || can_submit() || !ln->inflight.empty();
        };
        // sleeping is raised before the last look (a synchronous caller pushes,
        // then looks at it: one of the two sees the other)
        for (;;) {
            ln->sleeping.store(1);
            if (go()) break;
            if (straggler) ln->cv_work.wait_for(lk, std::chrono::microseconds(20)); // copies take ~0.1 us
            else ln->cv_work.wait(lk);
        }
        ln->sleeping.store(0);
        if (a->stop && ln->sealed.empty() && ln->inflight.empty() && ln->parked.empty() &&
            !ln->sync_head.load() && ln->sync_pending.empty())
            return;
        if (sync_placeable_locked(*ln)) place_sync_locked(a, *ln);
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
            t_sub[(size_t)s] = Clock::now();
            AGG_TRACE(trace, 'S', s, n, rev);
            const int rc = srtp_pipeline_submit_ex(ln->pl, s, rev, 1, -1, 1, n, bytes, 0);
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
        // Pipelining (file comment): one bundle in flight, room for another
        // and a free slot -- wait for it only until half a round trip after
        // its submit, then seal what has arrived and go submit that as well.
        if (kPipe > 1 && (a->opts.flags & SRTP_AGG_SEAL_IDLE) && ln->inflight.size() + ln->sealed.size() < kPipe &&
            ln->inflight.size() < max_inflight && !a->stop) {
            const auto t_seal = t_sub[(size_t)s] + std::chrono::microseconds((long)(rt_us / 2));
            bool done = false, sealed_more = false;
            for (;;) {
                lk.unlock();
                done = srtp_pipeline_query(ln->pl, s) != 0;
                lk.lock();
                if (done || a->stop || !ln->sealed.empty()) break;
                if (Clock::now() >= t_seal) {
                    for (int d = 0; d < 2; d++)
                        if (resv_n(ln->resv[d].load()) > 0) {
                            seal_locked(a, *ln, d);
                            sealed_more = true;
                            AGG_TRACE(trace, 'T', -1, 0u, d);
                        }
                    if (sealed_more || sync_placeable_locked(*ln)) break;
                }
                const auto now = Clock::now();
                ln->cv_work.wait_for(lk, now < t_seal ? std::min<Clock::duration>(t_seal - now, std::chrono::microseconds(kPollUs))
                                                       : Clock::duration(std::chrono::microseconds(kPollUs)));
            }
            if (!done) continue; // submit what was sealed (or placed), then come back
        }
        lk.unlock();
        AGG_TRACE(trace, 'W', s, sl.n, sl.reverse);
        (void)srtp_pipeline_wait(ln->pl, s);
        AGG_TRACE(trace, 'D', s, sl.n, sl.reverse);
        {
            const double us = std::chrono::duration<double, std::micro>(Clock::now() - t_sub[(size_t)s]).count();
            rt_us = 0.875 * rt_us + 0.125 * us;
        }
        // queue entries hold the slot until their owners release them; the
        // lane holds it too until this loop is done
        uint32_t nq = 0;
        for (uint32_t i = 0; i < sl.n; i++) nq += !sl.hole[i] && sl.qents[i];
        if (nq) sl.holds.store(nq + 1u, std::memory_order_relaxed);
        touched.clear();
        // callbacks outside the lock, in bundle order; synchronous callers get
        // their packet's bytes (as much as it occupied before or after, within
        // its room) and wake; queue entries get their results published
        tl_in_callback = a;
        for (uint32_t i = 0; i < sl.n; i++) {
            if (sl.hole[i]) continue;
            const int32_t st = sl.h.status[i];
            if (QEntry *qe = sl.qents[i]) {
                sl.qents[i] = nullptr;
                qe->c.status = st;
                qe->c.len = sl.h.len[i];
                qe->c.data = sl.h.seg + sl.h.off[i];
                qe->slot = &sl;
                qe->lane = ln;
                srtp_queue *q = qe->q;
                if (std::find(touched.begin(), touched.end(), q) == touched.end()) {
                    q->lane_refs.fetch_add(1, std::memory_order_relaxed); // ordered by the release below
                    touched.push_back(q);
                }
                qe->ready.store(1, std::memory_order_release);
                continue;
            }
            if (sl.waiters[i]) { // synchronous callers: below, over the wake helpers
                waiters.push_back(i);
                continue;
            }
            if (a->cb) a->cb(a->user, sl.cookies[i], st, sl.h.seg + sl.h.off[i], sl.h.len[i]);
        }
        tl_in_callback = nullptr;
        if (!waiters.empty()) {
            // each caller's result and wake-up; callers are independent, so the
            // order does not matter: split over the helpers in runs of 16
            const int nw = (int)waiters.size();
            const int parts = a->wakers ? std::min(a->wakers->size() + 1, (nw + 15) / 16) : 1;
            auto part = [&](int q) {
                for (int k = nw * q / parts; k < nw * (q + 1) / parts; k++) {
                    const uint32_t i = waiters[(size_t)k];
                    Waiter *w = sl.waiters[i];
                    sl.waiters[i] = nullptr;
                    const uint32_t nl = sl.h.len[i];
                    const uint32_t ol = (uint32_t)(uintptr_t)sl.cookies[i]; // the length submitted
                    memcpy(w->out, sl.h.seg + sl.h.off[i], std::min(std::max(nl, ol), sl.h.cap[i]));
                    w->status = sl.h.status[i];
                    w->len = nl;
                    w->done.store(1, std::memory_order_release);
                    futex_wake(&w->done);
                }
            };
            if (parts > 1) a->wakers->run(parts, part);
            else part(0);
            waiters.clear();
        }
        if (!touched.empty()) {
            // ready (release) before waiting (seq_cst), against the owner's
            // waiting before ready: one of the two sees the other
            std::atomic_thread_fence(std::memory_order_seq_cst);
            for (srtp_queue *q : touched) {
                if (q->waiting.load()) {
                    q->wake.fetch_add(1);
                    futex_wake(&q->wake);
                }
                q->lane_refs.fetch_sub(1, std::memory_order_release); // destroy may free q now
            }
        }
        lk.lock();
        ln->inflight.pop_front();
        a->completed += sl.n_real;
        a->bundles++;
        if (nq == 0 || sl.holds.fetch_sub(1) == 1) {
            slot_free_locked(a, *ln, sl);
        } else {
            sl.state = kHeld; // freed by the last release (queue_release)
            seal_if_idle_locked(a, *ln);
            ln->cv_space.notify_all(); // queue submitters waiting for a slot look at their entries
            a->cv_idle.notify_all();
        }
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
    if (!out || n_lanes == 0) return SRTP_EINVAL; // cb NULL: only synchronous calls (srtp_aggregator_transform)
    *out = nullptr;
    srtp_aggregator_opts o;
    if (opts) o = *opts;
    else srtp_aggregator_opts_default(&o);
    // the reservation word holds 24 bits of packets and 32 of bytes
    if (o.max_packets == 0 || o.max_packets > 0xffffffu || o.max_bytes < 64 ||
        o.max_bytes > 0xffffffffull || o.depth < 3 || o.depth > 16 || (o.flags & ~(uint32_t)SRTP_AGG_SEAL_IDLE))
        return SRTP_EINVAL;
    srtp_engine_opts eo{};
    for (size_t l = 0; l < n_lanes; l++)
        if (!engines[l] || srtp_engine_get_opts(engines[l], &eo) != SRTP_OK) return SRTP_EINVAL;
    srtp_aggregator *a = new (std::nothrow) srtp_aggregator();
    if (!a) return SRTP_ENOMEM;
    a->d = d;
    a->opts = o;
    a->cb = cb;
    a->user = user;
    a->blk = o.max_packets < kBlock ? o.max_packets : kBlock;
    a->n_blk = o.max_packets / a->blk;
    a->blk_bytes = (uint32_t)std::max<size_t>(64, (o.max_bytes / a->n_blk) & ~(size_t)15);
    a->n_kinds = eo.max_transformers;
    a->kinds.reset(new (std::nothrow) std::atomic<int32_t>[a->n_kinds]);
    if (!a->kinds) {
        delete a;
        return SRTP_ENOMEM;
    }
    for (uint32_t t = 0; t < a->n_kinds; t++) a->kinds[t].store(-2, std::memory_order_relaxed);
    // lanes whose engines share a GPU keep each bundle on one stream (see
    // SRTP_PIPE_ONE_STREAM): spread over the device's few hardware queues, the
    // copy streams made every lane wait behind the others' copy events.  A lane
    // alone on its GPU keeps them for large bundles (two in flight overlap);
    // the pipeline puts small ones on the engine's stream by itself.
    std::vector<int32_t> dev(n_lanes, -1);
    for (size_t l = 0; l < n_lanes; l++) {
        srtp_engine_opts lo;
        if (srtp_engine_get_opts(engines[l], &lo) == SRTP_OK) dev[l] = lo.device;
    }
    for (size_t l = 0; l < n_lanes; l++) {
        a->lanes.emplace_back(new Lane());
        Lane &ln = *a->lanes.back();
        ln.idx = (uint32_t)l;
        ln.e = engines[l];
        const bool shared = std::count(dev.begin(), dev.end(), dev[l]) > 1;
        const int rc = srtp_pipeline_create_ex(ln.e, o.max_packets, o.max_bytes, o.depth,
                                               shared ? SRTP_PIPE_ONE_STREAM : 0u, &ln.pl);
        if (rc != SRTP_OK) {
            destroy_lanes(a);
            delete a;
            return rc;
        }
        ln.n_slots = o.depth;
        ln.slots.reset(new Slot[(size_t)o.depth]);
        for (int i = 0; i < o.depth; i++) {
            Slot &sl = ln.slots[i];
            sl.idx = i;
            srtp_pipeline_slot_get(ln.pl, i, &sl.h);
            sl.cookies.resize(o.max_packets);
            sl.waiters.assign(o.max_packets, nullptr);
            sl.qents.assign(o.max_packets, nullptr);
            sl.hole.assign(o.max_packets, 0);
            sl.blocks.reset(new Block[a->n_blk]);
            for (uint32_t k = 0; k < o.max_packets; k++) sl.h.len[k] = kNoLen;
        }
    }
    for (size_t l = 0; l < a->lanes.size(); l++) a->lanes[l]->thread = std::thread(lane_loop, a, a->lanes[l].get(), (uint32_t)l);
    {   // wake helpers: a quarter of the CPUs this process may run on, at most 4
        cpu_set_t cs;
        int ncpu = 4;
        if (sched_getaffinity(0, sizeof cs, &cs) == 0) ncpu = CPU_COUNT(&cs);
        const int nh = std::min(4, ncpu / 4);
        if (nh > 0) a->wakers.reset(new (std::nothrow) WakePool(nh));
    }
    a->flusher = std::thread(flush_loop, a);
    *out = a;
    return SRTP_OK;
}

// A packet into its lane's open bundle (srtp_aggregator_submit / _transform):
// copy_len bytes of pkt, length len, room cap; w != nullptr: a synchronous
// caller's entry.
// qe: a completion queue's entry; its queue's oldest outstanding entry
// (q_head, or nullptr when the queue has none) bounds a wait for a slot: the
// submit returns SRTP_EAGAIN once that entry has completed (the caller then
// reaps, which frees slots), so a thread never waits on slots that only its
// own reaping can free.
int submit_entry(srtp_aggregator *a, int32_t reverse, int32_t tid, const uint8_t *pkt, uint32_t copy_len,
                 uint32_t len, uint32_t cap, uint32_t flags, uint64_t cookie, Waiter *w, QEntry *qe = nullptr,
                 const QEntry *q_head = nullptr) {
    if (a->closing.load()) return SRTP_EINVAL; // destroy has begun
    const int dir = reverse ? 1 : 0;
    const size_t need = need_of(cap);
    if (need > a->opts.max_bytes) return SRTP_EINVAL;
    size_t lane = 0;
    if (a->d) {
        const int32_t sh = srtp_dispatch_route(a->d, tid, pkt, copy_len < len ? copy_len : len);
        lane = sh < 0 ? 0 : (size_t)sh; // an unknown transformer: the engine reports it SKIPPED
    }
    Lane &ln = *a->lanes[lane];
    const bool in_cb = tl_in_callback == a;
    int s;
    uint32_t i;
    size_t off;
    if (!try_reserve(a, ln, (uint32_t)lane, dir, need, s, i, off)) {
        Clock::time_point held_since{};
        std::unique_lock<std::mutex> lk(a->mu);
        for (;;) {
            if (a->stop || a->closing.load()) return SRTP_EINVAL;
            if (try_reserve(a, ln, (uint32_t)lane, dir, need, s, i, off)) break;
            seal_locked(a, ln, dir); // full (or none open)
            const int f = free_slot_locked(ln, in_cb);
            if (f >= 0) {
                open_locked(a, ln, dir, f);
                continue;
            }
            if (in_cb) { // never wait for a slot from a callback: park the packet
                ln.parked.push_back(Parked{dir, tid, flags, cookie, std::vector<uint8_t>(pkt, pkt + len)});
                return SRTP_OK;
            }
            if (q_head) {
                // A queue's submit waits for a slot while its oldest packet is
                // in flight; once that one has completed, for at most
                // kHeldWait more (other owners' reaps free slots meanwhile),
                // then SRTP_EAGAIN: its owner reaps, releasing what it holds.
                if (q_head->ready.load(std::memory_order_acquire)) {
                    if (held_since == Clock::time_point{}) held_since = Clock::now();
                    else if (Clock::now() - held_since > kHeldWait) return SRTP_EAGAIN;
                }
                // (completions may come from another lane: poll)
                ln.cv_space.wait_for(lk, std::chrono::microseconds(100));
                continue;
            }
            ln.cv_space.wait(lk); // backpressure: every slot is sealed, in flight or held
        }
    }
    ln.slots[s].waiters[i] = w;
    ln.slots[s].qents[i] = qe;
    fill(ln, s, i, off, tid, pkt, len, cap, need, flags, cookie, copy_len);
    producer_seal_if_idle(a, ln, dir);
    return SRTP_OK;
}

// Releases the entries [from, to) of a queue's ring: each slot's holds drop by
// its entries' count, and the release that reaches zero frees the slot.
void queue_release(srtp_queue *q, uint64_t from, uint64_t to) {
    Slot *cur = nullptr;
    Lane *cur_lane = nullptr;
    uint32_t k = 0;
    auto drop = [&] {
        if (cur && cur->holds.fetch_sub(k) == k) {
            std::lock_guard<std::mutex> lk(q->a->mu);
            slot_free_locked(q->a, *cur_lane, *cur);
        }
    };
    for (uint64_t x = from; x < to; x++) {
        QEntry &e = q->ring[x % q->cap];
        if (!e.slot) continue;
        if (e.slot != cur) {
            drop();
            cur = e.slot;
            cur_lane = e.lane;
            k = 0;
        }
        k++;
        e.slot = nullptr;
    }
    drop();
}

// The owner waits for entry e of its queue: a short spin, then the futex.
void queue_wait(srtp_queue *q, QEntry &e) {
    for (int i = 0; i < 256; i++) {
        if (e.ready.load(std::memory_order_acquire)) return;
        __builtin_ia32_pause();
    }
    for (;;) {
        const uint32_t w0 = q->wake.load(std::memory_order_acquire);
        q->waiting.store(1);
        std::atomic_thread_fence(std::memory_order_seq_cst);
        if (e.ready.load(std::memory_order_acquire)) break;
        futex_wait(&q->wake, w0);
    }
    q->waiting.store(0, std::memory_order_relaxed);
}

} // namespace

extern "C" {

int srtp_aggregator_opts_default(srtp_aggregator_opts *o) {
    if (!o) return SRTP_EINVAL;
    o->max_packets = 1u << 14;
    o->max_bytes = (size_t)24 << 20;
    o->deadline_us = 1000;
    o->depth = 4;
    o->flags = SRTP_AGG_SEAL_IDLE;
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
    if (!a || !a->cb || (!pkt && len) || len > 65535u - 16u) return SRTP_EINVAL;
    // protect appends up to 16 bytes (SRTCP E|index + a 12-byte tag): the
    // in-place form of RawPacket.append / grow; unprotect only shrinks
    const uint32_t cap = reverse ? len : len + 16u;
    return submit_entry(a, reverse, tid, pkt, len, len, cap, flags, cookie, nullptr);
}

int srtp_aggregator_transform(srtp_aggregator *a, int32_t reverse, int32_t tid, const uint8_t *pkt,
                              uint32_t copy_len, uint32_t len, uint32_t cap, uint32_t flags,
                              uint8_t *out, int32_t *status, uint32_t *out_len) {
    if (!a || !out || !status || !out_len || (!pkt && copy_len) || copy_len > cap || len > 65535u ||
        cap > 65535u)
        return SRTP_EINVAL;
    if (tl_in_callback == a) return SRTP_EINVAL; // would wait for its own lane
    if (need_of(cap) > a->opts.max_bytes) return SRTP_EINVAL;
    if (len > cap) { // RawPacket.isInvalid: what k_parse reports, without a round trip
        *status = SRTP_STATUS_DROP_INVALID;
        *out_len = len;
        return SRTP_OK;
    }
    struct Inside { // counted before the closing check: destroy waits for every caller inside
        srtp_aggregator *a;
        ~Inside() { a->sync_callers.fetch_sub(1); }
    } inside{a};
    a->sync_callers.fetch_add(1);
    if (a->closing.load()) return SRTP_EINVAL;
    SyncReq r;
    r.pkt = pkt;
    r.copy_len = copy_len;
    r.len = len;
    r.cap = cap;
    r.flags = flags;
    r.tid = tid;
    r.reverse = reverse ? 1 : 0;
    r.w.out = out;
    size_t lane = 0;
    if (a->d) {
        const int32_t sh = srtp_dispatch_route(a->d, tid, pkt, copy_len < len ? copy_len : len);
        lane = sh < 0 ? 0 : (size_t)sh;
    }
    Lane &ln = *a->lanes[lane];
    r.next = ln.sync_head.load();
    while (!ln.sync_head.compare_exchange_weak(r.next, &r)) {
    }
    if (ln.sleeping.load()) {
        std::lock_guard<std::mutex> lk(a->mu);
        ln.cv_work.notify_all();
    }
    while (r.w.done.load(std::memory_order_acquire) == 0) futex_wait(&r.w.done, 0);
    *status = r.w.status;
    *out_len = r.w.len;
    return SRTP_OK;
}

int srtp_aggregator_transformer_info(srtp_aggregator *a, int32_t t, int32_t *kind, int32_t *fwd_rtcp_tag_len) {
    if (!a || t < 0 || (uint32_t)t >= a->n_kinds) return SRTP_EINVAL;
    srtp_engine *e = a->lanes[0]->e;
    int32_t k = a->kinds[(size_t)t].load(std::memory_order_acquire);
    if (k < 0 || fwd_rtcp_tag_len) {
        const int rc = srtp_transformer_info(e, t, &k, fwd_rtcp_tag_len);
        if (rc != SRTP_OK) return rc;
        a->kinds[(size_t)t].store(k, std::memory_order_release); // a transformer's kind never changes
    }
    if (kind) *kind = k;
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
        // refuse new submits (callbacks' forwards included), then drain every
        // accepted packet: a packet accepted is always delivered
        a->closing.store(true);
        seal_all_locked(a);
        for (;;) {
            // queues hold slots whose bytes their owners still read: every
            // queue must be destroyed first (see the header)
            if (pending_locked(a) == 0 && a->sync_callers.load() == 0 && a->queues.load() == 0) break;
            seal_all_locked(a); // parked callback packets placed since, stragglers' slots
            a->cv_idle.wait_for(lk, std::chrono::milliseconds(1));
        }
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

int srtp_queue_create(srtp_aggregator *a, uint32_t max_inflight, srtp_queue **out) {
    if (!a || !out || max_inflight == 0 || max_inflight > (1u << 20)) return SRTP_EINVAL;
    *out = nullptr;
    if (a->closing.load()) return SRTP_EINVAL;
    srtp_queue *q = new (std::nothrow) srtp_queue();
    if (!q) return SRTP_ENOMEM;
    q->ring.reset(new (std::nothrow) QEntry[max_inflight]);
    if (!q->ring) {
        delete q;
        return SRTP_ENOMEM;
    }
    q->a = a;
    q->cap = max_inflight;
    for (uint32_t i = 0; i < max_inflight; i++) q->ring[i].q = q;
    a->queues.fetch_add(1);
    *out = q;
    return SRTP_OK;
}

int srtp_queue_submit(srtp_queue *q, int32_t reverse, int32_t tid, const uint8_t *pkt, uint32_t copy_len,
                      uint32_t len, uint32_t cap, uint32_t flags, uint64_t cookie) {
    if (!q || (!pkt && copy_len) || copy_len > cap || cap > 65535u || len > 65535u) return SRTP_EINVAL;
    srtp_aggregator *a = q->a;
    if (tl_in_callback == a) return SRTP_EINVAL; // a lane's own thread must not wait on its lanes
    if (need_of(cap) > a->opts.max_bytes) return SRTP_EINVAL;
    if (q->tail - q->head >= q->cap) return SRTP_EAGAIN; // reap first
    QEntry &e = q->ring[q->tail % q->cap];
    e.slot = nullptr;
    e.lane = nullptr;
    e.c = srtp_completion{};
    e.c.cookie = cookie;
    e.c.in_len = len;
    e.c.len = len;
    e.c.reverse = reverse ? 1 : 0;
    e.c.tid = tid;
    if ((flags & SRTP_PKT_FLAG_SKIP) || len > cap) {
        // untouched, as the engine would report it: a null element or one the
        // predicate rejected (SKIPPED), RawPacket.isInvalid (DROP_INVALID)
        e.c.status = (flags & SRTP_PKT_FLAG_SKIP) ? SRTP_STATUS_SKIPPED : SRTP_STATUS_DROP_INVALID;
        e.ready.store(1, std::memory_order_relaxed);
        q->tail++;
        return SRTP_OK;
    }
    e.ready.store(0, std::memory_order_relaxed);
    // completions still held: the caller must release (reap) before it may
    // wait for a slot that they could be holding
    if (q->rel_from != q->rel_to) {
        std::lock_guard<std::mutex> lk(a->mu); // (cheap check first: any free slot at all?)
        bool any = false;
        for (auto &ln : a->lanes)
            for (int i = 0; i < ln->n_slots && !any; i++) any = ln->slots[i].state == kFree;
        if (!any) return SRTP_EAGAIN;
    }
    // a wait for a slot ends when the queue's oldest packet completes (file comment)
    const QEntry *q_head = q->tail > q->head ? &q->ring[q->head % q->cap] : nullptr;
    const int rc = submit_entry(a, reverse, tid, pkt, copy_len, len, cap,
                                flags & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE), cookie, nullptr, &e,
                                q_head);
    if (rc != SRTP_OK) return rc;
    q->tail++;
    return SRTP_OK;
}

int srtp_queue_reap(srtp_queue *q, srtp_completion *out, uint32_t max, int32_t wait) {
    if (!q || (!out && max) || max > (uint32_t)INT_MAX) return SRTP_EINVAL;
    queue_release(q, q->rel_from, q->rel_to);
    q->rel_from = q->rel_to = q->head;
    uint32_t n = 0;
    while (n < max && q->head < q->tail) {
        QEntry &e = q->ring[q->head % q->cap];
        if (!e.ready.load(std::memory_order_acquire)) {
            if (n > 0 || !wait) break;
            queue_wait(q, e);
        }
        out[n++] = e.c;
        q->head++;
    }
    q->rel_to = q->head;
    return (int)n;
}

void srtp_queue_release(srtp_queue *q) {
    if (!q) return;
    queue_release(q, q->rel_from, q->rel_to);
    q->rel_from = q->rel_to = q->head;
}

srtp_aggregator *srtp_queue_aggregator(srtp_queue *q) { return q ? q->a : nullptr; }

int32_t srtp_queue_outstanding(srtp_queue *q) { return q ? (int32_t)(q->tail - q->head) : 0; }

void srtp_queue_destroy(srtp_queue *q) {
    if (!q) return;
    // every submitted packet completes, then every slot it holds is released
    queue_release(q, q->rel_from, q->rel_to);
    while (q->head < q->tail) {
        QEntry &e = q->ring[q->head % q->cap];
        if (!e.ready.load(std::memory_order_acquire)) queue_wait(q, e);
        queue_release(q, q->head, q->head + 1);
        q->head++;
    }
    while (q->lane_refs.load(std::memory_order_acquire)) std::this_thread::yield();
    srtp_aggregator *a = q->a;
    delete q;
    std::lock_guard<std::mutex> lk(a->mu);
    a->queues.fetch_sub(1);
    a->cv_idle.notify_all();
}

} // extern "C"
