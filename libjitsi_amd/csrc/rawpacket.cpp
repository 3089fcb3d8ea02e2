// rawpacket.cpp -- RawPacket[] marshalling for the Java drop-in.
//
// What a JNI shim under PacketTransformer.transform / reverseTransform(RawPacket[])
// needs, in C: each element's buffer, offset, length and flags are packed
// into a bundle segment, the bundle runs on the engine (or the multi-GPU
// dispatcher), and the results are written back into the callers' buffers in
// place -- exactly where the reference's per-packet calls leave them:
//
//   * SinglePacketTransformer.java:121-216: array order; a null element (or one
//     the packet predicate rejects: SRTP_PKT_FLAG_SKIP) is not touched; a drop
//     is reported so the caller can null the element; a throw is reported with
//     the index of the first throwing element, after every packet was written
//     back -- the earlier packets transformed, the thrower keeping the
//     mutations made before its throw (e.g. authenticatePacket's shrink),
//     its transformer's later packets untouched (NOT_PROCESSED);
//   * RawPacket.append (RawPacket.java:203-220): SRTP protect appends the tag in
//     place when the buffer has room after the payload, else into a new buffer
//     of exactly length + tag at offset 0;
//   * RawPacket.grow (:885-893): SRTCP protect always moves to a new buffer of
//     length + 4 + tag at offset 0 (SRTCPCryptoContext.java:413);
//   * RawPacket.shrink (:1284-1292): unprotect shrinks in place, also for a
//     packet whose tag check fails.
//
// A new buffer cannot be allocated here (it is a Java byte[]): such an
// element gets need_len[i] = the new buffer's length, its result stays in
// the batch (srtp_rawpacket_result), and the shim allocates the array, copies
// the result to offset 0 and sets buffer / offset = 0 / length.  Everything
// else is written in place into the buffers the caller passed (the JNI
// shim's own copies of the Java arrays, written back with SetByteArrayRegion:
// no JNI critical region spans a GPU call).  The Python mirror (libjitsi_amd/srtp.py
// SRTPTransformer.transform) calls these same functions.
#include <algorithm>
#include <new>
#include <stdlib.h>
#include <string.h>
#include <vector>

#include "../../include/srtp_mi355x.h"

struct srtp_rawpacket_batch {
    srtp_engine *e = nullptr;   // engine mode: a pinned pipeline slot is the staging
    srtp_dispatch *d = nullptr; // dispatch mode: host staging (the dispatcher pins per shard)
    // srtp_rawpacket_batch_set_aggregator: small arrays that cannot throw go
    // through this queue on the aggregator's lanes (shared bundles)
    srtp_aggregator *agg = nullptr;
    std::vector<srtp_completion> comps;
    bool via_queue = false;               // the last call took the queue
    std::vector<const uint8_t *> res_ptr; // its results (srtp_rawpacket_result)
    std::vector<uint32_t> res_len;
    std::vector<uint8_t> grown;           // bytes of its results that need a new buffer
    srtp_pipeline *pl = nullptr;
    uint32_t pl_packets = 0;
    size_t pl_bytes = 0;
    // dispatch-mode staging: a segment registered for DMA (srtp_host_alloc),
    // so the dispatcher's shards move it in place, with no second copy
    uint8_t *seg = nullptr;
    size_t seg_cap = 0;
    bool seg_registered = false;
    std::vector<uint32_t> order; // packing order: grouped by shard
    std::vector<uint32_t> off, len, cap, flags;
    std::vector<int32_t> tids, status;
    // the current call's arrays (pipeline slot or the vectors above)
    uint8_t *s_seg = nullptr;
    uint32_t *s_off = nullptr, *s_len = nullptr, *s_cap = nullptr, *s_flags = nullptr;
    int32_t *s_tids = nullptr, *s_status = nullptr;
    uint32_t n = 0;
};

namespace {

constexpr uint32_t kTrailerRoom = 16; // SRTCP E|index (4) + a 12-byte tag: the most protect appends

size_t region(uint32_t cap) { return ((size_t)cap + 15) & ~(size_t)15; }

srtp_engine *engine_of(const srtp_rawpacket_batch *b) {
    return b->e ? b->e : srtp_dispatch_engine(b->d, 0);
}

void release_seg(srtp_rawpacket_batch *b) {
    if (b->seg_registered) (void)srtp_host_free(b->seg);
    else free(b->seg);
    b->seg = nullptr;
    b->seg_cap = 0;
    b->seg_registered = false;
}

// Staging for n packets / bytes: the pipeline slot (grown by recreating the
// pipeline) or the registered host segment and vectors.
int stage(srtp_rawpacket_batch *b, uint32_t n, size_t bytes) {
    if (b->e) {
        if (!b->pl || n > b->pl_packets || bytes > b->pl_bytes) {
            if (b->pl) srtp_pipeline_destroy(b->pl);
            b->pl = nullptr;
            const uint32_t np = std::max<uint32_t>(std::max<uint32_t>(n, 64), b->pl_packets * 2);
            const size_t nb = std::max<size_t>(std::max<size_t>(bytes, (size_t)1 << 16), b->pl_bytes * 2);
            // one synchronous bundle at a time: no copy streams to overlap
            const int rc = srtp_pipeline_create_ex(b->e, np, nb, 1, SRTP_PIPE_ONE_STREAM | SRTP_PIPE_POLL_CROWDED, &b->pl);
            if (rc != SRTP_OK) return rc;
            b->pl_packets = np;
            b->pl_bytes = nb;
        }
        srtp_pipeline_slot sl;
        const int rc = srtp_pipeline_slot_get(b->pl, 0, &sl);
        if (rc != SRTP_OK) return rc;
        b->s_seg = sl.seg; b->s_off = sl.off; b->s_len = sl.len; b->s_cap = sl.cap;
        b->s_flags = sl.flags; b->s_tids = sl.tids; b->s_status = sl.status;
    } else {
        if (bytes > b->seg_cap) {
            release_seg(b);
            const size_t nb = (std::max<size_t>(std::max<size_t>(bytes, (size_t)1 << 20), 2 * b->seg_cap) + 4095) &
                              ~(size_t)4095;
            // pinned memory of the engine's (srtp_host_alloc): the shards' DMA
            // moves it in place; without it (a pinning limit) copies do
            void *p = nullptr;
            b->seg_registered = srtp_host_alloc(nb, &p) == SRTP_OK;
            b->seg = static_cast<uint8_t *>(b->seg_registered ? p : aligned_alloc(4096, nb));
            if (!b->seg) return SRTP_ENOMEM;
            b->seg_cap = nb;
        }
        try {
            b->off.resize(n); b->len.resize(n); b->cap.resize(n); b->flags.resize(n);
            b->tids.resize(n); b->status.resize(n);
        } catch (...) {
            return SRTP_ENOMEM;
        }
        b->s_seg = b->seg; b->s_off = b->off.data(); b->s_len = b->len.data();
        b->s_cap = b->cap.data(); b->s_flags = b->flags.data(); b->s_tids = b->tids.data();
        b->s_status = b->status.data();
    }
    return SRTP_OK;
}

// The region an element gets (RawPacket.isInvalid compares the length with
// it): the buffer after the offset, plus room for the trailer on protect --
// the in-place form of append / grow.  avail = the buffer's bytes after offset.
uint32_t element_cap(int32_t reverse, uint32_t avail, uint32_t length) {
    const bool fits = length <= avail;
    const uint64_t c = (fits && !reverse) ? std::max<uint64_t>(avail, (uint64_t)length + kTrailerRoom) : avail;
    return (uint32_t)std::min<uint64_t>(c, 65535u);
}

// Write-back plan of one processed element (SinglePacketTransformer +
// RawPacket.append / grow / shrink): st / nl = the engine's status and length
// of the packet, old = its length before, avail = the buffer's bytes after
// the offset.  *need = 0: *copy bytes of the result go back in place at the
// offset; else the reference allocates a new buffer of *need bytes at offset 0,
// which receives *copy bytes of the result.  Returns SRTP_OK or a negative
// SRTP_E*.  info(kind, rtcp_tag) gives the transformer's kind and, when
// rtcp_tag != nullptr, its forward factory's SRTCP tag length.
template <class Info>
int plan_back(int32_t reverse, int32_t st, uint32_t avail, uint32_t old, uint32_t nl, Info &&info, uint32_t *copy,
              uint32_t *need) {
    *need = 0;
    *copy = 0;
    if (st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED || st < 0) return SRTP_OK;
    if (old > avail) return SRTP_OK; // RawPacket.isInvalid: untouched (DROP_INVALID)
    if (!reverse && st == SRTP_STATUS_OK) {
        int32_t kind = SRTP_KIND_RTP, rtcp_tag = 0;
        int rc = info(&kind, nullptr);
        if (rc != SRTP_OK) return rc;
        if (kind == SRTP_KIND_RTCP) {
            // grow(4 + tag) then append(E|index, tag): a new buffer of exactly the
            // new length; with NULL authentication nothing is appended and the
            // buffer is length + 4 + the policy's tag length (the forward
            // factory's SRTCP policy: a context kept across an SDES rekey with a
            // different tag length is the one case this does not cover)
            *copy = nl;
            if (nl != old) {
                *need = nl;
                return SRTP_OK;
            }
            rc = info(&kind, &rtcp_tag);
            if (rc != SRTP_OK) return rc;
            *need = old + 4u + (uint32_t)rtcp_tag;
            return SRTP_OK;
        }
        if (nl != old) {
            *copy = nl;
            if (nl > avail) *need = nl; // append reallocates: exactly length + tag
            return SRTP_OK;
        }
    }
    *copy = std::min(old, avail);
    return SRTP_OK;
}

// The same, applied: in place into dst (buffer + offset), or returns need_len
// (the result stays at res for the caller's new buffer), or a negative SRTP_E*.
template <class Info>
int64_t write_back(int32_t reverse, int32_t st, uint8_t *dst, uint32_t avail, uint32_t old, const uint8_t *res,
                   uint32_t nl, Info &&info) {
    uint32_t copy = 0, need = 0;
    const int rc = plan_back(reverse, st, avail, old, nl, info, &copy, &need);
    if (rc != SRTP_OK) return rc;
    if (need) return need;
    if (copy) memcpy(dst, res, copy);
    return 0;
}

constexpr uint32_t kQueueArray = 8192; // arrays up to this size may take the batch's queue
constexpr uint32_t kTagsAny = 0x1fffu; // tag lengths 0..12: every policy the engine takes

// The caller's element i as a queue submit (srtp_rawpacket_submit's rules).
int submit_element(srtp_queue *q, int32_t reverse, int32_t tid, const uint8_t *buf, uint32_t buf_len,
                   uint32_t offset, uint32_t length, uint32_t flags, uint64_t cookie) {
    if (!buf || (flags & SRTP_PKT_FLAG_SKIP))
        return srtp_queue_submit(q, reverse, tid, nullptr, 0, 0, 0, SRTP_PKT_FLAG_SKIP, cookie);
    const uint32_t avail = offset <= buf_len ? buf_len - offset : 0u;
    if (length > avail || length > 65535u) // RawPacket.isInvalid: completes untouched
        return srtp_queue_submit(q, reverse, tid, nullptr, 0, std::min<uint32_t>(length, 65535u), 0, 0, cookie);
    const uint32_t cap = element_cap(reverse, avail, length);
    return srtp_queue_submit(q, reverse, tid, buf + offset, std::min(avail, cap), length, cap,
                             flags & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE), cookie);
}

// srtp_rawpacket_transform through the batch's queue: every element submitted,
// every completion written back as it is reaped.  Only for arrays no packet of
// which can throw (so the aggregator's run without abort-on-throw is the
// reference's result).  Returns 1 when the array is not eligible.
int transform_via_queue(srtp_rawpacket_batch *b, int32_t reverse, const int32_t *tids, int32_t tid,
                        uint8_t *const *bufs, const uint32_t *buf_len, const uint32_t *offset, uint32_t *length,
                        const uint32_t *flags, int32_t *status, uint32_t *need_len, uint32_t n, int32_t *thrown) {
    if (!b->agg || n > kQueueArray) return 1;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t fl = flags ? flags[i] : 0u;
        if (!bufs[i] || (fl & SRTP_PKT_FLAG_SKIP)) continue;
        const uint32_t avail = offset[i] <= buf_len[i] ? buf_len[i] - offset[i] : 0u;
        if (length[i] > avail) continue; // untouched
        int32_t kind = SRTP_KIND_RTP;
        if (srtp_aggregator_transformer_info(b->agg, tids ? tids[i] : tid, &kind, nullptr) != SRTP_OK) return 1;
        const uint32_t cap = std::min(avail, element_cap(reverse, avail, length[i]));
        if (srtp_packet_may_throw(kind, reverse, bufs[i] + offset[i], length[i], cap, fl, kTagsAny)) return 1;
    }
    // The queue lives for this call only: a queue outliving it would hold the
    // aggregator (srtp_aggregator_destroy waits for every queue), and the
    // batch belongs to a thread that may outlive the aggregator's owner.
    srtp_queue *q = nullptr;
    {
        const int rc = srtp_queue_create(b->agg, kQueueArray, &q);
        if (rc != SRTP_OK) return rc;
    }
    struct QueueOf { // destroyed on every return below (after what was queued completed)
        srtp_queue *q;
        ~QueueOf() { srtp_queue_destroy(q); }
    } q_guard{q};
    std::vector<uint8_t> completed;
    try {
        b->comps.resize(kQueueArray);
        b->res_ptr.assign(n, nullptr);
        b->res_len.assign(n, 0u);
        completed.assign(n, 0u);
    } catch (...) {
        return SRTP_ENOMEM;
    }
    b->grown.clear();
    std::vector<size_t> grown_at;
    uint32_t done = 0;
    int err = SRTP_OK;
    auto reap = [&](int32_t wait) {
        const int k = srtp_queue_reap(q, b->comps.data(), kQueueArray, wait);
        if (k < 0) return k;
        for (int j = 0; j < k; j++) {
            const srtp_completion &c = b->comps[(size_t)j];
            const uint32_t i = (uint32_t)c.cookie;
            const int32_t st = c.status < 0 ? SRTP_STATUS_ERR_INTERNAL : c.status;
            status[i] = st;
            need_len[i] = 0;
            completed[i] = 1u;
            done++;
            if (!bufs[i] || st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED) continue;
            const uint32_t avail = offset[i] <= buf_len[i] ? buf_len[i] - offset[i] : 0u;
            uint32_t copy = 0, need = 0;
            const int rc = plan_back(reverse, st, avail, c.in_len, c.len, [&](int32_t *kind, int32_t *tag) {
                return srtp_aggregator_transformer_info(b->agg, c.tid, kind, tag);
            }, &copy, &need);
            if (rc != SRTP_OK) {
                err = rc;
                continue;
            }
            if (need) { // kept for srtp_rawpacket_result
                grown_at.resize(n, SIZE_MAX);
                grown_at[i] = b->grown.size();
                b->grown.insert(b->grown.end(), c.data, c.data + copy);
                need_len[i] = need;
                b->res_len[i] = copy;
            } else {
                if (copy) memcpy(bufs[i] + offset[i], c.data, copy);
                b->res_ptr[i] = bufs[i] + offset[i];
                b->res_len[i] = c.len;
            }
            if (c.data) length[i] = c.len;
            if (st == SRTP_STATUS_ERR_MALFORMED && (*thrown < 0 || (int32_t)i < *thrown)) *thrown = (int32_t)i;
        }
        srtp_queue_release(q); // written back: the slots go back at once
        return SRTP_OK;
    };
    // the results of the elements that completed stay readable
    // (srtp_rawpacket_result); the others are left untouched with
    // SRTP_STATUS_ERR_INTERNAL, as the dispatcher leaves chunks never submitted
    auto finish = [&](int rc) {
        for (uint32_t i = 0; i < n; i++) {
            if (need_len[i] && completed[i]) b->res_ptr[i] = b->grown.data() + grown_at[i];
            if (!completed[i]) {
                status[i] = SRTP_STATUS_ERR_INTERNAL;
                need_len[i] = 0;
            }
        }
        b->via_queue = true;
        b->n = n;
        return rc;
    };
    for (uint32_t i = 0; i < n; i++) need_len[i] = 0;
    for (uint32_t i = 0; i < n; i++) {
        for (;;) {
            int rc2;
            const int rc = submit_element(q, reverse, tids ? tids[i] : tid, bufs[i], buf_len[i], offset[i],
                                          length[i], flags ? flags[i] : 0u, i);
            if (rc == SRTP_OK) break;
            if (rc == SRTP_EAGAIN) rc2 = reap(1);
            else rc2 = rc; // nothing of this element was queued
            if (rc2 != SRTP_OK) {
                // what was queued completes (written back) before the error returns
                while (srtp_queue_outstanding(q) > 0 && reap(1) == SRTP_OK) {
                }
                return finish(rc2);
            }
        }
    }
    while (done < n) {
        const int rc = reap(1);
        if (rc != SRTP_OK) {
            while (srtp_queue_outstanding(q) > 0 && reap(1) == SRTP_OK) {
            }
            return finish(rc);
        }
    }
    return finish(err);
}

} // namespace

extern "C" {

int srtp_rawpacket_batch_create(srtp_engine *e, srtp_rawpacket_batch **out) {
    if (!e || !out) return SRTP_EINVAL;
    srtp_rawpacket_batch *b = new (std::nothrow) srtp_rawpacket_batch();
    if (!b) return SRTP_ENOMEM;
    b->e = e;
    *out = b;
    return SRTP_OK;
}

int srtp_rawpacket_batch_create_dispatch(srtp_dispatch *d, srtp_rawpacket_batch **out) {
    if (!d || !out) return SRTP_EINVAL;
    srtp_rawpacket_batch *b = new (std::nothrow) srtp_rawpacket_batch();
    if (!b) return SRTP_ENOMEM;
    b->d = d;
    *out = b;
    return SRTP_OK;
}

void srtp_rawpacket_batch_destroy(srtp_rawpacket_batch *b) {
    if (!b) return;
    if (b->pl) srtp_pipeline_destroy(b->pl);
    release_seg(b);
    delete b;
}

int srtp_rawpacket_transform(srtp_rawpacket_batch *b, int32_t reverse, const int32_t *tids, int32_t tid,
                             uint8_t *const *bufs, const uint32_t *buf_len, const uint32_t *offset,
                             uint32_t *length, const uint32_t *flags, int32_t *status,
                             uint32_t *need_len, uint32_t n, int32_t *thrown) {
    if (!b || (n && (!bufs || !buf_len || !offset || !length || !status || !need_len)) || !thrown)
        return SRTP_EINVAL;
    *thrown = -1;
    b->n = 0;
    b->via_queue = false;
    if (n == 0) return SRTP_OK;
    {
        const int rc = transform_via_queue(b, reverse, tids, tid, bufs, buf_len, offset, length, flags, status,
                                           need_len, n, thrown);
        if (rc != 1) return rc;
    }
    srtp_engine *eng = engine_of(b);
    // Packing (the JNI shim's copy of each buffer):
    // region i holds the buffer's bytes from the packet's offset on, so the
    // reference's reads past `length` (getHeaderLength's extension field,
    // readRegionToBuff) see the same bytes; cap is the buffer's length after
    // the offset (RawPacket.isInvalid compares against it), plus room for the
    // trailer on protect -- the in-place form of append / grow.
    std::vector<uint32_t> avail(n), ccap(n);
    size_t bytes = 0;
    for (uint32_t i = 0; i < n; i++) {
        const bool skip = !bufs[i] || (flags && (flags[i] & SRTP_PKT_FLAG_SKIP));
        if (skip) {
            avail[i] = 0;
            ccap[i] = 16;
        } else {
            avail[i] = offset[i] <= buf_len[i] ? buf_len[i] - offset[i] : 0u;
            ccap[i] = element_cap(reverse, avail[i], length[i]);
        }
        bytes += region(ccap[i]);
    }
    int rc = stage(b, n, bytes);
    if (rc != SRTP_OK) return rc;
    // Over a dispatcher of several shards, the regions are laid out grouped by
    // the shard the dispatcher will route each packet to (in array order
    // within a shard), so each shard's packets lie back to back and its chunks
    // move by DMA in place.  The routing here only needs to agree with the
    // dispatcher's for the layout to pay; results never depend on it.
    const int32_t ns = b->d ? srtp_dispatch_num_shards(b->d) : 1;
    const uint32_t *ord = nullptr;
    if (ns > 1) {
        try {
            b->order.resize(n);
        } catch (...) {
            return SRTP_ENOMEM;
        }
        std::vector<uint32_t> at((size_t)ns + 1, 0u);
        std::vector<int32_t> sh(n);
        for (uint32_t i = 0; i < n; i++) {
            const bool skip = !bufs[i] || (flags && (flags[i] & SRTP_PKT_FLAG_SKIP));
            int32_t s = 0;
            if (!skip && length[i] <= ccap[i] && length[i] <= avail[i])
                s = srtp_dispatch_route(b->d, tids ? tids[i] : tid, bufs[i] + offset[i], length[i]);
            sh[i] = s < 0 ? 0 : s;
            at[(size_t)sh[i] + 1]++;
        }
        for (int32_t s = 0; s < ns; s++) at[(size_t)s + 1] += at[(size_t)s];
        for (uint32_t i = 0; i < n; i++) b->order[at[(size_t)sh[i]]++] = i;
        ord = b->order.data();
    }
    size_t pos = 0;
    for (uint32_t q = 0; q < n; q++) {
        const uint32_t i = ord ? ord[q] : q;
        const bool skip = !bufs[i] || (flags && (flags[i] & SRTP_PKT_FLAG_SKIP));
        const size_t r = region(ccap[i]);
        b->s_off[i] = (uint32_t)pos;
        b->s_cap[i] = ccap[i];
        b->s_tids[i] = tids ? tids[i] : tid;
        if (skip) {
            b->s_len[i] = 0;
            b->s_flags[i] = SRTP_PKT_FLAG_SKIP;
            memset(b->s_seg + pos, 0, r);
        } else {
            b->s_len[i] = length[i];
            b->s_flags[i] = flags ? (flags[i] & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE)) : 0u;
            const size_t c = std::min<size_t>(avail[i], ccap[i]);
            memcpy(b->s_seg + pos, bufs[i] + offset[i], c);
            memset(b->s_seg + pos + c, 0, r - c);
        }
        pos += r;
    }
    if (b->e) {
        rc = srtp_pipeline_submit(b->pl, 0, reverse, 1, -1, 1, n, pos);
        if (rc == SRTP_OK) rc = srtp_pipeline_wait(b->pl, 0);
    } else {
        rc = srtp_dispatch_transform_host(b->d, reverse, b->s_tids, -1, b->s_seg, pos, b->s_off, b->s_len,
                                          b->s_cap, b->s_flags, b->s_status, n);
    }
    if (rc != SRTP_OK) return rc;
    b->n = n;
    // Write-back (SinglePacketTransformer + RawPacket.append / grow / shrink).
    int32_t info_tid = -1, info_kind = SRTP_KIND_RTP;
    for (uint32_t i = 0; i < n; i++) {
        need_len[i] = 0;
        const int32_t st = b->s_status[i];
        status[i] = st;
        if (!bufs[i] || st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED) continue;
        const int32_t t = tids ? tids[i] : tid;
        const int64_t need = write_back(reverse, st, bufs[i] + offset[i], avail[i], length[i],
                                        b->s_seg + b->s_off[i], b->s_len[i], [&](int32_t *kind, int32_t *tag) {
            if (!tag && t == info_tid) {
                *kind = info_kind;
                return SRTP_OK;
            }
            const int rc = srtp_transformer_info(eng, t, kind, tag);
            if (rc == SRTP_OK) {
                info_tid = t;
                info_kind = *kind;
            }
            return rc;
        });
        if (need < 0) return (int)need;
        need_len[i] = (uint32_t)need;
        length[i] = b->s_len[i];
        if (st == SRTP_STATUS_ERR_MALFORMED && *thrown < 0) *thrown = (int32_t)i;
    }
    return SRTP_OK;
}

int srtp_rawpacket_result(srtp_rawpacket_batch *b, uint32_t i, const uint8_t **data, uint32_t *len) {
    if (!b || !data || !len || i >= b->n) return SRTP_EINVAL;
    if (b->via_queue) {
        if (!b->res_ptr[i]) return SRTP_EINVAL; // untouched element
        *data = b->res_ptr[i];
        *len = b->res_len[i];
        return SRTP_OK;
    }
    *data = b->s_seg + b->s_off[i];
    *len = b->s_len[i];
    return SRTP_OK;
}

int srtp_rawpacket_batch_set_aggregator(srtp_rawpacket_batch *b, srtp_aggregator *a) {
    if (!b) return SRTP_EINVAL;
    b->agg = a; // (the queue path makes a queue per call on it)
    return SRTP_OK;
}

int srtp_rawpacket_submit(srtp_queue *q, int32_t reverse, int32_t tid, const uint8_t *buf, uint32_t buf_len,
                          uint32_t offset, uint32_t length, uint32_t flags, uint64_t cookie) {
    if (!q) return SRTP_EINVAL;
    return submit_element(q, reverse, tid, buf, buf_len, offset, length, flags, cookie);
}

int srtp_rawpacket_complete(srtp_queue *q, const srtp_completion *c, uint32_t avail, uint32_t *copy_len,
                            uint32_t *need_len) {
    if (!q || !c || !copy_len || !need_len) return SRTP_EINVAL;
    srtp_aggregator *a = srtp_queue_aggregator(q);
    const int rc = plan_back(c->reverse, c->status, avail, c->in_len, c->len, [&](int32_t *kind, int32_t *tag) {
        return srtp_aggregator_transformer_info(a, c->tid, kind, tag);
    }, copy_len, need_len);
    if (rc == SRTP_OK && !c->data) *copy_len = 0; // completed at submit: untouched
    return rc;
}

int srtp_rawpacket_transform_one(srtp_aggregator *a, int32_t reverse, int32_t tid, uint8_t *buf,
                                 uint32_t buf_len, uint32_t offset, uint32_t *length, uint32_t flags,
                                 int32_t *status, uint32_t *need_len, uint8_t *grow, uint32_t grow_cap) {
    if (!a || !length || !status || !need_len || !grow) return SRTP_EINVAL;
    *need_len = 0;
    if (!buf || (flags & SRTP_PKT_FLAG_SKIP)) { // a null element / the predicate said no: untouched
        *status = SRTP_STATUS_SKIPPED;
        return SRTP_OK;
    }
    const uint32_t avail = offset <= buf_len ? buf_len - offset : 0u;
    const uint32_t old = *length;
    if (old > 65535u || old > avail) { // RawPacket.isInvalid, as the array path reports it: untouched
        *status = SRTP_STATUS_DROP_INVALID;
        return SRTP_OK;
    }
    const uint32_t cap = element_cap(reverse, avail, old);
    if (grow_cap < cap) return SRTP_EINVAL;
    uint32_t nl = 0;
    int rc = srtp_aggregator_transform(a, reverse, tid, buf + offset, std::min(avail, cap), old, cap,
                                       flags & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE), grow, status, &nl);
    if (rc != SRTP_OK) return rc;
    const int32_t st = *status;
    if (st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED) return SRTP_OK;
    const int64_t need = write_back(reverse, st, buf + offset, avail, old, grow, nl,
                                    [&](int32_t *kind, int32_t *tag) {
                                        return srtp_aggregator_transformer_info(a, tid, kind, tag);
                                    });
    if (need < 0) return (int)need;
    *need_len = (uint32_t)need;
    *length = nl;
    return SRTP_OK;
}

} // extern "C"
