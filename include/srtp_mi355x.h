/*
 * srtp_mi355x.h -- C ABI of the MI355X SRTP/SRTCP packet-crypto engine.
 *
 * Drop-in boundary for libjitsi's SRTP hot path.  Each entry point replaces a
 * reference Java API (paths relative to src/org/jitsi/impl/neomedia/):
 *
 *   srtp_factory_create        <- new SRTPContextFactory(sender, masterKey,
 *                                 masterSalt, srtpPolicy, srtcpPolicy)
 *                                 transform/srtp/SRTPContextFactory.java:50-68
 *   srtp_factory_close         <- SRTPContextFactory.close()          :74-86
 *   srtp_transformer_create    <- new SRTPTransformer(fwd, rev)
 *                                 transform/srtp/SRTPTransformer.java:82-90,
 *                                 new SRTCPTransformer(fwd, rev)
 *                                 transform/srtp/SRTCPTransformer.java:73-80
 *   srtp_transformer_set_factory <- SRTPTransformer.setContextFactory :100-125,
 *                                 SRTCPTransformer.updateFactory      :92-117
 *   srtp_transformer_close     <- SRTPTransformer.close() :132-150,
 *                                 SRTCPTransformer.close() :124-142
 *   srtp_transform_device /    <- PacketTransformer.transform(RawPacket[]) and
 *   srtp_transform_host           .reverseTransform(RawPacket[])
 *                                 transform/PacketTransformer.java:28-53 as
 *                                 implemented by SinglePacketTransformer
 *                                 transform/SinglePacketTransformer.java:121-216
 *                                 over SRTPTransformer.transform/reverseTransform
 *                                 transform/srtp/SRTPTransformer.java:185-219
 *                                 (per packet: SRTPCryptoContext.transformPacket
 *                                 :658-705 / reverseTransformPacket :572-642,
 *                                 SRTCPCryptoContext.transformPacket :391-427 /
 *                                 reverseTransformPacket :315-374)
 *   srtp_engine_opts.check_replay <- ConfigurationService property
 *                                 ...srtp.SRTPCryptoContext.checkReplay
 *                                 (SRTPCryptoContext.java:80-121)
 *
 * Packet bundle model (RawPacket[] -> packed segment).  Packet i occupies
 * seg[off[i] .. off[i] + cap[i]) and its current RTP/RTCP length is len[i]
 * (RawPacket.length).  The engine works in place: protect appends the tag (and
 * for SRTCP the E|index word) inside cap[i]; unprotect shrinks len[i].
 * Requirements: off[i] % 16 == 0, cap[i] <= 65535, and the segment must be
 * readable and writable up to off[i] + roundup16(cap[i]) for every packet.
 * status[i] receives one SRTP_STATUS_* value; "drop" statuses correspond to
 * the reference returning null for that element.
 *
 * Ownership: the caller owns every buffer; the engine owns contexts, session
 * keys and device scratch, and zeroes keys when factories are closed.
 * Threading: calls on one engine are serialised internally and are safe from
 * any host thread: each call makes the engine's device current for its
 * duration and restores the caller's device (one process may drive engines on
 * several GPUs).  Bundles of one engine are processed in submission order
 * (== the order the reference's `synchronized` contexts give): a bundle
 * submitted on another stream than the engine's previous bundle waits for
 * that bundle on the device, with no host stall.  Control-plane calls
 * (factory/transformer close and rekey, context state, stats) first wait for
 * every bundle the engine has enqueued.  Independent directions that should
 * overlap on the device use one engine each (e.g. a send-side and a
 * receive-side engine).
 */
#ifndef SRTP_MI355X_H
#define SRTP_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRTP_MI355X_ABI_VERSION 3

/* SRTPPolicy constants (transform/srtp/SRTPPolicy.java:29-63) */
#define SRTP_NULL_ENCRYPTION 0
#define SRTP_AESCM_ENCRYPTION 1
#define SRTP_AESF8_ENCRYPTION 2 /* SRTPCipherF8 (SDES F8_128_HMAC_SHA1_80) */
#define SRTP_TWOFISH_ENCRYPTION 3   /* counter mode over Twofish (ZRTP "2FS") */
#define SRTP_TWOFISHF8_ENCRYPTION 4 /* F8 over Twofish */
#define SRTP_NULL_AUTHENTICATION 0
#define SRTP_HMACSHA1_AUTHENTICATION 1
#define SRTP_SKEIN_AUTHENTICATION 2 /* Skein-512 MAC, tag_len * 8 output bits (ZRTP "SK32"/"SK64") */

/* transformer kinds */
#define SRTP_KIND_RTP 0  /* SRTPTransformer */
#define SRTP_KIND_RTCP 1 /* SRTCPTransformer */

/* per-packet status */
#define SRTP_STATUS_OK 0
#define SRTP_STATUS_DROP_REPLAY 1     /* checkReplay() false */
#define SRTP_STATUS_DROP_AUTH 2       /* authenticatePacket() false */
#define SRTP_STATUS_DROP_VERSION 3    /* (byte0 & 0xC0) != 0x80 (SRTPTransformer.java:189) */
#define SRTP_STATUS_DROP_NO_CONTEXT 4 /* factory closed, no context for the SSRC */
#define SRTP_STATUS_ERR_CAPACITY 5    /* cap[i] too small for the appended trailer */
#define SRTP_STATUS_ERR_MALFORMED 6   /* the reference throws on this packet */
#define SRTP_STATUS_DROP_INVALID 7    /* len < 12 or len > cap (RawPacket.isInvalid) */
#define SRTP_STATUS_NOT_PROCESSED 8   /* after an ERR_MALFORMED with abort_on_error */
#define SRTP_STATUS_SKIPPED 9         /* SRTP_PKT_FLAG_SKIP (null element / predicate) */
#define SRTP_STATUS_ERR_INTERNAL 10   /* no walk reached the packet: an engine bug (never expected);
                                         the packet and its context are left as they were */
#define SRTP_NUM_STATUS 11

/* per-packet flags (javax.media.Buffer values read at SRTPCryptoContext.java:609) */
#define SRTP_PKT_FLAG_DISCARD 0x2u
#define SRTP_PKT_FLAG_SILENCE 0x4u
#define SRTP_PKT_FLAG_SKIP 0x80000000u

/* return codes */
#define SRTP_OK 0
#define SRTP_EINVAL -1
#define SRTP_ENOMEM -2
#define SRTP_EFULL -3   /* context / factory / transformer table full */
#define SRTP_EDEVICE -4 /* HIP runtime error */
#define SRTP_EPOLICY -5 /* policy outside the implemented ciphers x MACs (see srtp_factory_create) */
#define SRTP_EAGAIN -6  /* srtp_queue_submit: the queue is full, or no slot is free while it holds
                           completed packets -- reap, then submit again */

typedef struct srtp_engine srtp_engine;

/* SRTPPolicy(encType, encKeyLength, authType, authKeyLength, authTagLength,
 * saltKeyLength) -- SRTPPolicy.java:107-120 */
typedef struct {
    int32_t enc_type, enc_key_len, auth_type, auth_key_len, auth_tag_len, salt_key_len;
} srtp_policy;

typedef struct {
    int32_t device;            /* HIP device ordinal */
    int32_t check_replay;      /* SRTPCryptoContext.checkReplay, default 1 */
    int32_t abort_on_error;    /* SinglePacketTransformer rethrow semantics, default 1 */
    uint32_t max_contexts;     /* (transformer, SSRC) contexts, default 1<<20 (table of
                                  next_pow2(2 * max_contexts) slots, 40 B each) */
    uint32_t max_factories;    /* default 1<<16 */
    uint32_t max_transformers; /* default 1<<16 */
    uint32_t max_batch;        /* initial scratch size in packets (grows), default 1<<16 */
} srtp_engine_opts;

typedef struct {
    int32_t roc, s_l, seq_num_set, guessed_roc; /* SRTP context */
    int32_t sent_index, received_index;         /* SRTCP context */
    uint64_t replay_window;
    uint32_t key_set;                           /* internal session-key slot */
} srtp_ctx_state;

int srtp_engine_opts_default(srtp_engine_opts *opts);
int srtp_engine_create(const srtp_engine_opts *opts, srtp_engine **out);
void srtp_engine_destroy(srtp_engine *e);
/* the options the engine was created with */
int srtp_engine_get_opts(srtp_engine *e, srtp_engine_opts *out);
const char *srtp_engine_last_error(srtp_engine *e);

int srtp_factory_create(srtp_engine *e, int32_t sender, const uint8_t *master_key,
                        int32_t key_len, const uint8_t *master_salt, int32_t salt_len,
                        const srtp_policy *srtp, const srtp_policy *srtcp, int32_t *out_factory);
int srtp_factory_close(srtp_engine *e, int32_t factory);

int srtp_transformer_create(srtp_engine *e, int32_t kind, int32_t fwd_factory,
                            int32_t rev_factory, int32_t *out_transformer);
int srtp_transformer_set_factory(srtp_engine *e, int32_t transformer, int32_t factory,
                                 int32_t forward);
int srtp_transformer_close(srtp_engine *e, int32_t transformer);
/* The transformer's kind and its forward factory's SRTCP policy tag length
 * (what RawPacket.grow sizes an SRTCP packet with, SRTCPCryptoContext.java:413). */
int srtp_transformer_info(srtp_engine *e, int32_t transformer, int32_t *kind,
                          int32_t *fwd_rtcp_tag_len);

/* Process one bundle whose buffers are device (HBM) pointers on the engine's
 * device; asynchronous on `stream` (a hipStream_t of that device; NULL = its
 * default stream, ordered with the caller's default-stream work).  For a
 * send-side and a receive-side engine to overlap on the device, pass each its
 * own stream (srtp_engine_stream).  tids == NULL means every
 * packet belongs to `tid`; otherwise tids[i] (device array) names packet i's
 * transformer.  flags may be NULL.  reverse = 0: transform (protect),
 * reverse = 1: reverseTransform (unprotect).  The caller guarantees what
 * srtp_transform_host checks on the host: every packet region [off[i],
 * off[i] + cap[i] rounded up to 16) lies inside the segment, off[i] is 16-byte
 * aligned and cap[i] <= 65535 (the device arrays are not read back to check). */
int srtp_transform_device(srtp_engine *e, int32_t reverse, const int32_t *tids, int32_t tid,
                          uint8_t *seg, const uint32_t *off, uint32_t *len, const uint32_t *cap,
                          const uint32_t *flags, int32_t *status, uint32_t n, void *stream);

/* Same with host buffers: copies to HBM, runs, copies back, synchronises.
 * seg_bytes is the size of the host segment. */
int srtp_transform_host(srtp_engine *e, int32_t reverse, const int32_t *tids, int32_t tid,
                        uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                        const uint32_t *cap, const uint32_t *flags, int32_t *status, uint32_t n);

/* The engine's own non-blocking stream, created with the engine so that each
 * engine gets a hardware queue of its own (streams created later may share
 * one, which serialises them): srtp_transform_host and the pipeline run their
 * kernels on it, and srtp_transform_device callers can. */
void *srtp_engine_stream(srtp_engine *e);
/* stream == NULL: wait for every bundle this engine has enqueued (any stream) */
int srtp_engine_sync(srtp_engine *e, void *stream);
/* returns 1 and fills *out if the transformer has a context for ssrc, else 0 */
int srtp_get_context_state(srtp_engine *e, int32_t transformer, uint32_t ssrc,
                           srtp_ctx_state *out);
/* number of live contexts in the engine's table */
int64_t srtp_engine_num_contexts(srtp_engine *e);

/* Per-engine counters (SURVEY.md 5 metrics).  The reference keeps none for
 * auth / replay failures (SRTPCryptoContext.java:635-638 logs at debug level)
 * and counts only exceptions (SinglePacketTransformer.java:42,54-59,140-148);
 * here every final per-packet status is counted, cumulatively since engine
 * creation.  ctx_overflow counts packets that found no free context slot (they
 * get SRTP_STATUS_DROP_NO_CONTEXT); ctx_live / ctx_tombstones / ctx_slots
 * describe the context table at the time of the call. */
typedef struct {
    uint64_t bundles, packets;           /* bundles / packets submitted */
    uint64_t status[SRTP_NUM_STATUS];    /* final statuses, indexed by SRTP_STATUS_* */
    uint64_t roc_rechecks;               /* unprotect tags re-checked under a ROC the walk
                                            guessed differently from the speculation */
    uint64_t repaired;                   /* packets whose speculative decryption was redone */
    uint64_t ctx_overflow;               /* packets refused a new context: table full */
    uint64_t ctx_live, ctx_tombstones, ctx_slots;
    uint64_t rehashes;                   /* context-table rebuilds (tombstone cleanup) */
    uint64_t chain_stalls;               /* walk tiles that gave up waiting for a long chain's
                                            state from the tiles before (never expected; the
                                            chain is then walked serially from the exact state
                                            by the last tile to finish, so results stay exact) */
    uint64_t long_walked;                /* packets of chains of 32+ packets that the wave-wide
                                            speculation could not take and were walked one at
                                            a time (the slow path) */
    uint64_t holes;                      /* bundle-former holes: SRTP_PKT_FLAG_SKIP entries of no
                                            transformer (tid < 0) that srtp_aggregator_* seals
                                            unclaimed; not in status[SRTP_STATUS_SKIPPED] */
    uint64_t small_bundles;              /* bundles run by k_small: every phase in one launch */
} srtp_stats;
int srtp_engine_stats(srtp_engine *e, srtp_stats *out);

/* Test hooks (0 in production): SRTP_DEBUG_FORCE_CHAIN_STALL makes every third
 * chain-pass walk tile give up its look-back at once, which exercises the
 * stall fix-up (srtp_stats.chain_stalls) that a tile preempted for seconds
 * would take.  Results must not change. */
#define SRTP_DEBUG_FORCE_CHAIN_STALL 0x1u
/* SRTP_DEBUG_FORCE_WIDE runs bundles of every size on the split path (the
 * cipher and the MAC as two kernels, which bundles of 2048-65536 packets take
 * when every key set is AES-CM or NULL cipher with HMAC-SHA1), so that every
 * parity case exercises it; SRTP_DEBUG_NO_WIDE keeps every bundle off it
 * (A/B measurements).  Results must not change. */
#define SRTP_DEBUG_FORCE_WIDE 0x2u
#define SRTP_DEBUG_NO_WIDE 0x4u
/* SRTP_DEBUG_NO_SMALL keeps bundles of up to 255 packets off k_small (the
 * whole bundle -- parse, sort, walk, keystream, MAC -- in one workgroup and
 * one launch, which such bundles take under the split path's key-set rule);
 * FORCE_WIDE and NO_WIDE keep them off it too. */
#define SRTP_DEBUG_NO_SMALL 0x8u
int srtp_engine_set_debug(srtp_engine *e, uint32_t flags);

/* Context-state export / import: lets a stream's ROC, s_l,
 * replay window and SRTCP indices follow it to another engine or GPU (SSRC
 * re-sharding, failover) or survive a transformer rebuild.  The reference keeps
 * this state inside SRTPCryptoContext (srtp/SRTPCryptoContext.java:96-135) with
 * no API for it; DtlsPacketTransformer rebuilds contexts from scratch on rekey
 * (tf/dtls/DtlsPacketTransformer.java:614-642).
 *
 * srtp_export_contexts writes up to `max` (ssrc, state) pairs of the
 * transformer's contexts and sets *count to the number it has (which may
 * exceed max).  srtp_set_context_state creates or overwrites the transformer's
 * context for ssrc with *st (key_set ignored); its session keys are those of
 * the transformer's forward (forward = 1) or reverse factory, which must be
 * open.  Both synchronise the engine's device. */
int srtp_export_contexts(srtp_engine *e, int32_t transformer, uint32_t *ssrcs,
                         srtp_ctx_state *states, uint32_t max, uint32_t *count);
int srtp_set_context_state(srtp_engine *e, int32_t transformer, uint32_t ssrc, int32_t forward,
                           const srtp_ctx_state *st);

/* Exact context snapshots (the dispatcher's abort rollback, dispatch.cpp):
 * srtp_contexts_save copies the contexts (tids[i], ssrcs[i]) -- their whole
 * record, key set included, as an opaque srtp_ctx_raw -- and sets present[i]
 * to 0 where the transformer has no context for ssrcs[i].  srtp_contexts_restore
 * puts such a snapshot back: the context is created or overwritten where
 * present[i] != 0 and removed where present[i] == 0, so the table is as it
 * was when the snapshot was taken.  The (tid, ssrc) pairs of one restore call
 * must be distinct.  Both wait for the engine's enqueued bundles.  No
 * reference API (SRTPCryptoContext's state is private). */
typedef struct {
    uint64_t w[4];
} srtp_ctx_raw;
int srtp_contexts_save(srtp_engine *e, uint32_t n, const int32_t *tids, const uint32_t *ssrcs,
                       srtp_ctx_raw *out, int32_t *present);
int srtp_contexts_restore(srtp_engine *e, uint32_t n, const int32_t *tids, const uint32_t *ssrcs,
                          const srtp_ctx_raw *in, const int32_t *present);

/* Per-stage kernel timing with HIP events recorded on the bundle's stream
 * (measurement hook for bench.py; off by default). */
#define SRTP_STAGE_PARSE 0
#define SRTP_STAGE_SORT 1
#define SRTP_STAGE_VERIFY 2
#define SRTP_STAGE_WALK 3
#define SRTP_STAGE_PROTECT 4
#define SRTP_STAGE_DECRYPT 5
#define SRTP_NUM_STAGES 6
int srtp_engine_set_timing(srtp_engine *e, int32_t enable);
/* Waits for the recorded events, adds each stage's total milliseconds and
 * bundle count since the last read into ms[] / count[], and resets. */
int srtp_engine_read_timing(srtp_engine *e, double *ms, uint64_t *count);

/* Host bundle pipeline (SURVEY.md 8d end-to-end timing, 8f.2 bundle former):
 * `depth` slots of pinned host memory the caller packs bundles into directly
 * (the RawPacket[] -> packed-segment marshalling a JNI shim does; see
 * INTEGRATION.md), each moved H2D on a copy stream, processed by the engine on
 * its stream in submission order, and moved D2H on a second copy stream, so
 * slot i's copies overlap slot j's kernels.  Replaces the reference's
 * per-packet calls through PacketTransformer.transform/reverseTransform
 * (transform/PacketTransformer.java:28-53) fed 1-element arrays by
 * RTPConnectorInputStream.java:425-452 / RTPConnectorOutputStream.java:268-300.
 *
 * srtp_pipeline_slot_get returns slot i's pinned arrays (seg holds seg_cap
 * bytes; the per-packet arrays hold max_packets entries).  srtp_pipeline_submit
 * enqueues slot i's first n packets (seg_bytes of segment) as one bundle for
 * transformer `tid`, or per packet from slot.tids when use_tids != 0; flags
 * are passed when use_flags != 0.  It first waits for the slot's previous
 * bundle.  srtp_pipeline_wait blocks until slot i's results (seg, len, status)
 * are back in its pinned arrays.  Packet regions are validated as in
 * srtp_transform_host. */
typedef struct srtp_pipeline srtp_pipeline;
typedef struct {
    uint8_t *seg;
    size_t seg_cap;
    uint32_t *off, *len, *cap, *flags;
    int32_t *tids, *status;
    uint32_t max_packets;
} srtp_pipeline_slot;
int srtp_pipeline_create(srtp_engine *e, uint32_t max_packets, size_t max_seg_bytes,
                         int32_t depth, srtp_pipeline **out);
void srtp_pipeline_destroy(srtp_pipeline *pl);
int srtp_pipeline_slot_get(srtp_pipeline *pl, int32_t slot, srtp_pipeline_slot *out);
int srtp_pipeline_submit(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                         int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes);
int srtp_pipeline_wait(srtp_pipeline *pl, int32_t slot);
/* 1 when slot's bundle has come back (srtp_pipeline_wait then returns without
 * blocking) or none is in flight, 0 while it is still running, < 0 on error. */
int srtp_pipeline_query(srtp_pipeline *pl, int32_t slot);
/* srtp_pipeline_create with flags.  SRTP_PIPE_ONE_STREAM puts the copies on
 * the engine's own stream instead of two copy streams of the pipeline's: a
 * bundle's H2D, kernels and D2H then run in order with no cross-stream
 * events.  For engines that share a GPU (several dispatcher shards or
 * aggregator lanes on one device): every stream maps onto one of the device's
 * few hardware queues (GPU_MAX_HW_QUEUES, 4 by default), and a queue that
 * holds one engine's kernel waiting on its copy event stalls every other
 * engine's work behind it.  Without the flag, bundles of up to 1 MB still
 * copy on the engine's stream (their round trip is fixed costs, and two
 * cross-stream events are among them); larger ones use the copy streams. */
#define SRTP_PIPE_ONE_STREAM 0x1u
/* SRTP_PIPE_POLL_CROWDED: a wait on this pipeline polls the bundle's event
 * (sleeping between polls) instead of spinning in hipEventSynchronize while
 * more than 4 threads of the process
 * wait on such pipelines -- for one pipeline per caller thread (the 1-packet
 * RawPacket path): 64 spinning callers took the host's cores from the threads
 * enqueueing the next bundles.  Few waiters keep the spin's quicker wake-up. */
#define SRTP_PIPE_POLL_CROWDED 0x2u
int srtp_pipeline_create_ex(srtp_engine *e, uint32_t max_packets, size_t max_seg_bytes, int32_t depth,
                            uint32_t flags, srtp_pipeline **out);
/* srtp_pipeline_submit with the bundle's abort-on-throw chosen per bundle:
 * abort_on_error = -1 the engine's option, 1 SinglePacketTransformer's abort of
 * a throwing transformer's later packets (one RawPacket[] call), 0 none (every
 * packet its own 1-element array: the bundle former's bundles).  One engine
 * can so serve both kinds of call with the same contexts. */
int srtp_pipeline_submit_ex(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                            int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                            int32_t abort_on_error);

/* Registered host memory: the zero-copy host path.  srtp_host_register pins
 * [ptr, ptr + bytes) for DMA by every device of the process (hipHostRegister,
 * portable) -- a long-lived buffer pool, e.g. the JVM's direct ByteBuffers a
 * media server receives into, registered once.  Ranges may not overlap;
 * srtp_host_unregister takes the pointer that was registered, and the caller
 * must not unregister or free a range while a call uses it.
 * srtp_host_is_registered tells whether [ptr, ptr + bytes) lies inside one
 * registered range.  srtp_host_alloc allocates such a range as pinned memory
 * of the engine's own (hipHostMalloc; freed with srtp_host_free): the DMA
 * engines read it at the full PCIe rate, while registered pageable memory of
 * 4-KB pages may move slower.  A JVM would wrap it as a direct ByteBuffer
 * (NewDirectByteBuffer).  No reference API: the reference's packets are heap
 * byte[]s copied by every JNI call (src/native/openssl/).
 *
 * srtp_pipeline_submit_host is srtp_pipeline_submit_ex with the segment read
 * from, and written back to, registered caller memory (host_seg, seg_bytes)
 * instead of the slot's seg: the slot's per-packet arrays still describe the
 * bundle (off relative to host_seg).  srtp_dispatch_transform_host does this
 * by itself for every chunk of a shard whose packets lie back to back in a
 * registered segment, so a one-shard dispatcher moves a registered bundle
 * with no host copy at all.
 *
 * srtp_pipeline_submit_gather is the form for packets scattered over
 * registered memory (a shard's share of an interleaved bundle): the slot's
 * arrays lay the bundle out in the slot (off, cap, ...), and packet j's region
 * (cap[j] rounded to 16 bytes) is read by the GPU from host_base + src_off[j]
 * over PCIe before the bundle runs, and written back there after it --
 * [host_base, host_base + host_bytes) must be registered; at most 32768
 * packets.  srtp_dispatch_transform_host / _submit_host use it for every
 * chunk of a registered bundle whose packets do not lie back to back, so a
 * many-shard dispatcher moves a registered bundle with no host copy of its
 * bytes either.  (Round 6; the registration maps the memory for the GPU.) */
int srtp_host_register(void *ptr, size_t bytes);
int srtp_host_unregister(void *ptr);
int srtp_host_alloc(size_t bytes, void **out);
int srtp_host_free(void *ptr);
int32_t srtp_host_is_registered(const void *ptr, size_t bytes);
int srtp_pipeline_submit_host(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                              int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                              int32_t abort_on_error, uint8_t *host_seg);
int srtp_pipeline_submit_gather(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                                int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                                int32_t abort_on_error, uint8_t *host_base, size_t host_bytes,
                                const uint32_t *src_off);

/* Bundle aggregator over the pipeline: per-packet submits
 * from any number of threads become bundles.  Replaces the reference's
 * one-packet-at-a-time calls through the transform chain
 * (RTPConnectorInputStream.java:425-452 receive, RTPConnectorOutputStream.java
 * :268-300,652-830 send; each a 1-element array through
 * SinglePacketTransformer.java:121-216).
 *
 * srtp_aggregator_submit copies one packet (len bytes; protect leaves 16
 * bytes of trailer room) into the open bundle of its direction; a bundle is
 * sealed when it holds max_packets packets or max_bytes bytes, when its oldest
 * packet has waited deadline_us, or on srtp_aggregator_flush.  Sealed bundles
 * run in sealing order; when one completes, `cb` is called (on the
 * aggregator's dispatch thread) once per packet, in bundle order, with the
 * packet's cookie, final status (SRTP_STATUS_*; -1 if the bundle could not be
 * submitted) and processed bytes, valid only during the call.  So packets
 * of one direction -- and thus of one transformer -- complete in the order
 * they were accepted (per submitting thread when several threads submit).
 * Every packet is its own 1-element array, as in the reference: one packet's
 * exception (SRTP_STATUS_ERR_MALFORMED) does not stop the others (the bundles
 * run without abort-on-throw whatever the engine's abort_on_error, so one
 * engine or dispatcher serves this and srtp_rawpacket_transform alike).  When
 * every slot is sealed or in flight, submit blocks (backpressure).  flush
 * seals the open bundles and waits until every packet accepted before it has
 * completed; destroy refuses new submits (SRTP_EINVAL, also from callbacks),
 * waits until every accepted packet has completed, then stops the threads.  Submits take no lock: each thread fills its own block of 16
 * entries of the open bundle (one compare-and-swap per block on the bundle,
 * one per packet on the thread's own block), so producers do not share a
 * written cache line per packet; entries of a block left unclaimed when the
 * bundle is sealed go to the engine as SRTP_PKT_FLAG_SKIP holes (counted as
 * SKIPPED in srtp_engine_stats, no callback).  Callbacks may submit (e.g.
 * forward a received packet); a submit made from a callback never blocks: when
 * no slot is free the packet is parked and placed in the first slot the
 * aggregator frees, ahead of other producers.  Producers outside callbacks
 * leave one slot of each lane (depth - 1 usable) for callback submits.  flush
 * from a callback returns SRTP_EINVAL and destroy from a callback does
 * nothing.  cb may be NULL for an aggregator that serves only synchronous
 * calls (srtp_aggregator_transform); srtp_aggregator_submit then returns
 * SRTP_EINVAL. */
typedef struct srtp_aggregator srtp_aggregator;
#define SRTP_AGG_SEAL_IDLE 0x1 /* seal a lane's open bundle at once while the lane has no
                                  bundle in flight (adaptive: bundles grow with the load) */
typedef struct {
    uint32_t max_packets; /* per bundle, default 1<<14 */
    size_t max_bytes;     /* per bundle (segment), default 24 MB */
    uint32_t deadline_us; /* default 1000 */
    int32_t depth;        /* pipeline slots (3..16), default 4 */
    uint32_t flags;       /* SRTP_AGG_*, default SRTP_AGG_SEAL_IDLE */
} srtp_aggregator_opts;
typedef void (*srtp_aggregator_cb)(void *user, uint64_t cookie, int32_t status, const uint8_t *data,
                                   uint32_t len);
int srtp_aggregator_opts_default(srtp_aggregator_opts *opts);
int srtp_aggregator_create(srtp_engine *e, const srtp_aggregator_opts *opts, srtp_aggregator_cb cb,
                           void *user, srtp_aggregator **out);
int srtp_aggregator_submit(srtp_aggregator *a, int32_t reverse, int32_t tid, const uint8_t *pkt,
                           uint32_t len, uint32_t flags, uint64_t cookie);
int srtp_aggregator_flush(srtp_aggregator *a);
int srtp_aggregator_stats(srtp_aggregator *a, uint64_t *accepted, uint64_t *completed,
                          uint64_t *bundles);
void srtp_aggregator_destroy(srtp_aggregator *a);
/* The synchronous per-packet call: SinglePacketTransformer.transform /
 * reverseTransform(RawPacket) (SinglePacketTransformer.java:113,169 as
 * SRTPTransformer.java:185-219 / SRTCPTransformer.java:175-207 implement
 * it) from any number of threads at once.  The packet -- copy_len bytes of
 * pkt (what lies behind its length, e.g. an extension header the reference
 * reads past it), RTP/RTCP length len, buffer room cap >= len (in-place
 * protect needs 16 bytes behind the packet) -- joins the lane's open bundle
 * like a submit, so concurrent callers share bundles; the call returns when
 * its bundle has completed, with the packet's final status, length and bytes
 * (max(len, *out_len) bytes to out, which holds at least cap bytes).  It
 * never calls the aggregator's callback.  With SRTP_AGG_SEAL_IDLE a call into
 * an idle lane is sealed at once, so a lone caller waits one GPU round trip
 * and concurrent callers coalesce behind the bundle in flight; deadline_us
 * bounds the wait for a seal otherwise.  Not from a callback (SRTP_EINVAL). */
int srtp_aggregator_transform(srtp_aggregator *a, int32_t reverse, int32_t tid, const uint8_t *pkt,
                              uint32_t copy_len, uint32_t len, uint32_t cap, uint32_t flags,
                              uint8_t *out, int32_t *status, uint32_t *out_len);
/* Transformer t's kind (read without a lock after the first call) and, when
 * fwd_rtcp_tag_len != NULL, its forward factory's SRTCP tag length
 * (srtp_transformer_info on the first shard). */
int srtp_aggregator_transformer_info(srtp_aggregator *a, int32_t t, int32_t *kind,
                                     int32_t *fwd_rtcp_tag_len);

/* Completion queues: the asynchronous per-packet call.  The
 * reference's connectors already queue: RTPConnectorOutputStream.write hands
 * packets to a send thread that drains them (RTPConnectorOutputStream.java
 * :652-830, runInSendThread :775), and the receive thread hands on every
 * datagram (RTPConnectorInputStream.java:425-452,780-806).  Such a thread owns
 * a queue, submits every packet it has and reaps the results, so it keeps
 * many packets in flight instead of one.
 *
 * srtp_queue_submit: one packet as srtp_aggregator_transform takes it
 * (copy_len bytes of pkt, length len, room cap >= copy_len) joins its lane's
 * open bundle (the aggregator's sealing rules apply); cookie is the caller's.
 * A packet with SRTP_PKT_FLAG_SKIP, or with len > cap (RawPacket.isInvalid),
 * completes at once with SRTP_STATUS_SKIPPED / SRTP_STATUS_DROP_INVALID and
 * no bytes.  Returns SRTP_EAGAIN when max_inflight packets are outstanding;
 * when no slot is free it waits for one, but only until the queue's oldest
 * outstanding packet has completed (then SRTP_EAGAIN: the caller reaps and
 * submits again), or at once when the last reap's completions are still
 * held (not released).
 *
 * srtp_queue_reap: up to max completions, in SUBMISSION order (so per
 * transformer and SSRC the reference's order), into out; with wait != 0 it
 * blocks until at least one is there when any packet is outstanding.
 * Returns the count.  out[i].data points at the packet's processed bytes in
 * the aggregator's pinned slot (max(len, in_len) bytes, within cap; NULL for
 * packets completed at submit) and stays valid until the next reap or
 * destroy of this queue (or srtp_queue_release): reaping releases the
 * previous reap's packets, and a slot is reused only when every packet of it
 * has been released -- so a caller done with its completions releases them
 * (srtp_queue_release) rather than holding slots until its next reap.
 *
 * A queue belongs to one thread at a time (submit and reap are not
 * thread-safe on one queue); queues of one aggregator are independent.
 * Packets of one direction and lane still run in the order the aggregator
 * accepted them across all its producers.  srtp_queue_destroy waits for the
 * queue's outstanding packets; every queue must be destroyed before its
 * aggregator (srtp_aggregator_destroy waits for that).  Not from an
 * aggregator callback (SRTP_EINVAL). */
typedef struct srtp_queue srtp_queue;
typedef struct {
    uint64_t cookie;     /* as submitted */
    int32_t status;      /* SRTP_STATUS_* (-1: the bundle could not be submitted) */
    uint32_t len;        /* the packet's length after the call */
    uint32_t in_len;     /* its length at submit */
    int32_t reverse;     /* as submitted */
    int32_t tid;         /* as submitted */
    const uint8_t *data; /* processed bytes (see above) */
} srtp_completion;
int srtp_queue_create(srtp_aggregator *a, uint32_t max_inflight, srtp_queue **out);
int srtp_queue_submit(srtp_queue *q, int32_t reverse, int32_t tid, const uint8_t *pkt, uint32_t copy_len,
                      uint32_t len, uint32_t cap, uint32_t flags, uint64_t cookie);
int srtp_queue_reap(srtp_queue *q, srtp_completion *out, uint32_t max, int32_t wait);
/* Releases the last reap's completions (their data pointers become invalid). */
void srtp_queue_release(srtp_queue *q);
/* packets submitted and not yet reaped */
int32_t srtp_queue_outstanding(srtp_queue *q);
srtp_aggregator *srtp_queue_aggregator(srtp_queue *q);
void srtp_queue_destroy(srtp_queue *q);

/* In-process multi-GPU dispatcher (SURVEY.md 8b engine_create(devices, opts),
 * 8e): one engine per shard, shard i on device devices[i] (a device may host
 * several shards).  A host bundle is split by shard = srtp_shard_of(SSRC)
 * (RTP: RawPacket.getSSRC, RTCP: getRTCPSSRC) -- SRTP contexts are per
 * (transformer, SSRC), SRTPTransformer.java:62,152-175, so each GPU owns its
 * SSRCs' state and nothing crosses GPUs.  Every shard's sub-bundle keeps
 * bundle order; statuses, lengths and packet bytes are scattered back in
 * place.  Results are identical to one engine processing the whole bundle,
 * including SinglePacketTransformer's abort-on-throw
 * (SinglePacketTransformer.java:134-155,190-210), which the dispatcher
 * reproduces across shards by rolling back a throwing transformer's later
 * packets and the contexts they touched (see dispatch.cpp): a bundle costs at
 * most two runs per shard however many of its packets throw.  Factories and
 * transformers are created on every shard with the same ids as one engine
 * would assign.  srtp_dispatch_plan is the host-only split (no GPU needed):
 * per packet its shard (-1: handled without an engine) and whether it could
 * throw (may_throw, only with abort_on_error); it returns 2 if some packet
 * could throw (the bundle needs context snapshots), else 1.  kinds[t] =
 * transformer t's kind, tag_mask bit T = some policy has tag length T. */
typedef struct srtp_dispatch srtp_dispatch;
int32_t srtp_shard_of(uint32_t ssrc, int32_t n_shards);
int32_t srtp_dispatch_plan(int32_t n_shards, int32_t abort_on_error, int32_t reverse,
                           const int32_t *kinds, int32_t n_transformers, uint32_t tag_mask,
                           const int32_t *tids, int32_t tid, const uint8_t *seg, size_t seg_bytes,
                           const uint32_t *off, const uint32_t *len, const uint32_t *cap,
                           const uint32_t *flags, uint32_t n, int32_t *shard, int32_t *may_throw);
int srtp_dispatch_create(const int32_t *devices, int32_t n_shards, const srtp_engine_opts *opts,
                         srtp_dispatch **out);
void srtp_dispatch_destroy(srtp_dispatch *d);
const char *srtp_dispatch_last_error(srtp_dispatch *d);
int32_t srtp_dispatch_num_shards(srtp_dispatch *d);
srtp_engine *srtp_dispatch_engine(srtp_dispatch *d, int32_t shard);
int srtp_dispatch_factory_create(srtp_dispatch *d, int32_t sender, const uint8_t *master_key,
                                 int32_t key_len, const uint8_t *master_salt, int32_t salt_len,
                                 const srtp_policy *srtp, const srtp_policy *srtcp, int32_t *out);
int srtp_dispatch_factory_close(srtp_dispatch *d, int32_t factory);
int srtp_dispatch_transformer_create(srtp_dispatch *d, int32_t kind, int32_t fwd, int32_t rev,
                                     int32_t *out);
int srtp_dispatch_transformer_set_factory(srtp_dispatch *d, int32_t transformer, int32_t factory,
                                          int32_t forward);
int srtp_dispatch_transformer_close(srtp_dispatch *d, int32_t transformer);
int srtp_dispatch_transform_host(srtp_dispatch *d, int32_t reverse, const int32_t *tids, int32_t tid,
                                 uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                                 const uint32_t *cap, const uint32_t *flags, int32_t *status,
                                 uint32_t n);
/* Asynchronous host bundles (no reference API: RTPConnectorOutputStream's
 * send thread, RTPConnectorOutputStream.java:268-300, hands each packet on
 * and goes back to its queue).  srtp_dispatch_submit_host does the work of
 * srtp_dispatch_transform_host but returns once the bundle's last chunks are
 * on their way to the GPUs, with a ticket; srtp_dispatch_wait_host(ticket)
 * returns when its statuses, lengths and bytes are in the caller's arrays,
 * with the bundle's result.  The arrays must stay valid, and untouched by the
 * caller, until that wait returns.  The next submit overlaps its packing and
 * H2D with the previous bundle's last D2H.  Bundles run in submission order
 * on every shard (each context sees its packets in that order, as from
 * synchronous calls), and a synchronous call is ordered with them too.  Every
 * ticket must be waited for (at most 64 may be outstanding: SRTP_EAGAIN
 * beyond); waiting for one also completes -- but does not consume -- the
 * bundles submitted before it.  A bundle with a packet that could throw under
 * abort-on-throw (the rollback above) runs to completion inside its submit.
 * srtp_dispatch_destroy completes bundles never waited for. */
int srtp_dispatch_submit_host(srtp_dispatch *d, int32_t reverse, const int32_t *tids, int32_t tid,
                              uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                              const uint32_t *cap, const uint32_t *flags, int32_t *status, uint32_t n,
                              uint64_t *ticket);
int srtp_dispatch_wait_host(srtp_dispatch *d, uint64_t ticket);
int srtp_dispatch_get_context_state(srtp_dispatch *d, int32_t transformer, uint32_t ssrc,
                                    srtp_ctx_state *out);
int srtp_dispatch_set_context_state(srtp_dispatch *d, int32_t transformer, uint32_t ssrc,
                                    int32_t forward, const srtp_ctx_state *st);
/* srtp_stats summed over the shards */
int srtp_dispatch_stats(srtp_dispatch *d, srtp_stats *out);
/* Host time of srtp_dispatch_transform_host since creation, in ns: [0] plan
 * and split, [1] packing into the shards' pinned slots and enqueueing each
 * chunk's copies and kernels, [2] waiting for the
 * shards' bundles (H2D + kernels + D2H), [3] scattering results back (1-3
 * summed over the shards' worker threads), [4] wall time of the calls, [5]
 * number of calls. */
int srtp_dispatch_host_times(srtp_dispatch *d, uint64_t ns[6]);
/* The shard a packet of transformer `tid` goes to (as srtp_dispatch_transform_host
 * routes it: its SSRC's shard, shard 0 for a packet shorter than 12 bytes);
 * -1 for an unknown transformer.  Does not wait for bundles in flight. */
int32_t srtp_dispatch_route(srtp_dispatch *d, int32_t tid, const uint8_t *pkt, uint32_t len);
/* 1 when the reference could throw on this packet of a transformer of `kind`
 * (SRTP_KIND_*) -- the per-packet test of srtp_dispatch_plan, a superset of the
 * engine's SRTP_STATUS_ERR_MALFORMED: RawPacket.getHeaderLength,
 * SRTPCipherCTR.process / SRTPCipherF8.process bounds, RawPacket.getSRTCPIndex
 * -- for policies whose tag lengths are in tag_mask (bit T: tag length T, bit
 * 0: NULL authentication); pkt holds cap bytes (a smaller cap only widens the
 * superset: the header may then seem to end past it).  0 for a
 * packet that is skipped or invalid (len < 12 or len > cap).  Host only. */
int32_t srtp_packet_may_throw(int32_t kind, int32_t reverse, const uint8_t *pkt, uint32_t len, uint32_t cap,
                              uint32_t flags, uint32_t tag_mask);
/* The aggregator over a dispatcher: one lane per shard (its own pinned slots
 * and dispatch thread); each packet goes to the lane of its shard, so
 * per-packet submits from one process reach every GPU.  Callbacks of
 * different shards run concurrently on the lanes' threads; the packets of
 * one shard -- hence of one (transformer, SSRC) context -- and one direction
 * complete in the order they were accepted.  opts apply per lane; every
 * shard's engine must have abort_on_error = 0. */
int srtp_aggregator_create_dispatch(srtp_dispatch *d, const srtp_aggregator_opts *opts,
                                    srtp_aggregator_cb cb, void *user, srtp_aggregator **out);

/* RawPacket[] marshalling for the Java drop-in (the JNI shim
 * src/native/srtp_mi355x/ calls exactly this).  PacketTransformer.transform /
 * reverseTransform(RawPacket[]) as SinglePacketTransformer.java:121-216 runs
 * it: element i is bufs[i] (NULL: a null element, skipped) with the RawPacket's
 * buffer length, offset, length and flags (SRTP_PKT_FLAG_SKIP: the packet
 * predicate rejected it; FLAG_DISCARD / FLAG_SILENCE as RawPacket.getFlags).
 * Packs the elements into a bundle of transformer tids[i] (tids == NULL: tid),
 * runs it, and writes each result back into its buffer in place, as the
 * reference leaves it: status[i] (drops: the caller replaces the element with
 * null; the RawPacket keeps what was done to it -- e.g. the shrink of a failed
 * tag check), length[i] updated.  need_len[i] != 0 where the reference
 * allocates a new buffer -- RawPacket.append without room after the payload
 * (RawPacket.java:203-220), and RawPacket.grow for every SRTCP protect
 * (:885-893): the caller allocates need_len[i] bytes, copies the result from
 * srtp_rawpacket_result to offset 0, and sets buffer / offset 0 / length.
 * *thrown = the first element the reference throws on (SRTP_STATUS_ERR_MALFORMED;
 * -1: none): every element was written back, the thrower keeps its partial
 * mutation, its transformer's later packets are NOT_PROCESSED and untouched,
 * and the caller rethrows.  A batch is the staging of one calling thread
 * (pinned memory for an engine); results stay valid until its next call. */
typedef struct srtp_rawpacket_batch srtp_rawpacket_batch;
int srtp_rawpacket_batch_create(srtp_engine *e, srtp_rawpacket_batch **out);
int srtp_rawpacket_batch_create_dispatch(srtp_dispatch *d, srtp_rawpacket_batch **out);
void srtp_rawpacket_batch_destroy(srtp_rawpacket_batch *b);
int srtp_rawpacket_transform(srtp_rawpacket_batch *b, int32_t reverse, const int32_t *tids, int32_t tid,
                             uint8_t *const *bufs, const uint32_t *buf_len, const uint32_t *offset,
                             uint32_t *length, const uint32_t *flags, int32_t *status,
                             uint32_t *need_len, uint32_t n, int32_t *thrown);
int srtp_rawpacket_result(srtp_rawpacket_batch *b, uint32_t i, const uint8_t **data, uint32_t *len);
/* Arrays of up to 8192 packets none of which can throw (srtp_packet_may_throw)
 * then go through a completion queue on aggregator a -- whose lanes must be
 * over the batch's engine or dispatcher -- instead of a bundle of their own:
 * concurrent callers' arrays share bundles, and no caller waits behind
 * another's GPU round trip.  The results are the same (no packet can throw, so
 * abort-on-throw has nothing to stop); other arrays keep the batch's own
 * bundle.  The queue lives for one srtp_rawpacket_transform call, so a batch
 * holds nothing on the aggregator between calls (srtp_aggregator_destroy
 * waits only for calls in progress).  If the call fails part-way, the elements
 * that did not complete get SRTP_STATUS_ERR_INTERNAL and are left untouched.
 * a = NULL turns this off. */
int srtp_rawpacket_batch_set_aggregator(srtp_rawpacket_batch *b, srtp_aggregator *a);
/* One RawPacket through SinglePacketTransformer.transform / reverseTransform
 * (RawPacket) (SinglePacketTransformer.java:113,169; every
 * RTPConnector*Stream call and DtlsPacketTransformer.transformSrtp,
 * DtlsPacketTransformer.java:1544-1564, hands the transformer one packet at
 * a time), coalesced with concurrent callers' packets through the aggregator
 * (srtp_aggregator_transform).  The element marshalling and write-back are
 * srtp_rawpacket_transform's for an array of one: buf (NULL: a null element)
 * of buf_len bytes holds the packet at offset with *length bytes; *status,
 * *length and the bytes in buf are updated in place; *need_len != 0 where the
 * reference reallocates (RawPacket.append / grow), the result then being the
 * first *need_len bytes of grow, which must hold grow_cap >= *length + 16
 * bytes and at least the bytes from offset to the end of buf (min 65535).
 * SRTP_STATUS_ERR_MALFORMED: the reference throws (the packet keeps its
 * partial mutation); the caller rethrows. */
int srtp_rawpacket_transform_one(srtp_aggregator *a, int32_t reverse, int32_t tid, uint8_t *buf,
                                 uint32_t buf_len, uint32_t offset, uint32_t *length, uint32_t flags,
                                 int32_t *status, uint32_t *need_len, uint8_t *grow, uint32_t grow_cap);
/* The per-packet call, asynchronous (a connector's send thread
 * or receive loop keeping many packets in flight): one RawPacket element as
 * srtp_rawpacket_transform_one takes it (buf NULL or flags with
 * SRTP_PKT_FLAG_SKIP: SKIPPED; *length past the buffer: DROP_INVALID, both
 * completed at once) submitted to queue q (srtp_queue_submit; SRTP_EAGAIN:
 * reap first).  Each completion reaped from q then goes back into its
 * RawPacket by srtp_rawpacket_complete, given the buffer's bytes after the
 * packet's offset (avail): *need_len == 0: *copy_len bytes of c->data go back
 * in place at the offset; else the reference allocates a new buffer of
 * *need_len bytes (RawPacket.append / grow) at offset 0 that receives
 * *copy_len bytes of c->data.  Either way the RawPacket's length becomes
 * c->len; SRTP_STATUS_ERR_MALFORMED is the reference's throw (the packet keeps
 * its partial mutation), other non-OK statuses its null. */
int srtp_rawpacket_submit(srtp_queue *q, int32_t reverse, int32_t tid, const uint8_t *buf, uint32_t buf_len,
                          uint32_t offset, uint32_t length, uint32_t flags, uint64_t cookie);
int srtp_rawpacket_complete(srtp_queue *q, const srtp_completion *c, uint32_t avail, uint32_t *copy_len,
                            uint32_t *need_len);
/* Devices the engine can use (hipGetDeviceCount; 0 without a GPU): what the
 * Java drop-in sizes its dispatcher with. */
int32_t srtp_device_count(void);

/* Control-plane crypto without a GPU (used by CPU-side tests): RFC 3711 4.3
 * session keys exactly as SRTPCryptoContext.deriveSrtpKeys (rtcp = 0) /
 * SRTCPCryptoContext.deriveSrtcpKeys (rtcp = 1). */
int srtp_derive_session_keys(const uint8_t master_key[16], const uint8_t master_salt[14],
                             int32_t rtcp, uint8_t enc_key[16], uint8_t auth_key[20],
                             uint8_t salt_key[14]);
/* The same for a 16- or 32-byte master key (AES-128 / AES-256 PRF, RFC 6188
 * 4.1): enc_key receives key_len bytes. */
int srtp_derive_session_keys_n(const uint8_t *master_key, int32_t key_len,
                               const uint8_t master_salt[14], int32_t rtcp, uint8_t *enc_key,
                               uint8_t auth_key[20], uint8_t salt_key[14]);
/* The same with the policy's cipher as the PRF: AES for SRTP_AESCM / AESF8 /
 * NULL, Twofish for SRTP_TWOFISH(F8)_ENCRYPTION (BaseSRTPCryptoContext.java
 * :197-226 keys that cipher with the master key). */
int srtp_derive_session_keys_for(int32_t enc_type, const uint8_t *master_key, int32_t key_len,
                                 const uint8_t master_salt[14], int32_t rtcp, uint8_t *enc_key,
                                 uint8_t auth_key[20], uint8_t salt_key[14]);
/* The same with an auth key of auth_len bytes (1..64; 32 for ZRTP's Skein
 * policies, whose authKeyLength is 32: ZRTPTransformEngine.java:867-872). */
int srtp_derive_session_keys_auth(int32_t enc_type, const uint8_t *master_key, int32_t key_len,
                                  const uint8_t master_salt[14], int32_t rtcp, uint8_t *enc_key,
                                  uint8_t *auth_key, int32_t auth_len, uint8_t salt_key[14]);
/* Skein-512 (version 1.3) keyed with key[0..key_len) (key_len 0: the plain
 * hash), out_bits (1..512) output bits: the tag bccontrib's SkeinMac computes
 * for SRTPPolicy.SKEIN_AUTHENTICATION (BaseSRTPCryptoContext.java:244-248). */
int srtp_skein512_mac(const uint8_t *key, int32_t key_len, int32_t out_bits, const uint8_t *msg,
                      size_t n, uint8_t *out);
/* One block of the policy's cipher: AES-128/256 (key_len 16 / 32) or Twofish
 * (enc_type SRTP_TWOFISH*, key_len 16 / 24 / 32). */
int srtp_block_encrypt(int32_t enc_type, const uint8_t *key, int32_t key_len, const uint8_t in[16],
                       uint8_t out[16]);

/* DTLS-SRTP keying (control plane, host only): what
 * DtlsPacketTransformer.initializeSRTPTransformer does after the handshake
 * (transform/dtls/DtlsPacketTransformer.java:549-690).
 *
 * srtp_tls_export_keying_material is the RFC 5705 exporter the reference calls
 * through BouncyCastle's TlsContext.exportKeyingMaterial(ExporterLabel.dtls_srtp,
 * null, n) (:614-617): PRF(master_secret, label, client_random ||
 * server_random)[0..out_len) with no context value.  prf selects the TLS PRF
 * of the negotiated version: SRTP_TLS_PRF_TLS10 (DTLS 1.0, RFC 2246 5: P_MD5 xor
 * P_SHA1 over the secret's halves -- the version the reference offers,
 * TlsClientImpl.java:148-155) or SRTP_TLS_PRF_SHA256 (DTLS 1.2, RFC 5246 5).
 * The label for DTLS-SRTP is SRTP_DTLS_EXPORTER_LABEL.
 *
 * srtp_dtls_profile_keys fills the policies of a negotiated protection profile
 * (:574-612; the _32 profiles keep a 10-byte SRTCP tag) and splits
 * keying_material_len = 2 * (key + salt) bytes of exported material as client
 * key | server key | client salt | server salt (:618-638).  km == NULL fills
 * only the lengths and policies.  Unknown profile: SRTP_EPOLICY (the
 * reference's IllegalArgumentException).
 *
 * srtp_dtls_transformer_create builds both factories (the client's is a sender
 * iff is_client, the server's iff !is_client: :639-652) and a transformer of
 * `kind` whose forward factory is this side's own and reverse the peer's
 * (:653-690).  NULL-cipher profiles, which export no master key (the
 * reference then fails deriving session keys), return
 * SRTP_EPOLICY.  out_factories (may be NULL) receives {client, server} factory ids
 * -- the caller closes them with the transformer, as
 * SRTPTransformer.close() closes both (SRTPTransformer.java:132-150). */
#define SRTP_PROFILE_AES128_CM_HMAC_SHA1_80 0x0001
#define SRTP_PROFILE_AES128_CM_HMAC_SHA1_32 0x0002
#define SRTP_PROFILE_NULL_HMAC_SHA1_80 0x0005
#define SRTP_PROFILE_NULL_HMAC_SHA1_32 0x0006
#define SRTP_TLS_PRF_TLS10 0
#define SRTP_TLS_PRF_SHA256 1
#define SRTP_DTLS_EXPORTER_LABEL "EXTRACTOR-dtls_srtp"
typedef struct {
    srtp_policy srtp, srtcp;
    int32_t key_len, salt_len, keying_material_len;
    uint8_t client_key[16], server_key[16];
    uint8_t client_salt[14], server_salt[14];
} srtp_dtls_keys;
int srtp_tls_export_keying_material(int32_t prf, const uint8_t *master_secret, int32_t secret_len,
                                    const uint8_t client_random[32], const uint8_t server_random[32],
                                    const char *label, uint8_t *out, int32_t out_len);
int srtp_dtls_profile_keys(int32_t profile, const uint8_t *km, int32_t km_len, srtp_dtls_keys *out);
int srtp_dtls_transformer_create(srtp_engine *e, int32_t profile, int32_t is_client, int32_t kind,
                                 const uint8_t *km, int32_t km_len, int32_t *out_transformer,
                                 int32_t out_factories[2]);

#ifdef __cplusplus
}
#endif
#endif
