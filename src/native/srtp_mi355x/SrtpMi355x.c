/*
 * SrtpMi355x.c -- JNI shim between libjitsi's Java transformers and the
 * MI355X SRTP engine (include/srtp_mi355x.h, libsrtp_mi355x.so).
 *
 * Built like libjnopenssl next to src/native/openssl/ (INTEGRATION.md 2):
 *
 *   gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       src/native/srtp_mi355x/SrtpMi355x.c -Llibjitsi_amd -lsrtp_mi355x -o libjnsrtp_mi355x.so
 *
 * The image has no JDK, so here it is compiled unmodified against a stub JNI
 * header and driven through a toy JVM (tests/jni_stub/, tests/test_jni_shim.py).
 *
 * Everything below the JNI calls is srtp_* C ABI that the GPU tests exercise
 * (the RawPacket[] marshalling is srtp_rawpacket_transform, tested through
 * ctypes in tests/test_rawpacket.py).  Conventions of src/native/openssl:
 * native handles are jlong casts of heap pointers (BlockCipher.c:64-73),
 * errors come back as negative return codes that the Java side turns into a
 * RuntimeException (OpenSSLBlockCipher.java:310-313).  Unlike BlockCipher.c,
 * whose critical regions span a CPU call, packet bytes are copied in and out
 * with Get/SetByteArrayRegion: a GPU round trip must not stall the JVM's GC.
 *
 * Java side: org.jitsi.impl.neomedia.transform.srtp.mi355x.SrtpMi355x (the
 * native declarations), GpuSRTPTransformer / GpuSRTCPTransformer (the
 * SinglePacketTransformer drop-ins), GpuSRTPContextFactory.
 */
#include <jni.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "srtp_mi355x.h"

#define JFN(name) Java_org_jitsi_impl_neomedia_transform_srtp_mi355x_SrtpMi355x_##name
#define H(x) ((void *)(intptr_t)(x))

/* ---- engine / dispatcher (one per process: every GPU of the node) ---- */

JNIEXPORT jlong JNICALL JFN(dispatchCreate)(JNIEnv *env, jclass c, jintArray devices, jboolean checkReplay,
                                            jint maxContexts) {
    srtp_engine_opts o;
    srtp_engine_opts_default(&o);
    o.check_replay = checkReplay ? 1 : 0;
    if (maxContexts > 0) o.max_contexts = (uint32_t)maxContexts;
    jsize n = (*env)->GetArrayLength(env, devices);
    jint dev[256];
    if (n < 1 || n > 256) return 0;
    (*env)->GetIntArrayRegion(env, devices, 0, n, dev);
    srtp_dispatch *d = NULL;
    return srtp_dispatch_create((const int32_t *)dev, n, &o, &d) == SRTP_OK ? (jlong)(intptr_t)d : 0;
}

JNIEXPORT void JNICALL JFN(dispatchDestroy)(JNIEnv *env, jclass c, jlong d) {
    srtp_dispatch_destroy((srtp_dispatch *)H(d));
}

/* SRTPContextFactory(sender, masterKey, masterSalt, srtpPolicy, srtcpPolicy):
 * policies as int[6] {encType, encKeyLength, authType, authKeyLength,
 * authTagLength, saltKeyLength} (SRTPPolicy.java:107-120). */
JNIEXPORT jint JNICALL JFN(factoryCreate)(JNIEnv *env, jclass c, jlong d, jboolean sender, jbyteArray key,
                                          jbyteArray salt, jintArray srtpPol, jintArray srtcpPol) {
    jint p1[6], p2[6];
    int32_t id = -1;
    (*env)->GetIntArrayRegion(env, srtpPol, 0, 6, p1);
    (*env)->GetIntArrayRegion(env, srtcpPol, 0, 6, p2);
    jsize kl = (*env)->GetArrayLength(env, key), sl = (*env)->GetArrayLength(env, salt);
    jbyte k[64], s[64];
    if (kl > 64 || sl > 64) return SRTP_EINVAL;
    (*env)->GetByteArrayRegion(env, key, 0, kl, k);
    (*env)->GetByteArrayRegion(env, salt, 0, sl, s);
    /* copies the session keys to every GPU: no array is held meanwhile */
    int rc = srtp_dispatch_factory_create((srtp_dispatch *)H(d), sender, (const uint8_t *)k, kl,
                                          (const uint8_t *)s, sl, (const srtp_policy *)p1,
                                          (const srtp_policy *)p2, &id);
    memset(k, 0, sizeof k); /* the master key does not stay on the stack */
    memset(s, 0, sizeof s);
    return rc == SRTP_OK ? id : rc;
}

JNIEXPORT jint JNICALL JFN(factoryClose)(JNIEnv *env, jclass c, jlong d, jint f) {
    return srtp_dispatch_factory_close((srtp_dispatch *)H(d), f);
}

JNIEXPORT jint JNICALL JFN(transformerCreate)(JNIEnv *env, jclass c, jlong d, jint kind, jint fwd, jint rev) {
    int32_t id = -1;
    int rc = srtp_dispatch_transformer_create((srtp_dispatch *)H(d), kind, fwd, rev, &id);
    return rc == SRTP_OK ? id : rc;
}

/* SRTPTransformer.setContextFactory / SRTCPTransformer.updateFactory */
JNIEXPORT jint JNICALL JFN(transformerSetFactory)(JNIEnv *env, jclass c, jlong d, jint t, jint f,
                                                  jboolean forward) {
    return srtp_dispatch_transformer_set_factory((srtp_dispatch *)H(d), t, f, forward ? 1 : 0);
}

JNIEXPORT jint JNICALL JFN(transformerClose)(JNIEnv *env, jclass c, jlong d, jint t) {
    return srtp_dispatch_transformer_close((srtp_dispatch *)H(d), t);
}

/* ---- RawPacket[] (PacketTransformer.transform / reverseTransform) ---- */

/* One srtp_rawpacket_batch per Java thread, owned here: created on the
 * thread's first array call and destroyed when the thread exits (a pthread key
 * destructor), so a media thread that dies does not leak its pinned staging.
 * Arrays that cannot throw go through the aggregator's lanes
 * (srtp_rawpacket_batch_set_aggregator); the others run as one bundle. */
struct tl_batch {
    srtp_rawpacket_batch *b;
    jlong d, agg;
};
static pthread_key_t batch_key;
static pthread_once_t batch_once = PTHREAD_ONCE_INIT;

static void batch_free(void *p) {
    struct tl_batch *t = p;
    srtp_rawpacket_batch_destroy(t->b);
    free(t);
}
static void batch_key_init(void) { pthread_key_create(&batch_key, batch_free); }

static srtp_rawpacket_batch *thread_batch(jlong d, jlong agg) {
    pthread_once(&batch_once, batch_key_init);
    struct tl_batch *t = pthread_getspecific(batch_key);
    if (t && t->d == d && t->agg == agg) return t->b;
    if (t) { /* another dispatcher (a test's second JVM): start over */
        pthread_setspecific(batch_key, NULL);
        batch_free(t);
    }
    t = calloc(1, sizeof *t);
    if (!t) return NULL;
    if (srtp_rawpacket_batch_create_dispatch((srtp_dispatch *)H(d), &t->b) != SRTP_OK) {
        free(t);
        return NULL;
    }
    srtp_rawpacket_batch_set_aggregator(t->b, (srtp_aggregator *)H(agg));
    t->d = d;
    t->agg = agg;
    pthread_setspecific(batch_key, t);
    return t->b;
}

static jfieldID fid_buffer, fid_offset, fid_length, fid_flags;

static int raw_packet_ids(JNIEnv *env) {
    if (fid_flags) return 0;
    jclass rp = (*env)->FindClass(env, "org/jitsi/impl/neomedia/RawPacket");
    if (!rp) return -1;
    /* RawPacket.java:53-73 */
    fid_buffer = (*env)->GetFieldID(env, rp, "buffer", "[B");
    fid_offset = (*env)->GetFieldID(env, rp, "offset", "I");
    fid_length = (*env)->GetFieldID(env, rp, "length", "I");
    fid_flags = (*env)->GetFieldID(env, rp, "flags", "I");
    return fid_buffer && fid_offset && fid_length && fid_flags ? 0 : -1;
}

/* transform (reverse = false) / reverseTransform (reverse = true) of pkts in
 * place, as SinglePacketTransformer.java:121-216 does per element: skip[i]
 * != 0 where the packet predicate rejected element i.  Dropped elements are
 * set to null, packets that the reference gives a new buffer
 * (RawPacket.append / grow) get one.  Returns 0, 1 + the index of the first
 * element the reference throws on (the Java side rethrows after this
 * returns: every element is written back), or a negative SRTP_E* code.
 *
 * No array stays pinned across the GPU round trip: each element's bytes from
 * its offset on are copied out with GetByteArrayRegion into one native block,
 * srtp_rawpacket_transform runs on that block, and the bytes it may have
 * changed go back with SetByteArrayRegion (BlockCipher.c:194-229 likewise
 * holds its critical region only around a CPU call).  Two elements sharing one
 * byte[] stay consistent: each writes back only its own range. */
JNIEXPORT jint JNICALL JFN(transformPackets)(JNIEnv *env, jclass c, jlong d, jlong agg, jboolean reverse,
                                             jint tid, jobjectArray pkts, jintArray skip) {
    if (!pkts || raw_packet_ids(env) != 0) return SRTP_EINVAL;
    srtp_rawpacket_batch *b = thread_batch(d, agg);
    if (!b) return SRTP_ENOMEM;
    const jsize n = (*env)->GetArrayLength(env, pkts);
    if (n == 0) return 0;
    if ((*env)->PushLocalFrame(env, 2 * n + 16) != 0) return SRTP_ENOMEM;
    jobject *objs = calloc((size_t)n, sizeof *objs);
    jbyteArray *arrs = calloc((size_t)n, sizeof *arrs);
    uint8_t **bufs = calloc((size_t)n, sizeof *bufs);
    uint32_t *u = calloc((size_t)n * 6, sizeof *u); /* buf_len, offset, length, flags, need_len, java offset */
    int32_t *status = calloc((size_t)n, sizeof *status);
    uint8_t *block = NULL;
    jint *sk = skip ? (*env)->GetIntArrayElements(env, skip, NULL) : NULL;
    int rc = SRTP_ENOMEM;
    if (!objs || !arrs || !bufs || !u || !status) goto out;
    uint32_t *buf_len = u, *offset = u + n, *length = u + 2 * n, *flags = u + 3 * n, *need = u + 4 * n,
             *joff = u + 5 * n;
    size_t total = 0;
    for (jsize i = 0; i < n; i++) {
        objs[i] = (*env)->GetObjectArrayElement(env, pkts, i);
        if (!objs[i]) continue;
        arrs[i] = (jbyteArray)(*env)->GetObjectField(env, objs[i], fid_buffer);
        const uint32_t al = arrs[i] ? (uint32_t)(*env)->GetArrayLength(env, arrs[i]) : 0u;
        const jint jo = (*env)->GetIntField(env, objs[i], fid_offset);
        joff[i] = jo < 0 ? UINT32_MAX : (uint32_t)jo; /* a negative offset holds nothing */
        length[i] = (uint32_t)(*env)->GetIntField(env, objs[i], fid_length);
        flags[i] = (uint32_t)(*env)->GetIntField(env, objs[i], fid_flags) &
                   (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE);
        if (sk && sk[i]) flags[i] |= SRTP_PKT_FLAG_SKIP;
        /* the native copy holds the buffer from the packet's offset on (what
         * the reference may read: the packet and the bytes behind it) */
        buf_len[i] = joff[i] <= al ? al - joff[i] : 0u;
        offset[i] = 0;
        total += buf_len[i];
    }
    block = malloc(total ? total : 1);
    if (!block) goto out;
    total = 0;
    for (jsize i = 0; i < n; i++) {
        if (!arrs[i]) continue;
        bufs[i] = block + total;
        /* an offset outside the buffer holds nothing: no region call (it would
         * throw), the engine reports the packet invalid */
        if (buf_len[i]) (*env)->GetByteArrayRegion(env, arrs[i], (jsize)joff[i], (jsize)buf_len[i], (jbyte *)bufs[i]);
        total += buf_len[i];
    }
    int32_t thrown = -1;
    uint32_t *old_len = calloc((size_t)n, sizeof *old_len);
    if (!old_len) goto out;
    for (jsize i = 0; i < n; i++) old_len[i] = length[i];
    rc = srtp_rawpacket_transform(b, reverse ? 1 : 0, NULL, tid, bufs, buf_len, offset, length, flags, status,
                                  need, (uint32_t)n, &thrown);
    if (rc != SRTP_OK) {
        free(old_len);
        goto out;
    }
    for (jsize i = 0; i < n; i++) {
        const int32_t st = status[i];
        if (!objs[i] || st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED) continue;
        if (need[i]) { /* RawPacket.append / grow: a new byte[] at offset 0 */
            const uint8_t *data;
            uint32_t dl;
            jbyteArray nb = (*env)->NewByteArray(env, (jsize)need[i]);
            if (!nb || srtp_rawpacket_result(b, (uint32_t)i, &data, &dl) != SRTP_OK) {
                rc = SRTP_ENOMEM;
                free(old_len);
                goto out;
            }
            (*env)->SetByteArrayRegion(env, nb, 0, (jsize)dl, (const jbyte *)data);
            (*env)->SetObjectField(env, objs[i], fid_buffer, nb);
            (*env)->SetIntField(env, objs[i], fid_offset, 0);
        } else if (arrs[i]) { /* in place: the bytes up to the longer of the two lengths */
            uint32_t w = old_len[i] > length[i] ? old_len[i] : length[i];
            if (w > buf_len[i]) w = buf_len[i];
            if (w) (*env)->SetByteArrayRegion(env, arrs[i], (jsize)joff[i], (jsize)w, (const jbyte *)bufs[i]);
        }
        (*env)->SetIntField(env, objs[i], fid_length, (jint)length[i]);
        if (st != SRTP_STATUS_OK && st != SRTP_STATUS_ERR_MALFORMED)
            (*env)->SetObjectArrayElement(env, pkts, i, NULL); /* the reference returned null */
    }
    free(old_len);
    rc = thrown >= 0 ? thrown + 1 : 0;
out:
    if (sk) (*env)->ReleaseIntArrayElements(env, skip, sk, JNI_ABORT);
    free(block);
    free(objs);
    free(arrs);
    free(bufs);
    free(u);
    free(status);
    (*env)->PopLocalFrame(env, NULL);
    return rc;
}

/* ---- the per-packet path (SinglePacketTransformer.transform(RawPacket)) ---- */

JNIEXPORT jint JNICALL JFN(deviceCount)(JNIEnv *env, jclass c) {
    return srtp_device_count();
}

/* One aggregator per process over the dispatcher: its lanes coalesce the
 * per-packet calls of every JVM thread into GPU bundles.  Each lane (one per
 * GPU) holds `depth` pinned slots of bundles of up to maxPackets packets /
 * maxMegabytes of packet bytes, pinned on the host and on the device: the
 * pinned-memory budget is depth x maxMegabytes per GPU.  Values <= 0 take the
 * defaults, 16384 packets / 24 MB / 8 slots (192 MB per GPU): the queued path
 * (GpuPacketQueue, 64 threads x 256 in flight) ran at 9-13 M calls/s there
 * against 4-6 M with 4096 / 8 / 6 (profiles/r05/kernel_experiments.md 4,
 * profiles/r06/sync/).  The Java side reads them from the configuration
 * (SrtpMi355x.LANE_*_PNAME). */
JNIEXPORT jlong JNICALL JFN(aggregatorCreate)(JNIEnv *env, jclass c, jlong d, jint maxPackets, jint maxMegabytes,
                                              jint depth) {
    srtp_aggregator_opts o;
    srtp_aggregator_opts_default(&o); /* SRTP_AGG_SEAL_IDLE */
    o.max_packets = maxPackets > 0 ? (uint32_t)maxPackets : 16384u;
    o.max_bytes = (size_t)(maxMegabytes > 0 ? maxMegabytes : 24) << 20;
    o.depth = depth > 0 ? depth : 8;
    srtp_aggregator *a = NULL;
    return srtp_aggregator_create_dispatch((srtp_dispatch *)H(d), &o, NULL, NULL, &a) == SRTP_OK
               ? (jlong)(intptr_t)a : 0;
}

JNIEXPORT void JNICALL JFN(aggregatorDestroy)(JNIEnv *env, jclass c, jlong a) {
    srtp_aggregator_destroy((srtp_aggregator *)H(a));
}

/* Per-thread native copies of one packet: its bytes from the offset on, and
 * the result where the reference reallocates. */
#define ONE_BYTES (65535 + 16)
static __thread uint8_t *tl_pkt, *tl_grow;

/* Reads a RawPacket's fields and copies its bytes from the offset on (at
 * most 65535: no region is larger) into the calling thread's buffer; *arr
 * NULL for a packet without a buffer. */
static int read_packet(JNIEnv *env, jobject pkt, jbyteArray *arr, uint32_t *joff, uint32_t *avail,
                       uint32_t *length, uint32_t *flags) {
    if (!tl_pkt) {
        tl_pkt = malloc(ONE_BYTES);
        tl_grow = malloc(ONE_BYTES);
        if (!tl_pkt || !tl_grow) return SRTP_ENOMEM;
    }
    *arr = (jbyteArray)(*env)->GetObjectField(env, pkt, fid_buffer);
    const uint32_t al = *arr ? (uint32_t)(*env)->GetArrayLength(env, *arr) : 0u;
    const jint jo = (*env)->GetIntField(env, pkt, fid_offset);
    *joff = jo < 0 ? UINT32_MAX : (uint32_t)jo;
    *length = (uint32_t)(*env)->GetIntField(env, pkt, fid_length);
    *flags = (uint32_t)(*env)->GetIntField(env, pkt, fid_flags) & (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE);
    *avail = *joff <= al ? al - *joff : 0u;
    if (*avail > 65535u) *avail = 65535u;
    if (*arr && *avail) (*env)->GetByteArrayRegion(env, *arr, (jsize)*joff, (jsize)*avail, (jbyte *)tl_pkt);
    return SRTP_OK;
}

/* transform / reverseTransform of one RawPacket (srtp_rawpacket_transform_one):
 * returns its SRTP_STATUS_* (the Java side returns null for a drop and throws
 * for SRTP_STATUS_ERR_MALFORMED) or a negative SRTP_E* code.  The call blocks
 * until the packet's bundle has come back; no Java array is held meanwhile. */
JNIEXPORT jint JNICALL JFN(transformOne)(JNIEnv *env, jclass c, jlong agg, jboolean reverse, jint tid,
                                         jobject pkt) {
    if (!pkt || raw_packet_ids(env) != 0) return SRTP_EINVAL;
    jbyteArray arr;
    uint32_t joff, avail, length, flags;
    int rc = read_packet(env, pkt, &arr, &joff, &avail, &length, &flags);
    if (rc != SRTP_OK) return rc;
    const uint32_t old = length;
    int32_t status = 0;
    uint32_t need = 0;
    rc = srtp_rawpacket_transform_one((srtp_aggregator *)H(agg), reverse ? 1 : 0, tid, arr ? tl_pkt : NULL,
                                      avail, 0, &length, flags, &status, &need, tl_grow, ONE_BYTES);
    if (rc != SRTP_OK) return rc;
    if (status == SRTP_STATUS_SKIPPED || (status == SRTP_STATUS_DROP_INVALID && old > avail)) return status;
    if (need) { /* RawPacket.append / grow: a new byte[] at offset 0 */
        jbyteArray nb = (*env)->NewByteArray(env, (jsize)need);
        if (!nb) return SRTP_ENOMEM;
        (*env)->SetByteArrayRegion(env, nb, 0, (jsize)length, (const jbyte *)tl_grow);
        (*env)->SetObjectField(env, pkt, fid_buffer, nb);
        (*env)->SetIntField(env, pkt, fid_offset, 0);
    } else if (arr) {
        uint32_t w = old > length ? old : length;
        if (w > avail) w = avail;
        if (w) (*env)->SetByteArrayRegion(env, arr, (jsize)joff, (jsize)w, (const jbyte *)tl_pkt);
    }
    (*env)->SetIntField(env, pkt, fid_length, (jint)length);
    return status;
}

/* ---- the asynchronous per-packet path (GpuPacketQueue) ---- */

/* A completion queue on the process's aggregator for one Java thread (a
 * connector's send thread, a receive loop): up to maxInFlight packets
 * submitted and not yet reaped. */
JNIEXPORT jlong JNICALL JFN(queueCreate)(JNIEnv *env, jclass c, jlong agg, jint maxInFlight) {
    srtp_queue *q = NULL;
    if (maxInFlight < 1) return 0;
    return srtp_queue_create((srtp_aggregator *)H(agg), (uint32_t)maxInFlight, &q) == SRTP_OK
               ? (jlong)(intptr_t)q : 0;
}

JNIEXPORT void JNICALL JFN(queueDestroy)(JNIEnv *env, jclass c, jlong q) {
    srtp_queue_destroy((srtp_queue *)H(q));
}

/* Submits one RawPacket (srtp_rawpacket_submit): 0, SRTP_EAGAIN (reap first)
 * or another negative SRTP_E* code.  The packet's bytes are copied now; the
 * RawPacket must not change until its completion is reaped, which writes the
 * result back.  skip: the transformer's packet predicate rejected it (it
 * completes untouched, in order). */
JNIEXPORT jint JNICALL JFN(queueSubmit)(JNIEnv *env, jclass c, jlong q, jboolean reverse, jint tid, jobject pkt,
                                        jboolean skip, jlong cookie) {
    if (!pkt || raw_packet_ids(env) != 0) return SRTP_EINVAL;
    if (skip)
        return srtp_rawpacket_submit((srtp_queue *)H(q), reverse ? 1 : 0, tid, NULL, 0, 0, 0, SRTP_PKT_FLAG_SKIP,
                                     (uint64_t)cookie);
    jbyteArray arr;
    uint32_t joff, avail, length, flags;
    const int rc = read_packet(env, pkt, &arr, &joff, &avail, &length, &flags);
    if (rc != SRTP_OK) return rc;
    return srtp_rawpacket_submit((srtp_queue *)H(q), reverse ? 1 : 0, tid, arr ? tl_pkt : NULL, avail, 0, length,
                                 flags, (uint64_t)cookie);
}

static __thread srtp_completion *tl_comps;
static __thread jint *tl_status;
static __thread uint32_t tl_comps_n;

/* Reaps up to status.length completions in submission order and writes each
 * back into its RawPacket -- ring[cookie % ring.length], the Java side's ring
 * of packets in flight -- as SinglePacketTransformer leaves it (in place, or a
 * new buffer where RawPacket.append / grow reallocate; length updated).
 * status[i] receives completion i's SRTP_STATUS_*.  wait: block until at least
 * one is there.  Returns the count, or a negative SRTP_E* code when nothing was
 * reaped: once completions are taken off the native queue their count is
 * always returned (so the Java ring stays in step with the native order), and
 * a completion that could not be written back -- its native result rejected,
 * or no memory for its new buffer (the OutOfMemoryError is cleared: the packet
 * is dropped, as the reference drops what it cannot transform) -- gets
 * SRTP_STATUS_ERR_INTERNAL, which GpuPacketQueue hands on as null. */
JNIEXPORT jint JNICALL JFN(queueReap)(JNIEnv *env, jclass c, jlong qh, jobjectArray ring, jintArray status,
                                      jboolean wait) {
    srtp_queue *q = (srtp_queue *)H(qh);
    if (!q || !ring || !status || raw_packet_ids(env) != 0) return SRTP_EINVAL;
    const jsize max = (*env)->GetArrayLength(env, status), rl = (*env)->GetArrayLength(env, ring);
    if (max < 1 || rl < 1) return SRTP_EINVAL;
    if (tl_comps_n < (uint32_t)max) {
        free(tl_comps);
        free(tl_status);
        tl_comps = malloc((size_t)max * sizeof *tl_comps);
        tl_status = malloc((size_t)max * sizeof *tl_status);
        tl_comps_n = tl_comps && tl_status ? (uint32_t)max : 0u;
        if (!tl_comps_n) return SRTP_ENOMEM;
    }
    const int n = srtp_queue_reap(q, tl_comps, (uint32_t)max, wait ? 1 : 0);
    if (n <= 0) return n;
    const int framed = (*env)->PushLocalFrame(env, 2 * n + 16) == 0;
    if (!framed) (*env)->ExceptionClear(env); /* its OutOfMemoryError: the statuses still go back */
    for (int i = 0; i < n; i++) {
        const srtp_completion *cp = &tl_comps[i];
        tl_status[i] = cp->status;
        /* without a local frame no write-back is attempted (each makes local refs) */
        jobject pkt = framed ? (*env)->GetObjectArrayElement(env, ring, (jsize)(cp->cookie % (uint64_t)rl)) : NULL;
        if (!pkt) {
            if (!framed) tl_status[i] = SRTP_STATUS_ERR_INTERNAL;
            continue;
        }
        jbyteArray arr = (jbyteArray)(*env)->GetObjectField(env, pkt, fid_buffer);
        const uint32_t al = arr ? (uint32_t)(*env)->GetArrayLength(env, arr) : 0u;
        const jint jo = (*env)->GetIntField(env, pkt, fid_offset);
        const uint32_t joff = jo < 0 ? UINT32_MAX : (uint32_t)jo;
        uint32_t avail = joff <= al ? al - joff : 0u;
        if (avail > 65535u) avail = 65535u;
        uint32_t copy = 0, need = 0;
        if (srtp_rawpacket_complete(q, cp, avail, &copy, &need) != SRTP_OK) {
            tl_status[i] = SRTP_STATUS_ERR_INTERNAL;
            continue;
        }
        if (need) { /* RawPacket.append / grow: a new byte[] at offset 0 */
            jbyteArray nb = (*env)->NewByteArray(env, (jsize)need);
            if (!nb) { /* OutOfMemoryError pending: cleared, the packet dropped */
                (*env)->ExceptionClear(env);
                tl_status[i] = SRTP_STATUS_ERR_INTERNAL;
                continue;
            }
            (*env)->SetByteArrayRegion(env, nb, 0, (jsize)copy, (const jbyte *)cp->data);
            (*env)->SetObjectField(env, pkt, fid_buffer, nb);
            (*env)->SetIntField(env, pkt, fid_offset, 0);
        } else if (copy && arr) {
            (*env)->SetByteArrayRegion(env, arr, (jsize)joff, (jsize)copy, (const jbyte *)cp->data);
        }
        if (cp->data) (*env)->SetIntField(env, pkt, fid_length, (jint)cp->len);
    }
    /* every result is in its Java array: the pinned slots go back at once */
    srtp_queue_release(q);
    (*env)->SetIntArrayRegion(env, status, 0, n, tl_status);
    if (framed) (*env)->PopLocalFrame(env, NULL);
    return n;
}
