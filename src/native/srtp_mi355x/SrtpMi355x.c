/*
 * SrtpMi355x.c -- JNI shim between libjitsi's Java transformers and the
 * MI355X SRTP engine (include/srtp_mi355x.h, libsrtp_mi355x.so).
 *
 * NOT COMPILED IN THIS REPOSITORY: the image has no JDK and no jni.h.  It is
 * the file a maintainer adds next to src/native/openssl/ and builds like
 * libjnopenssl:
 *
 *   gcc -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       src/native/srtp_mi355x/SrtpMi355x.c -Llibjitsi_amd -lsrtp_mi355x -o libjnsrtp_mi355x.so
 *
 * Everything below the JNI calls is srtp_* C ABI that the GPU tests exercise
 * (the RawPacket[] marshalling is srtp_rawpacket_transform, tested through
 * ctypes in tests/test_rawpacket.py).  Conventions of src/native/openssl:
 * native handles are jlong casts of heap pointers (BlockCipher.c:64-73),
 * arrays are pinned with GetPrimitiveArrayCritical (BlockCipher.c:199-222),
 * errors come back as negative return codes that the Java side turns into a
 * RuntimeException (OpenSSLBlockCipher.java:310-313).
 *
 * Java side: org.jitsi.impl.neomedia.transform.srtp.mi355x.SrtpMi355x (the
 * native declarations), GpuSRTPTransformer / GpuSRTCPTransformer (the
 * PacketTransformer drop-ins), GpuSRTPContextFactory.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

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
    jbyte *k = (*env)->GetPrimitiveArrayCritical(env, key, NULL);
    jbyte *s = (*env)->GetPrimitiveArrayCritical(env, salt, NULL);
    int rc = srtp_dispatch_factory_create((srtp_dispatch *)H(d), sender, (const uint8_t *)k, kl,
                                          (const uint8_t *)s, sl, (const srtp_policy *)p1,
                                          (const srtp_policy *)p2, &id);
    (*env)->ReleasePrimitiveArrayCritical(env, salt, s, JNI_ABORT);
    (*env)->ReleasePrimitiveArrayCritical(env, key, k, JNI_ABORT);
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

/* One srtp_rawpacket_batch per Java thread (a ThreadLocal<Long> on the Java side). */
JNIEXPORT jlong JNICALL JFN(batchCreate)(JNIEnv *env, jclass c, jlong d) {
    srtp_rawpacket_batch *b = NULL;
    return srtp_rawpacket_batch_create_dispatch((srtp_dispatch *)H(d), &b) == SRTP_OK ? (jlong)(intptr_t)b : 0;
}

JNIEXPORT void JNICALL JFN(batchDestroy)(JNIEnv *env, jclass c, jlong b) {
    srtp_rawpacket_batch_destroy((srtp_rawpacket_batch *)H(b));
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
 * returns: every element is written back), or a negative SRTP_E* code. */
JNIEXPORT jint JNICALL JFN(transformPackets)(JNIEnv *env, jclass c, jlong batch, jboolean reverse, jint tid,
                                             jobjectArray pkts, jintArray skip) {
    srtp_rawpacket_batch *b = (srtp_rawpacket_batch *)H(batch);
    if (!b || !pkts || raw_packet_ids(env) != 0) return SRTP_EINVAL;
    const jsize n = (*env)->GetArrayLength(env, pkts);
    if (n == 0) return 0;
    if ((*env)->PushLocalFrame(env, 2 * n + 16) != 0) return SRTP_ENOMEM;
    jobject *objs = calloc((size_t)n, sizeof *objs);
    jbyteArray *arrs = calloc((size_t)n, sizeof *arrs);
    uint8_t **bufs = calloc((size_t)n, sizeof *bufs);
    uint32_t *u = calloc((size_t)n * 6, sizeof *u); /* buf_len, offset, length, flags, need_len, (pad) */
    int32_t *status = calloc((size_t)n, sizeof *status);
    jint *sk = skip ? (*env)->GetIntArrayElements(env, skip, NULL) : NULL;
    int rc = SRTP_ENOMEM;
    if (!objs || !arrs || !bufs || !u || !status) goto out;
    uint32_t *buf_len = u, *offset = u + n, *length = u + 2 * n, *flags = u + 3 * n, *need = u + 4 * n;
    /* the fields first: no JNI call is allowed between the critical sections */
    for (jsize i = 0; i < n; i++) {
        objs[i] = (*env)->GetObjectArrayElement(env, pkts, i);
        if (!objs[i]) continue;
        arrs[i] = (jbyteArray)(*env)->GetObjectField(env, objs[i], fid_buffer);
        buf_len[i] = arrs[i] ? (uint32_t)(*env)->GetArrayLength(env, arrs[i]) : 0u;
        offset[i] = (uint32_t)(*env)->GetIntField(env, objs[i], fid_offset);
        length[i] = (uint32_t)(*env)->GetIntField(env, objs[i], fid_length);
        flags[i] = (uint32_t)(*env)->GetIntField(env, objs[i], fid_flags) &
                   (SRTP_PKT_FLAG_DISCARD | SRTP_PKT_FLAG_SILENCE);
        if (sk && sk[i]) flags[i] |= SRTP_PKT_FLAG_SKIP;
    }
    for (jsize i = 0; i < n; i++)
        if (arrs[i]) bufs[i] = (*env)->GetPrimitiveArrayCritical(env, arrs[i], NULL);
    int32_t thrown = -1;
    rc = srtp_rawpacket_transform(b, reverse ? 1 : 0, NULL, tid, bufs, buf_len, offset, length, flags, status,
                                  need, (uint32_t)n, &thrown);
    for (jsize i = n; i-- > 0;) /* written in place: mode 0 copies back if the VM copied */
        if (bufs[i]) (*env)->ReleasePrimitiveArrayCritical(env, arrs[i], bufs[i], 0);
    if (rc != SRTP_OK) goto out;
    for (jsize i = 0; i < n; i++) {
        const int32_t st = status[i];
        if (!objs[i] || st == SRTP_STATUS_SKIPPED || st == SRTP_STATUS_NOT_PROCESSED) continue;
        if (need[i]) { /* RawPacket.append / grow: a new byte[] at offset 0 */
            const uint8_t *data;
            uint32_t dl;
            jbyteArray nb = (*env)->NewByteArray(env, (jsize)need[i]);
            if (!nb || srtp_rawpacket_result(b, (uint32_t)i, &data, &dl) != SRTP_OK) {
                rc = SRTP_ENOMEM;
                goto out;
            }
            (*env)->SetByteArrayRegion(env, nb, 0, (jsize)dl, (const jbyte *)data);
            (*env)->SetObjectField(env, objs[i], fid_buffer, nb);
            (*env)->SetIntField(env, objs[i], fid_offset, 0);
        }
        (*env)->SetIntField(env, objs[i], fid_length, (jint)length[i]);
        if (st != SRTP_STATUS_OK && st != SRTP_STATUS_ERR_MALFORMED)
            (*env)->SetObjectArrayElement(env, pkts, i, NULL); /* the reference returned null */
    }
    rc = thrown >= 0 ? thrown + 1 : 0;
out:
    if (sk) (*env)->ReleaseIntArrayElements(env, skip, sk, JNI_ABORT);
    free(objs);
    free(arrs);
    free(bufs);
    free(u);
    free(status);
    (*env)->PopLocalFrame(env, NULL);
    return rc;
}
