/*
 * fakejvm.c -- TEST INFRASTRUCTURE: the JNI calls of tests/jni_stub/jni.h over
 * a toy object model, so that the real JNI shim (src/native/srtp_mi355x/
 * SrtpMi355x.c, compiled unmodified against the stub header into
 * tests/jni_stub/libfakejni.so) can be driven from Python through ctypes.
 *
 * Objects: byte[], int[], Object[] and org.jitsi.impl.neomedia.RawPacket
 * (fields buffer, offset, length, flags -- RawPacket.java:53-73).  Arrays are
 * copied in and out by Get/Set*ArrayRegion exactly as a JVM does; an
 * out-of-range region is recorded as a pending exception (the checks a JVM's
 * ArrayIndexOutOfBoundsException would make), which the tests assert is never
 * raised.  Nothing is garbage-collected: objects live until fj_reset().
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "jni.h"

enum { K_BYTES = 1, K_INTS, K_OBJS, K_PACKET, K_CLASS };

struct fj_obj {
    int kind;
    jsize len;        /* arrays */
    void *data;       /* arrays */
    jobject buffer;   /* RawPacket */
    jint offset, length, flags;
    struct fj_obj *next_alloc;
};

struct fj_field {
    int id; /* 0 buffer, 1 offset, 2 length, 3 flags */
};

static struct fj_field g_fields[4] = {{0}, {1}, {2}, {3}};
static struct fj_obj g_rawpacket_class = {.kind = K_CLASS};
static struct fj_obj *g_allocs;
static int g_exceptions, g_frames;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER; /* several "JVM threads" at once */

static struct fj_obj *alloc_obj(int kind) {
    struct fj_obj *o = calloc(1, sizeof *o);
    o->kind = kind;
    pthread_mutex_lock(&g_mu);
    o->next_alloc = g_allocs;
    g_allocs = o;
    pthread_mutex_unlock(&g_mu);
    return o;
}

static struct fj_obj *new_array(int kind, jsize len, size_t elem) {
    struct fj_obj *o = alloc_obj(kind);
    o->len = len;
    o->data = calloc(len ? (size_t)len : 1, elem);
    return o;
}

static int in_range(jarray a, jsize start, jsize len) {
    if (!a || start < 0 || len < 0 || start > a->len || len > a->len - start) {
        __atomic_add_fetch(&g_exceptions, 1, __ATOMIC_RELAXED);
        return 0;
    }
    return 1;
}

static jsize GetArrayLength(JNIEnv *env, jarray a) { return a ? a->len : 0; }
static void GetIntArrayRegion(JNIEnv *env, jintArray a, jsize s, jsize n, jint *buf) {
    if (in_range(a, s, n)) memcpy(buf, (jint *)a->data + s, (size_t)n * sizeof(jint));
}
static void GetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize s, jsize n, jbyte *buf) {
    if (in_range(a, s, n)) memcpy(buf, (jbyte *)a->data + s, (size_t)n);
}
static void SetByteArrayRegion(JNIEnv *env, jbyteArray a, jsize s, jsize n, const jbyte *buf) {
    if (in_range(a, s, n)) memcpy((jbyte *)a->data + s, buf, (size_t)n);
}
static jclass FindClass(JNIEnv *env, const char *name) {
    return strcmp(name, "org/jitsi/impl/neomedia/RawPacket") == 0 ? &g_rawpacket_class : NULL;
}
static jfieldID GetFieldID(JNIEnv *env, jclass c, const char *name, const char *sig) {
    if (c != &g_rawpacket_class) return NULL;
    if (!strcmp(name, "buffer") && !strcmp(sig, "[B")) return &g_fields[0];
    if (!strcmp(name, "offset") && !strcmp(sig, "I")) return &g_fields[1];
    if (!strcmp(name, "length") && !strcmp(sig, "I")) return &g_fields[2];
    if (!strcmp(name, "flags") && !strcmp(sig, "I")) return &g_fields[3];
    return NULL;
}
static jobject GetObjectField(JNIEnv *env, jobject o, jfieldID f) {
    return o && o->kind == K_PACKET && f->id == 0 ? o->buffer : NULL;
}
static jint GetIntField(JNIEnv *env, jobject o, jfieldID f) {
    if (!o || o->kind != K_PACKET) return 0;
    return f->id == 1 ? o->offset : f->id == 2 ? o->length : f->id == 3 ? o->flags : 0;
}
static void SetIntField(JNIEnv *env, jobject o, jfieldID f, jint v) {
    if (!o || o->kind != K_PACKET) return;
    if (f->id == 1) o->offset = v;
    else if (f->id == 2) o->length = v;
    else if (f->id == 3) o->flags = v;
}
static void SetObjectField(JNIEnv *env, jobject o, jfieldID f, jobject v) {
    if (o && o->kind == K_PACKET && f->id == 0) o->buffer = v;
}
static jobject GetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i) {
    return in_range(a, i, 1) ? ((jobject *)a->data)[i] : NULL;
}
static void SetObjectArrayElement(JNIEnv *env, jobjectArray a, jsize i, jobject v) {
    if (in_range(a, i, 1)) ((jobject *)a->data)[i] = v;
}
static jint PushLocalFrame(JNIEnv *env, jint cap) {
    __atomic_add_fetch(&g_frames, 1, __ATOMIC_RELAXED);
    return JNI_OK;
}
static jobject PopLocalFrame(JNIEnv *env, jobject r) {
    __atomic_sub_fetch(&g_frames, 1, __ATOMIC_RELAXED);
    return r;
}
/* fj_fail_new_arrays(k): the next k NewByteArray calls fail as a JVM out of
 * memory does (NULL, an OutOfMemoryError pending until ExceptionClear) */
static int g_fail_new, g_pending;
static jbyteArray NewByteArray(JNIEnv *env, jsize n) {
    if (__atomic_load_n(&g_fail_new, __ATOMIC_SEQ_CST) > 0 && __atomic_fetch_sub(&g_fail_new, 1, __ATOMIC_SEQ_CST) > 0) {
        __atomic_store_n(&g_pending, 1, __ATOMIC_SEQ_CST);
        return NULL;
    }
    return new_array(K_BYTES, n, 1);
}
static void ExceptionClear(JNIEnv *env) { __atomic_store_n(&g_pending, 0, __ATOMIC_SEQ_CST); }
static jint *GetIntArrayElements(JNIEnv *env, jintArray a, jboolean *is_copy) {
    if (is_copy) *is_copy = 0;
    return a ? (jint *)a->data : NULL;
}
static void ReleaseIntArrayElements(JNIEnv *env, jintArray a, jint *e, jint mode) {}
static void SetIntArrayRegion(JNIEnv *env, jintArray a, jsize s, jsize n, const jint *buf) {
    if (in_range(a, s, n)) memcpy((jint *)a->data + s, buf, (size_t)n * sizeof(jint));
}

static const struct JNINativeInterface_ g_table = {
    GetArrayLength, GetIntArrayRegion, GetByteArrayRegion, SetByteArrayRegion, FindClass,
    GetFieldID, GetObjectField, GetIntField, SetIntField, SetObjectField, GetObjectArrayElement,
    SetObjectArrayElement, PushLocalFrame, PopLocalFrame, NewByteArray, GetIntArrayElements,
    ReleaseIntArrayElements, SetIntArrayRegion, ExceptionClear,
};
static JNIEnv g_env = &g_table;

/* ---- the tests' side (ctypes) ---- */

JNIEXPORT JNIEnv *fj_env(void) { return &g_env; }
JNIEXPORT void fj_fail_new_arrays(int k) { __atomic_store_n(&g_fail_new, k, __ATOMIC_SEQ_CST); }
JNIEXPORT int fj_exception_pending(void) { return __atomic_load_n(&g_pending, __ATOMIC_SEQ_CST); }
JNIEXPORT jobject fj_rawpacket_class(void) { return &g_rawpacket_class; }

JNIEXPORT jbyteArray fj_new_bytes(const void *data, jsize n) {
    struct fj_obj *a = new_array(K_BYTES, n, 1);
    if (data && n) memcpy(a->data, data, (size_t)n);
    return a;
}
JNIEXPORT jintArray fj_new_ints(const jint *data, jsize n) {
    struct fj_obj *a = new_array(K_INTS, n, sizeof(jint));
    if (data && n) memcpy(a->data, data, (size_t)n * sizeof(jint));
    return a;
}
JNIEXPORT jobjectArray fj_new_objects(jsize n) { return new_array(K_OBJS, n, sizeof(jobject)); }
JNIEXPORT void fj_set_element(jobjectArray a, jsize i, jobject v) { ((jobject *)a->data)[i] = v; }
JNIEXPORT void fj_ints_read(jintArray a, jint *out) { memcpy(out, a->data, (size_t)a->len * sizeof(jint)); }
JNIEXPORT jobject fj_get_element(jobjectArray a, jsize i) { return ((jobject *)a->data)[i]; }

JNIEXPORT jobject fj_new_packet(jbyteArray buffer, jint offset, jint length, jint flags) {
    struct fj_obj *o = alloc_obj(K_PACKET);
    o->buffer = buffer;
    o->offset = offset;
    o->length = length;
    o->flags = flags;
    return o;
}
JNIEXPORT jbyteArray fj_packet_buffer(jobject p) { return p->buffer; }
JNIEXPORT jint fj_packet_offset(jobject p) { return p->offset; }
JNIEXPORT jint fj_packet_length(jobject p) { return p->length; }

JNIEXPORT jsize fj_bytes_len(jbyteArray a) { return a->len; }
JNIEXPORT void fj_bytes_read(jbyteArray a, void *out) { memcpy(out, a->data, (size_t)a->len); }

/* ---- "JVM threads" driving GpuPacketQueue, in C (no interpreter lock) ---- */

#define SHIM(name) Java_org_jitsi_impl_neomedia_transform_srtp_mi355x_SrtpMi355x_##name
jlong SHIM(queueCreate)(JNIEnv *env, jclass c, jlong agg, jint maxInFlight);
void SHIM(queueDestroy)(JNIEnv *env, jclass c, jlong q);
jint SHIM(queueSubmit)(JNIEnv *env, jclass c, jlong q, jboolean reverse, jint tid, jobject pkt, jboolean skip,
                       jlong cookie);
jint SHIM(queueReap)(JNIEnv *env, jclass c, jlong q, jobjectArray ring, jintArray status, jboolean wait);

/* One thread's GpuPacketQueue (GpuPacketQueue.java): its packets pkts[0..n)
 * submitted in order (reaping whenever a submit is refused, as
 * GpuPacketQueue.transform does), then the rest reaped (drain).  Out: each
 * packet's status in submission order, the most packets it had in flight,
 * and rc (0 or the first negative code). */
struct fj_job {
    jlong agg;
    jboolean reverse;
    jint depth, n;
    const jint *tids;
    jobject *pkts;
    jint *status;
    jint max_in_flight, rc;
};

static void *fj_drive(void *arg) {
    struct fj_job *j = arg;
    JNIEnv *env = &g_env;
    const jlong q = SHIM(queueCreate)(env, NULL, j->agg, j->depth);
    if (!q) {
        j->rc = -1;
        return NULL;
    }
    const jsize ns = j->depth < 1024 ? j->depth : 1024;
    jobjectArray ring = new_array(K_OBJS, j->depth, sizeof(jobject));
    jintArray st = new_array(K_INTS, ns, sizeof(jint));
    long sub = 0, rep = 0;
    for (jint i = 0; i <= j->n && !j->rc;) {
        const int more = i < j->n;
        if (more && sub - rep < j->depth) {
            ((jobject *)ring->data)[sub % j->depth] = j->pkts[i];
            const jint rc = SHIM(queueSubmit)(env, NULL, q, j->reverse, j->tids[i], j->pkts[i], 0, (jlong)sub);
            if (rc == 0) {
                sub++;
                i++;
                if (sub - rep > j->max_in_flight) j->max_in_flight = (jint)(sub - rep);
                continue;
            }
            if (rc != -6) { /* SRTP_EAGAIN: reap first */
                j->rc = rc;
                break;
            }
        }
        if (!more && rep == sub) break;
        const jint k = SHIM(queueReap)(env, NULL, q, ring, st, 1);
        if (k < 0) {
            j->rc = k;
            break;
        }
        for (jint m = 0; m < k; m++) j->status[rep++] = ((jint *)st->data)[m];
    }
    SHIM(queueDestroy)(env, NULL, q);
    return NULL;
}

JNIEXPORT int fj_drive_queues(struct fj_job *jobs, int n_jobs) {
    pthread_t *th = calloc((size_t)n_jobs, sizeof *th);
    if (!th) return -1;
    for (int k = 0; k < n_jobs; k++) pthread_create(&th[k], NULL, fj_drive, &jobs[k]);
    for (int k = 0; k < n_jobs; k++) pthread_join(th[k], NULL);
    free(th);
    return 0;
}

/* ---- the connector loops (GpuConnectorLoops.java Send / Receive) ----
 * The same steps as the Java loops over a GpuPacketQueue (GpuPacketQueue.java,
 * again in C): input arrives in bursts -- a poll / receive finds the current
 * burst's items, then "nothing yet" once; a waiting poll (nothing in flight)
 * releases the next burst at once.  packetize / createRawPacket copy the
 * buffer into a new RawPacket of exactly its length (so protect's trailer
 * makes RawPacket.append reallocate); send / handOn record the packet in
 * out[] in the order it is handed on.  Packets the queue completes with a
 * status other than OK / SKIPPED are dropped, as the sink does. */
struct fj_gq {
    jlong q;
    jobjectArray ring;
    jintArray st;
    long sub, rep;
    jint n, ns;
};
struct fj_loop {
    jlong agg;
    jboolean reverse;
    jint tid, n_in, depth;
    jobject *in;         /* [n_in] input buffers (byte[]) */
    const jint *bursts;  /* burst sizes, summing to n_in */
    jint n_bursts;
    jobject *out;        /* [n_in] packets handed on, in order */
    jint n_out, n_dropped, max_in_flight, polls_empty, rc;
};
static void gq_reap(JNIEnv *env, struct fj_gq *g, struct fj_loop *L, int wait) {
    if (g->sub == g->rep) return;
    const jint k = SHIM(queueReap)(env, NULL, g->q, g->ring, g->st, (jboolean)wait);
    if (k < 0) { L->rc = k; return; }
    for (jint m = 0; m < k; m++) {
        jobject pkt = ((jobject *)g->ring->data)[g->rep % g->n];
        const jint s = ((jint *)g->st->data)[m];
        g->rep++;
        if (s == 0 || s == 9) L->out[L->n_out++] = pkt; /* STATUS_OK / STATUS_SKIPPED: handed on */
        else L->n_dropped++;
    }
}
static void gq_transform(JNIEnv *env, struct fj_gq *g, struct fj_loop *L, jobject pkt) {
    while (!L->rc) {
        if (g->sub - g->rep < g->n) {
            ((jobject *)g->ring->data)[g->sub % g->n] = pkt;
            const jint rc = SHIM(queueSubmit)(env, NULL, g->q, L->reverse, L->tid, pkt, 0, (jlong)g->sub);
            if (rc == 0) {
                g->sub++;
                if (g->sub - g->rep > L->max_in_flight) L->max_in_flight = (jint)(g->sub - g->rep);
                return;
            }
            if (rc != -6) { L->rc = rc; return; } /* not SRTP_EAGAIN */
        }
        gq_reap(env, g, L, 1);
    }
}
/* one loop (send: reverse = 0, receive: reverse = 1; the steps are the same) */
static void *fj_loop_run(void *arg) {
    struct fj_loop *L = arg;
    JNIEnv *env = &g_env;
    struct fj_gq g = {0};
    g.n = L->depth;
    g.ns = L->depth < 1024 ? L->depth : 1024;
    g.q = SHIM(queueCreate)(env, NULL, L->agg, L->depth);
    if (!g.q) { L->rc = -1; return NULL; }
    g.ring = new_array(K_OBJS, g.n, sizeof(jobject));
    g.st = new_array(K_INTS, g.ns, sizeof(jint));
    jint next = 0, burst = 0, released = 0;
    while (!L->rc && (next < L->n_in || g.sub != g.rep)) {
        /* poll(outstanding ? 0 : 500) / receive(outstanding ? 1 ms : block) */
        const int waiting = g.sub == g.rep;
        if (next == released && burst < L->n_bursts && waiting) released += L->bursts[burst++];
        if (next == released) { /* nothing yet: reap what is due, then the next burst arrives */
            L->polls_empty++;
            gq_reap(env, &g, L, 1);
            if (burst < L->n_bursts) released += L->bursts[burst++];
            continue;
        }
        jbyteArray src = L->in[next++];
        struct fj_obj *b = new_array(K_BYTES, src->len, 1);
        memcpy(b->data, src->data, (size_t)src->len);
        gq_transform(env, &g, L, fj_new_packet(b, 0, src->len, 0));
        gq_reap(env, &g, L, 0); /* what is done, without waiting */
    }
    SHIM(queueDestroy)(env, NULL, g.q);
    return NULL;
}
JNIEXPORT int fj_run_loops(struct fj_loop *loops, int n) {
    pthread_t *th = calloc((size_t)n, sizeof *th);
    if (!th) return -1;
    for (int k = 0; k < n; k++) pthread_create(&th[k], NULL, fj_loop_run, &loops[k]);
    for (int k = 0; k < n; k++) pthread_join(th[k], NULL);
    free(th);
    return 0;
}

/* pending "exceptions" (out-of-range array regions) and unbalanced local frames */
JNIEXPORT int fj_exceptions(void) { return g_exceptions; }
JNIEXPORT int fj_frames(void) { return g_frames; }

JNIEXPORT void fj_reset(void) {
    while (g_allocs) {
        struct fj_obj *o = g_allocs;
        g_allocs = o->next_alloc;
        free(o->data);
        free(o);
    }
    g_exceptions = 0;
    g_frames = 0;
}
