// engine.cpp -- host side of the MI355X SRTP engine: the C ABI of
// include/srtp_mi355x.h.  Owns the HBM-resident tables (session keys,
// factories, transformers, the (transformer, SSRC) context hash table) and
// enqueues the bundle pipeline of srtp_kernels.hip on a HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include <stdlib.h>
#include <string.h>

#include "../../include/srtp_mi355x.h"
#include "host_crypto.h"
#include "srtp_kernels.h"

using namespace srtp;

struct srtp_engine {
    srtp_engine_opts opts{};
    hipStream_t stream = nullptr;
    std::mutex mu;
    std::string last_error;

    KeySet *d_keysets = nullptr;
    ExtKeys *d_extkeys = nullptr; // round keys of the k_ext key sets (same index)
    TwofishKeys *d_tfkeys = nullptr; // 2 per key set, allocated with the first Twofish factory
    SkeinKeys *d_skkeys = nullptr;   // 1 per key set, allocated with the first Skein factory
    uint32_t n_ext = 0;           // k_ext key sets created (F8, AES-256, Twofish, Skein): k_ext runs only when > 0
    uint32_t n_skein = 0;         // Skein-MAC key sets created: k_skein runs only when > 0
    uint32_t n_not_wide = 0;      // key sets the split path cannot run (not AES-CM / NULL cipher + HMAC-SHA1)
    uint32_t n_keysets = 0, max_keysets = 0;
    FactoryRec *d_factories = nullptr;
    std::vector<FactoryRec> factories;
    std::vector<int32_t> f_rtcp_tag; // per factory: its SRTCP policy's tag length (RawPacket.grow)
    TransformerRec *d_transformers = nullptr;
    std::vector<TransformerRec> transformers;
    uint64_t *d_ctx_keys = nullptr;
    CtxState *d_ctx = nullptr;
    uint32_t ctx_cap = 0;
    uint32_t *d_far = nullptr; // [ctx_cap] BundleArgs::far
    int ctx_bits = 0;

    // per-bundle scratch, sized for scratch_n packets
    uint32_t scratch_n = 0;
    uint32_t *p_slot = nullptr, *sk_in = nullptr, *sk_out = nullptr;
    WalkRec *sv_in = nullptr, *sv_out = nullptr;
    int32_t *w_status = nullptr;
    uint32_t *w_cw = nullptr, *w_len = nullptr, *gok = nullptr, *mid = nullptr;
    uint32_t *tailc = nullptr, *spec = nullptr;
    uint64_t *tile_link = nullptr;
    uint32_t *spos = nullptr;
    uint32_t *lord = nullptr; // [n] crypto kernels' lane order (the sort's first pass)
    uint32_t *cls_tile = nullptr; // [tiles][33] length classes per sort tile (k_parse, zeroed by k_walk)
    void *sort_temp = nullptr;
    size_t sort_temp_bytes = 0;
    // Two control blocks (BundleCtl + e_min row), alternating per bundle: each
    // bundle's k_parse resets the other one for the next bundle, so the common
    // case needs no memset launch.  ctl_clean / emin_filled track what is known
    // reset on the device (emin_filled = leading e_min entries at 0x7f7f7f7f).
    int32_t *e_min = nullptr; // [2][max_transformers]
    BundleCtl *ctl = nullptr; // [2]
    int ctl_cur = 0;
    bool ctl_clean[2] = {false, false};
    uint32_t emin_filled[2] = {0u, 0u};
    // stream of the previous bundle: a bundle on another stream first waits
    // for it (bundles of one engine share its scratch)
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    // recorded on the bundle's stream after each bundle: later bundles on other
    // streams wait for it on the device, control-plane calls on the host
    hipEvent_t ev_last = nullptr;
    // device-resident bundles (srtp_transform_device) end with ev_dev instead:
    // a device-scope release.  A system-scope one (ev_last) writes back and
    // invalidates the L2 and idles the queue ~10-13 us per bundle
    // (profiles/r05/events/); host-visible completion is fenced at sync time
    // instead (fence_to_host).
    hipEvent_t ev_dev = nullptr;
    bool last_dev = false;
    unsigned long long *d_count = nullptr; // [2] live / tombstone counts
    unsigned long long *d_counters = nullptr; // [kCountReplicas][kCtrStride]
#ifdef SRTP_STAMPS
    unsigned long long *d_stamps[2] = {nullptr, nullptr}; // diagnostic build: protect / unprotect
#endif
    uint64_t n_bundles = 0, n_packets = 0, n_rehash = 0, n_small = 0;
    uint32_t serial = 1;

    // staging for srtp_transform_host
    uint8_t *h_seg = nullptr;
    size_t h_seg_bytes = 0;
    uint32_t h_n = 0;
    uint32_t *h_off = nullptr, *h_len = nullptr, *h_cap = nullptr, *h_flags = nullptr;
    int32_t *h_status = nullptr, *h_tids = nullptr;

    // optional per-stage timing (HIP events on the bundle stream)
    bool timing = false;
    uint32_t dbg = 0;     // srtp_engine_set_debug test hooks
    struct Mark { int stage; hipEvent_t a, b; };
    std::vector<Mark> marks;
    std::vector<hipEvent_t> event_pool;
};

namespace {
constexpr uint32_t kSmallCtrMax = 8192u; // k_ctr_small takes bundles up to this size
// The split path (k_ctr_wide + k_mac_wide) for bundles of kWideMin..kWideMax
// packets: there the fused kernels' lane per packet leaves most CUs idle or
// latency-bound; from 2^17 packets on the fused kernels are faster
// (profiles/r06/kernel_experiments.md, bundle-size sweep)
#ifndef SRTP_WIDE_MIN
#define SRTP_WIDE_MIN 2048u
#endif
constexpr uint32_t kWideMin = SRTP_WIDE_MIN, kWideMax = 65536u;

int fail(srtp_engine *e, int code, const std::string &msg) {
    if (e) e->last_error = msg;
    return code;
}

#define HIPCHK(e, x)                                                                     \
    do {                                                                                 \
        hipError_t _err = (x);                                                           \
        if (_err != hipSuccess)                                                          \
            return fail((e), SRTP_EDEVICE, std::string(#x ": ") + hipGetErrorString(_err)); \
    } while (0)

template <class T> hipError_t dalloc(T **p, size_t count) {
    return hipMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T));
}

void dfree(void *p) {
    if (p) (void)hipFree(p);
}

// Profiles the engine implements: AES-CM with a 128- or 256-bit key, AES-F8
// (128), or NULL cipher x HMAC_SHA1 or NULL auth (SRTPPolicy.java; profile
// tables DtlsPacketTransformer.java:574-612, SDesTransformEngine.java:129-147;
// AES-256-CM is what SRTPCryptoContext does with encKeyLength 32, e.g. from
// ZRTP's AES3, ZRTPTransformEngine.java:873-900).  Tag length <= 12 keeps the
// reference's readRegionToBuff in range for every packet of >= 12 bytes.
bool is_twofish(int enc) { return enc == SRTP_TWOFISH_ENCRYPTION || enc == SRTP_TWOFISHF8_ENCRYPTION; }
bool is_f8(int enc) { return enc == SRTP_AESF8_ENCRYPTION || enc == SRTP_TWOFISHF8_ENCRYPTION; }

bool policy_ok(const srtp_policy *p, bool rtcp) {
    if (!p) return false;
    if (p->enc_type != SRTP_NULL_ENCRYPTION && p->enc_type != SRTP_AESCM_ENCRYPTION &&
        p->enc_type != SRTP_AESF8_ENCRYPTION && !is_twofish(p->enc_type))
        return false;
    if (p->enc_type != SRTP_NULL_ENCRYPTION && p->salt_key_len != 14) return false;
    if (p->enc_type == SRTP_AESF8_ENCRYPTION && p->enc_key_len != 16) return false;
    if ((p->enc_type == SRTP_AESCM_ENCRYPTION || is_twofish(p->enc_type)) && p->enc_key_len != 16 &&
        p->enc_key_len != 32)
        return false;
    // SRTCP F8 ciphers [8, 8 + length - 4 - tag) (SRTCPCryptoContext :285-291):
    // inside the packet only with an HMAC trailer of >= 4 tag bytes after it
    if (rtcp && is_f8(p->enc_type) &&
        (p->auth_type == SRTP_NULL_AUTHENTICATION || p->auth_tag_len < 4))
        return false;
    if (p->auth_type != SRTP_NULL_AUTHENTICATION && p->auth_type != SRTP_HMACSHA1_AUTHENTICATION &&
        p->auth_type != SRTP_SKEIN_AUTHENTICATION)
        return false;
    if (p->auth_type == SRTP_HMACSHA1_AUTHENTICATION && p->auth_key_len != 20) return false;
    // Skein (ZRTP "SK32"/"SK64", authKeyLen 32, ZRTPTransformEngine.java:867-872):
    // a key of one UBI block at most and a tag of >= 1 byte (the MAC's output
    // is tag_len * 8 bits, SRTPCryptoContext.java:421-428)
    if (p->auth_type == SRTP_SKEIN_AUTHENTICATION &&
        (p->auth_key_len < 1 || p->auth_key_len > 64 || p->auth_tag_len < 1))
        return false;
    if (p->auth_tag_len < 0 || p->auth_tag_len > 12) return false;
    return true;
}

// Master key bytes a policy uses (BaseSRTPCryptoContext copies encKeyLength
// of them, :187-190): 32 for the 256-bit AES-CM / Twofish policies, else 16
// (the NULL cipher keeps the AES-128 PRF, see srtp_factory_create).
int master_key_len(const srtp_policy *pol) {
    return pol->enc_type != SRTP_NULL_ENCRYPTION && pol->enc_key_len == 32 ? 32 : 16;
}

void build_keyset(const uint8_t *mk, const uint8_t ms[14], bool rtcp, const srtp_policy *pol,
                  KeySet *ks, ExtKeys *ext, TwofishKeys *tf, SkeinKeys *sk) {
    memset(ks, 0, sizeof *ks);
    memset(ext, 0, sizeof *ext);
    memset(tf, 0, 2 * sizeof *tf);
    memset(sk, 0, sizeof *sk);
    const int klen = master_key_len(pol);
    const bool twofish = is_twofish(pol->enc_type);
    const bool skein = pol->auth_type == SRTP_SKEIN_AUTHENTICATION;
    const int auth_len = skein ? pol->auth_key_len : 20;
    uint8_t enc[32], auth[64], salt[16] = {0};
    // RFC 3711 4.3 with the policy's cipher as the PRF -- AES-128, AES-256
    // (RFC 6188 4.1) or Twofish -- as deriveSrtpKeys :393-447 does with a key
    // of encKeyLength bytes (and an auth key of authKeyLength bytes)
    derive_session_keys_cipher(twofish, mk, klen, ms, rtcp, enc, auth, salt, auth_len);
    // SRTPCipherF8.deriveForIV :66-95: the IV' key is key ^ (salt || 0x55..)
    uint8_t m[32];
    for (int i = 0; i < klen; i++) m[i] = (uint8_t)(enc[i] ^ (i < 14 ? salt[i] : 0x55));
    if (twofish) { // k_ext, Twofish tables
        twofish_schedule(enc, klen, tf[0].K, tf[0].T);
        if (is_f8(pol->enc_type)) twofish_schedule(m, klen, tf[1].K, tf[1].T);
        ks->ext = 1;
    } else if (klen == 32) { // AES-256-CM: k_ext
        ext->nr = aes_expand_le(enc, 32, ext->rk);
        ks->ext = 1;
    } else {
        aes128_expand_le(enc, ks->rk);
    }
    if (pol->enc_type == SRTP_AESF8_ENCRYPTION) {
        ext->nr = aes_expand_le(m, 16, ext->rk);
        ks->ext = 1;
    }
    memset(m, 0, sizeof m);
    if (skein) { // SkeinMac keyed once: the packets' MACs start from g0 (k_skein)
        skein512_key_state(auth, auth_len, 8 * pol->auth_tag_len, sk->g0);
        ks->ext = 1;
    } else {
        hmac_sha1_midstates(auth, ks->ipad, ks->opad);
    }
    for (int i = 0; i < 4; i++)
        ks->salt[i] = (uint32_t)salt[4 * i] | ((uint32_t)salt[4 * i + 1] << 8) |
                      ((uint32_t)salt[4 * i + 2] << 16) | ((uint32_t)salt[4 * i + 3] << 24);
    ks->enc_type = pol->enc_type;
    ks->auth_type = pol->auth_type;
    ks->tag_len = pol->auth_tag_len;
    ks->kind = rtcp ? SRTP_KIND_RTCP : SRTP_KIND_RTP;
    memset(enc, 0, sizeof enc);
    memset(auth, 0, sizeof auth);
    memset(salt, 0, sizeof salt);
}

uint32_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return (uint32_t)std::min<uint64_t>(p, 1ull << 31);
}

void free_scratch(srtp_engine *e) {
    void *ptrs[] = {e->p_slot, e->sk_in, e->sk_out, e->sv_in, e->sv_out, e->w_status, e->w_cw,
                    e->w_len, e->gok, e->mid, e->tailc, e->spec, e->sort_temp,
                    e->spos, e->tile_link, e->lord, e->cls_tile};
    for (void *p : ptrs) dfree(p);
    e->p_slot = e->sk_in = e->sk_out = nullptr;
    e->sv_in = e->sv_out = nullptr;
    e->w_status = nullptr;
    e->w_cw = e->w_len = e->gok = e->mid = e->tailc = e->spec = nullptr;
    e->spos = nullptr;
    e->lord = nullptr;
    e->cls_tile = nullptr;
    e->tile_link = nullptr;
    e->sort_temp = nullptr;
    e->scratch_n = 0;
}

int quiesce(srtp_engine *e);

int ensure_scratch(srtp_engine *e, uint32_t n) {
    if (n <= e->scratch_n) return SRTP_OK;
    int qrc = quiesce(e); // the old scratch may still be in use by an enqueued bundle
    if (qrc != SRTP_OK) return qrc;
    free_scratch(e);
    uint32_t m = std::max<uint32_t>(n, 1024);
    HIPCHK(e, dalloc(&e->p_slot, m));
    HIPCHK(e, dalloc(&e->sk_in, m));
    HIPCHK(e, dalloc(&e->sk_out, m + 8)); // k_walk reads batches of 4 past a segment end
    HIPCHK(e, dalloc(&e->sv_in, m));
    HIPCHK(e, dalloc(&e->sv_out, m + 8));
    HIPCHK(e, dalloc(&e->w_status, m));
    HIPCHK(e, dalloc(&e->w_cw, m));
    HIPCHK(e, dalloc(&e->w_len, m));
    HIPCHK(e, dalloc(&e->gok, (size_t)2 * m));
    HIPCHK(e, dalloc(&e->mid, (size_t)5 * m));
    HIPCHK(e, dalloc(&e->tailc, (size_t)16 * m));
    HIPCHK(e, dalloc(&e->spec, m));
    HIPCHK(e, dalloc(&e->spos, m));
    HIPCHK(e, dalloc(&e->lord, m));
    {
        const uint32_t st = sort_tile_records();
        const size_t words = (size_t)((m + st - 1u) / st) * 33u;
        HIPCHK(e, dalloc(&e->cls_tile, words));
        HIPCHK(e, hipMemset(e->cls_tile, 0, words * 4));
    }
    // walk tiles' long-chain links: granules tagged with the bundle serial + 1,
    // so zeroed memory never reads as published
    const size_t link_words = (size_t)(m / kLongMin + 2) * 10; // per walk tile
    HIPCHK(e, dalloc(&e->tile_link, link_words));
    HIPCHK(e, hipMemset(e->tile_link, 0, link_words * sizeof(uint64_t)));
    e->sort_temp_bytes = sort_temp_bytes(m);
    HIPCHK(e, hipMalloc(&e->sort_temp, std::max<size_t>(e->sort_temp_bytes, 16)));
    // per-tile digit counts start at zero (each scan re-zeroes what it read)
    HIPCHK(e, hipMemset(e->sort_temp, 0, e->sort_temp_bytes));
    e->scratch_n = m;
    return SRTP_OK;
}

int sync_factory(srtp_engine *e, int32_t id) {
    HIPCHK(e, hipMemcpy(e->d_factories + id, &e->factories[id], sizeof(FactoryRec),
                        hipMemcpyHostToDevice));
    return SRTP_OK;
}

int sync_transformer(srtp_engine *e, int32_t id) {
    HIPCHK(e, hipMemcpy(e->d_transformers + id, &e->transformers[id], sizeof(TransformerRec),
                        hipMemcpyHostToDevice));
    return SRTP_OK;
}

int close_factory_locked(srtp_engine *e, int32_t id) {
    if (id < 0 || (size_t)id >= e->factories.size()) return SRTP_EINVAL;
    if (!e->factories[id].open) return SRTP_OK;
    e->factories[id].open = 0;
    return sync_factory(e, id);
}

hipEvent_t take_event(srtp_engine *e) {
    if (!e->event_pool.empty()) {
        hipEvent_t ev = e->event_pool.back();
        e->event_pool.pop_back();
        return ev;
    }
    hipEvent_t ev = nullptr;
    if (hipEventCreate(&ev) != hipSuccess) return nullptr;
    return ev;
}

// Records an event before a stage; end_stage records the matching one after.
struct StageTimer {
    srtp_engine *e;
    hipStream_t s;
    int stage;
    hipEvent_t a = nullptr;
    StageTimer(srtp_engine *e_, hipStream_t s_, int stage_) : e(e_), s(s_), stage(stage_) {
        if (!e->timing) return;
        a = take_event(e);
        if (a) (void)hipEventRecord(a, s);
    }
    ~StageTimer() {
        if (!a) return;
        hipEvent_t b = take_event(e);
        if (!b) return;
        (void)hipEventRecord(b, s);
        e->marks.push_back({stage, a, b});
    }
};

// Makes the engine's device current for the duration of one C-ABI call and
// restores the caller's device afterwards: every allocation, copy, launch and
// synchronisation of an engine happens on its device whatever the calling
// thread had current (a JVM thread may drive several engines).
struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

#define GUARD(e)                                                                         \
    DeviceGuard _guard((e)->opts.device);                                                \
    if (!_guard.ok) return fail((e), SRTP_EDEVICE, "hipSetDevice failed")

// Waits until every bundle this engine has enqueued (on any stream) and its
// own stream's work have completed: the precondition of every control-plane
// call that reads or rewrites device state the kernels use.
static hipEvent_t last_event(const srtp_engine *e) { return e->last_dev ? e->ev_dev : e->ev_last; }

// After a device-scope event: a system-scope release on `s` behind it, so
// that what the bundle wrote is visible to the host (a caller's zero-copy
// buffers) when the wait returns.
static int fence_to_host(srtp_engine *e, hipStream_t s) {
    if (!e->last_dev) return SRTP_OK;
    HIPCHK(e, hipStreamWaitEvent(s, e->ev_dev, 0));
    HIPCHK(e, hipEventRecord(e->ev_last, s));
    HIPCHK(e, hipEventSynchronize(e->ev_last));
    e->last_dev = false;
    return SRTP_OK;
}

int quiesce(srtp_engine *e) {
    if (e->have_last) HIPCHK(e, hipEventSynchronize(last_event(e)));
    if (e->have_last && e->last_dev) {
        int rc = fence_to_host(e, e->stream);
        if (rc != SRTP_OK) return rc;
    }
    if (e->stream) HIPCHK(e, hipStreamSynchronize(e->stream));
    return SRTP_OK;
}

// Live and tombstone slots of the context table.
int count_slots(srtp_engine *e, uint64_t *live, uint64_t *tomb) {
    unsigned long long c[2] = {0, 0};
    HIPCHK(e, hipMemsetAsync(e->d_count, 0, sizeof c, e->stream));
    HIPCHK(e, launch_count_contexts(e->d_ctx_keys, e->ctx_cap, e->d_count, e->stream));
    HIPCHK(e, hipMemcpyAsync(c, e->d_count, sizeof c, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    *live = c[0];
    *tomb = c[1];
    return SRTP_OK;
}

// Rebuilds the context table without tombstones (quiesced engine).  Transformer
// closes (every DTLS rekey) and abort rollbacks leave tombstones; inserts reuse
// them, and this keeps probe paths short once they pile up.
int rehash(srtp_engine *e, uint64_t live) {
    uint64_t *tk = nullptr;
    CtxState *tc = nullptr;
    int rc = SRTP_OK;
    if (dalloc(&tk, live) != hipSuccess || dalloc(&tc, live) != hipSuccess) {
        dfree(tk);
        return fail(e, SRTP_ENOMEM, "rehash scratch");
    }
    unsigned long long n = 0;
    hipStream_t s = e->stream;
    do {
        if (hipMemsetAsync(e->d_count, 0, 8, s) != hipSuccess ||
            launch_rehash_collect(e->d_ctx_keys, e->d_ctx, e->ctx_cap, tk, tc, e->d_count, s) != hipSuccess ||
            hipMemcpyAsync(&n, e->d_count, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = fail(e, SRTP_EDEVICE, "rehash collect");
            break;
        }
        if (n > live) { rc = fail(e, SRTP_EDEVICE, "rehash: live count changed"); break; }
        if (hipMemsetAsync(e->d_ctx_keys, 0xff, (size_t)e->ctx_cap * sizeof(uint64_t), s) != hipSuccess ||
            hipMemsetAsync(e->d_ctx, 0, (size_t)e->ctx_cap * sizeof(CtxState), s) != hipSuccess ||
            launch_rehash_insert(e->d_ctx_keys, e->d_ctx, e->ctx_cap - 1, tk, tc, (uint32_t)n, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) {
            rc = fail(e, SRTP_EDEVICE, "rehash insert");
            break;
        }
        e->n_rehash++;
    } while (0);
    dfree(tk);
    dfree(tc);
    return rc;
}

uint64_t mix64_host(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

} // namespace

extern "C" {

int srtp_engine_opts_default(srtp_engine_opts *o) {
    if (!o) return SRTP_EINVAL;
    o->device = 0;
    o->check_replay = 1;
    o->abort_on_error = 1;
    o->max_contexts = 1u << 20; // table of next_pow2(2 x max_contexts) slots
    o->max_factories = 1u << 16;
    o->max_transformers = 1u << 16;
    o->max_batch = 1u << 16;
    return SRTP_OK;
}

int srtp_engine_create(const srtp_engine_opts *opts, srtp_engine **out) {
    if (!out) return SRTP_EINVAL;
    *out = nullptr;
    srtp_engine_opts o;
    if (opts) o = *opts;
    else srtp_engine_opts_default(&o);
    if (o.max_contexts == 0 || o.max_factories == 0 || o.max_transformers == 0) return SRTP_EINVAL;
    srtp_engine *e = new (std::nothrow) srtp_engine();
    if (!e) return SRTP_ENOMEM;
    e->opts = o;
    int rc = SRTP_OK;
    DeviceGuard guard(o.device);
    do {
        if (!guard.ok) { rc = SRTP_EDEVICE; break; }
        if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) { rc = SRTP_EDEVICE; break; }
        if (hipEventCreateWithFlags(&e->ev_last, hipEventDisableTiming) != hipSuccess) { rc = SRTP_EDEVICE; break; }
        if (hipEventCreateWithFlags(&e->ev_dev, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
            rc = SRTP_EDEVICE;
            break;
        }
        uint32_t te0[256];
        aes_te0_le(te0);
        if (upload_tables(te0) != hipSuccess) { rc = SRTP_EDEVICE; break; }
        e->max_keysets = 2 * o.max_factories;
        e->ctx_cap = next_pow2(2ull * o.max_contexts);
        e->ctx_bits = 0;
        while ((1u << e->ctx_bits) < e->ctx_cap) e->ctx_bits++;
        if (dalloc(&e->d_keysets, e->max_keysets) != hipSuccess ||
            dalloc(&e->d_extkeys, e->max_keysets) != hipSuccess ||
            dalloc(&e->d_factories, o.max_factories) != hipSuccess ||
            dalloc(&e->d_transformers, o.max_transformers) != hipSuccess ||
            dalloc(&e->d_ctx_keys, e->ctx_cap) != hipSuccess ||
            dalloc(&e->d_ctx, e->ctx_cap) != hipSuccess ||
            dalloc(&e->d_far, e->ctx_cap) != hipSuccess ||
            dalloc(&e->e_min, 2 * (size_t)o.max_transformers) != hipSuccess ||
            dalloc(&e->ctl, 2) != hipSuccess || dalloc(&e->d_count, 2) != hipSuccess ||
            dalloc(&e->d_counters, (size_t)kCountReplicas * kCtrStride) != hipSuccess) {
            rc = SRTP_ENOMEM;
            break;
        }
        if (hipMemset(e->d_ctx_keys, 0xff, (size_t)e->ctx_cap * sizeof(uint64_t)) != hipSuccess ||
            hipMemset(e->d_ctx, 0, (size_t)e->ctx_cap * sizeof(CtxState)) != hipSuccess ||
            hipMemset(e->d_far, 0, (size_t)e->ctx_cap * sizeof(uint32_t)) != hipSuccess ||
            hipMemset(e->d_counters, 0, sizeof(unsigned long long) * kCountReplicas * kCtrStride) != hipSuccess) {
            rc = SRTP_EDEVICE;
            break;
        }
        rc = ensure_scratch(e, o.max_batch);
    } while (0);
    if (rc != SRTP_OK) {
        srtp_engine_destroy(e);
        return rc;
    }
    *out = e;
    return SRTP_OK;
}

void srtp_engine_destroy(srtp_engine *e) {
    if (!e) return;
    DeviceGuard guard(e->opts.device);
    (void)quiesce(e);
    if (e->d_keysets) // zero session keys before release
        (void)hipMemset(e->d_keysets, 0, (size_t)e->max_keysets * sizeof(KeySet));
    if (e->d_extkeys)
        (void)hipMemset(e->d_extkeys, 0, (size_t)e->max_keysets * sizeof(ExtKeys));
    if (e->d_tfkeys)
        (void)hipMemset(e->d_tfkeys, 0, 2 * (size_t)e->max_keysets * sizeof(TwofishKeys));
    if (e->d_skkeys)
        (void)hipMemset(e->d_skkeys, 0, (size_t)e->max_keysets * sizeof(SkeinKeys));
    free_scratch(e);
    for (auto &m : e->marks) {
        (void)hipEventDestroy(m.a);
        (void)hipEventDestroy(m.b);
    }
    for (auto ev : e->event_pool) (void)hipEventDestroy(ev);
    void *ptrs[] = {e->d_keysets, e->d_extkeys, e->d_tfkeys, e->d_skkeys, e->d_factories, e->d_transformers, e->d_ctx_keys, e->d_ctx,
                    e->d_far, e->e_min, e->ctl, e->d_count, e->d_counters, e->h_seg, e->h_off, e->h_len,
                    e->h_cap, e->h_flags, e->h_status, e->h_tids};
    for (void *p : ptrs) dfree(p);
    if (e->ev_last) (void)hipEventDestroy(e->ev_last);
    if (e->ev_dev) (void)hipEventDestroy(e->ev_dev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

const char *srtp_engine_last_error(srtp_engine *e) { return e ? e->last_error.c_str() : ""; }

int srtp_factory_create(srtp_engine *e, int32_t sender, const uint8_t *mk, int32_t key_len,
                        const uint8_t *ms, int32_t salt_len, const srtp_policy *srtp_pol,
                        const srtp_policy *srtcp_pol, int32_t *out) {
    if (!e || !out || !mk || !ms) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    // NULL-cipher profiles keep a 16-B master key + 14-B salt for the RFC 3711
    // 4.3 PRF (the reference throws there: SURVEY Q15) -- parity unpinned.
    if (!policy_ok(srtp_pol, false) || !policy_ok(srtcp_pol, true))
        return fail(e, SRTP_EPOLICY, "unsupported SRTP policy");
    if (key_len < std::max(master_key_len(srtp_pol), master_key_len(srtcp_pol)) || salt_len < 14)
        return fail(e, SRTP_EPOLICY, "master key / salt shorter than the policy");
    if (e->factories.size() >= e->opts.max_factories || e->n_keysets + 2 > e->max_keysets)
        return fail(e, SRTP_EFULL, "factory table full");
    KeySet ks[2];
    ExtKeys f8[2];
    std::vector<TwofishKeys> tf(4);
    SkeinKeys sk[2];
    build_keyset(mk, ms, false, srtp_pol, &ks[0], &f8[0], &tf[0], &sk[0]);
    build_keyset(mk, ms, true, srtcp_pol, &ks[1], &f8[1], &tf[2], &sk[1]);
    const bool any_skein = srtp_pol->auth_type == SRTP_SKEIN_AUTHENTICATION ||
                           srtcp_pol->auth_type == SRTP_SKEIN_AUTHENTICATION;
    if (any_skein) {
        if (!e->d_skkeys && dalloc(&e->d_skkeys, (size_t)e->max_keysets) != hipSuccess) {
            memset(sk, 0, sizeof sk);
            return fail(e, SRTP_ENOMEM, "Skein key table");
        }
        HIPCHK(e, hipMemcpy(e->d_skkeys + e->n_keysets, sk, sizeof sk, hipMemcpyHostToDevice));
        memset(sk, 0, sizeof sk);
        e->n_skein += (uint32_t)((srtp_pol->auth_type == SRTP_SKEIN_AUTHENTICATION) +
                                 (srtcp_pol->auth_type == SRTP_SKEIN_AUTHENTICATION));
    }
    if (is_twofish(srtp_pol->enc_type) || is_twofish(srtcp_pol->enc_type)) {
        if (!e->d_tfkeys && dalloc(&e->d_tfkeys, 2 * (size_t)e->max_keysets) != hipSuccess) {
            std::fill(tf.begin(), tf.end(), TwofishKeys{});
            return fail(e, SRTP_ENOMEM, "Twofish key table");
        }
        HIPCHK(e, hipMemcpy(e->d_tfkeys + 2 * (size_t)e->n_keysets, tf.data(), 4 * sizeof(TwofishKeys),
                            hipMemcpyHostToDevice));
    }
    std::fill(tf.begin(), tf.end(), TwofishKeys{});
    HIPCHK(e, hipMemcpy(e->d_keysets + e->n_keysets, ks, sizeof ks, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_extkeys + e->n_keysets, f8, sizeof f8, hipMemcpyHostToDevice));
    e->n_ext += (uint32_t)(ks[0].ext + ks[1].ext);
    for (const KeySet &k : ks)
        e->n_not_wide += (k.ext || k.auth_type != SRTP_HMACSHA1_AUTHENTICATION ||
                          (k.enc_type != SRTP_AESCM_ENCRYPTION && k.enc_type != SRTP_NULL_ENCRYPTION))
                             ? 1u : 0u;
    memset(ks, 0, sizeof ks);
    memset(f8, 0, sizeof f8);
    FactoryRec f;
    f.open = 1;
    f.ks_rtp = (int32_t)e->n_keysets;
    f.ks_rtcp = (int32_t)e->n_keysets + 1;
    f.sender = sender;
    e->n_keysets += 2;
    e->factories.push_back(f);
    e->f_rtcp_tag.push_back(srtcp_pol->auth_tag_len);
    int32_t id = (int32_t)e->factories.size() - 1;
    int rc = sync_factory(e, id);
    if (rc != SRTP_OK) return rc;
    *out = id;
    return SRTP_OK;
}

int srtp_factory_close(srtp_engine *e, int32_t factory) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    int rc = quiesce(e); // enqueued bundles may still read the factory record
    if (rc != SRTP_OK) return rc;
    return close_factory_locked(e, factory);
}

int srtp_transformer_create(srtp_engine *e, int32_t kind, int32_t fwd, int32_t rev, int32_t *out) {
    if (!e || !out) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    if (kind != SRTP_KIND_RTP && kind != SRTP_KIND_RTCP) return fail(e, SRTP_EINVAL, "bad kind");
    if (fwd < 0 || (size_t)fwd >= e->factories.size() || rev < 0 ||
        (size_t)rev >= e->factories.size())
        return fail(e, SRTP_EINVAL, "bad factory id");
    if (e->transformers.size() >= e->opts.max_transformers)
        return fail(e, SRTP_EFULL, "transformer table full");
    TransformerRec t;
    t.kind = kind; t.fwd = fwd; t.rev = rev; t.alive = 1;
    e->transformers.push_back(t);
    int32_t id = (int32_t)e->transformers.size() - 1;
    int rc = sync_transformer(e, id);
    if (rc != SRTP_OK) return rc;
    *out = id;
    return SRTP_OK;
}

int srtp_transformer_set_factory(srtp_engine *e, int32_t t, int32_t f, int32_t forward) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (t < 0 || (size_t)t >= e->transformers.size() || f < 0 || (size_t)f >= e->factories.size())
        return fail(e, SRTP_EINVAL, "bad id");
    GUARD(e);
    int qrc = quiesce(e); // enqueued bundles read the transformer and factory records
    if (qrc != SRTP_OK) return qrc;
    int32_t &slot = forward ? e->transformers[t].fwd : e->transformers[t].rev;
    if (slot >= 0 && slot != f) {
        int rc = close_factory_locked(e, slot);
        if (rc != SRTP_OK) return rc;
    }
    slot = f;
    return sync_transformer(e, t);
}

int srtp_transformer_info(srtp_engine *e, int32_t t, int32_t *kind, int32_t *fwd_rtcp_tag_len) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (t < 0 || (size_t)t >= e->transformers.size()) return fail(e, SRTP_EINVAL, "bad id");
    const TransformerRec &tr = e->transformers[(size_t)t];
    if (kind) *kind = tr.kind;
    if (fwd_rtcp_tag_len) *fwd_rtcp_tag_len = tr.fwd >= 0 ? e->f_rtcp_tag[(size_t)tr.fwd] : 0;
    return SRTP_OK;
}

int srtp_transformer_close(srtp_engine *e, int32_t t) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (t < 0 || (size_t)t >= e->transformers.size()) return fail(e, SRTP_EINVAL, "bad id");
    GUARD(e);
    int rc = quiesce(e); // enqueued bundles may still walk this transformer's contexts
    if (rc != SRTP_OK) return rc;
    TransformerRec &tr = e->transformers[t];
    rc = close_factory_locked(e, tr.fwd);
    if (rc != SRTP_OK) return rc;
    if (tr.rev != tr.fwd) {
        rc = close_factory_locked(e, tr.rev);
        if (rc != SRTP_OK) return rc;
    }
    HIPCHK(e, launch_remove_transformer(e->d_ctx_keys, e->d_ctx, e->ctx_cap, (uint32_t)t, e->stream));
    HIPCHK(e, hipStreamSynchronize(e->stream));
    // Tombstones from repeated closes (a DTLS rekey closes the old transformer)
    // are reused by inserts; rebuild once they hold a quarter of the table.
    uint64_t live = 0, tomb = 0;
    rc = count_slots(e, &live, &tomb);
    if (rc != SRTP_OK) return rc;
    if (tomb > e->ctx_cap / 4) return rehash(e, live);
    return SRTP_OK;
}

// A bundle of up to kSmallMaxN packets under the split path's key-set rule
// runs every phase in one launch (k_small), unless a debug hook needs the
// multi-kernel chain.
static bool small_path(const srtp_engine *e, uint32_t n) {
    const bool wide_ok = e->n_not_wide == 0 && !(e->dbg & SRTP_DEBUG_NO_WIDE);
    return wide_ok && n <= kSmallMaxN && !(e->dbg & SRTP_DEBUG_FORCE_CHAIN_STALL) &&
           !(e->dbg & (SRTP_DEBUG_FORCE_WIDE | SRTP_DEBUG_NO_SMALL));
}

// abort: SinglePacketTransformer's abort-on-throw for this bundle (-1: the
// engine's abort_on_error; 0: every packet is its own 1-element array)
// pk_host: k_small's direct mode (BundleArgs::pk_host); only for a bundle
// small_path takes
static int transform_locked(srtp_engine *e, int32_t reverse, const int32_t *tids, int32_t tid,
                            uint8_t *seg, const uint32_t *off, uint32_t *len, const uint32_t *cap,
                            const uint32_t *flags, int32_t *status, uint32_t n, hipStream_t s,
                            int32_t abort = -1, bool dev_event = false, const uint8_t *pk_host = nullptr,
                            uint8_t *pk_dev = nullptr, uint32_t pk_bytes = 0) {
    if (n == 0) return SRTP_OK;
    if (!seg || !off || !len || !cap || !status) return fail(e, SRTP_EINVAL, "null buffer");
    if (n > kRecIdxMask) return fail(e, SRTP_EINVAL, "bundle too large");
    if (!tids && (tid < 0 || (size_t)tid >= e->transformers.size()))
        return fail(e, SRTP_EINVAL, "bad transformer id");
    int rc = ensure_scratch(e, n);
    if (rc != SRTP_OK) return rc;
    // bundles of one engine share its scratch and run in submission order: a
    // bundle on another stream than the previous one waits for it on the device
    if (e->have_last && e->last_stream != s) HIPCHK(e, hipStreamWaitEvent(s, last_event(e), 0));
    BundleArgs a{};
    a.keysets = e->d_keysets;
    a.extkeys = e->d_extkeys;
    a.tfkeys = e->d_tfkeys;
    a.skkeys = e->d_skkeys;
    a.has_skein = e->n_skein ? 1 : 0;
    a.factories = e->d_factories;
    a.transformers = e->d_transformers;
    a.ctx_keys = e->d_ctx_keys;
    a.ctx = e->d_ctx;
    a.ctx_mask = e->ctx_cap - 1;
    a.far = e->d_far;
    a.n_transformers = (uint32_t)e->transformers.size();
    a.seg = seg; a.off = off; a.len = len; a.cap = cap; a.flags = flags; a.status = status;
    a.tids = tids; a.tid = tid; a.n = n;
    a.reverse = reverse ? 1 : 0;
    a.check_replay = e->opts.check_replay;
    a.abort_on_error = abort < 0 ? e->opts.abort_on_error : (abort ? 1 : 0);
    a.serial = e->serial++;
    a.dbg = e->dbg & SRTP_DEBUG_FORCE_CHAIN_STALL; // the kernels' hook (kDbgForceStall)
    a.counters = e->d_counters;
#ifdef SRTP_STAMPS
    if (!e->d_stamps[reverse ? 1 : 0])
        HIPCHK(e, hipMalloc(&e->d_stamps[reverse ? 1 : 0], (size_t)(1u << 20) * 8 * 8));
    a.stamps = e->d_stamps[reverse ? 1 : 0];
#endif
    a.p_slot = e->p_slot; a.sk_in = e->sk_in; a.sk_out = e->sk_out;
    a.sv_in = e->sv_in; a.sv_out = e->sv_out;
    a.w_status = e->w_status; a.w_cw = e->w_cw; a.w_len = e->w_len;
    a.gok = e->gok; a.mid = e->mid;
    a.tailc = e->tailc; a.spec = e->spec;
    a.tile_link = e->tile_link;
    a.spos = e->spos;
    a.lord = e->lord;
    a.cls_tile = e->cls_tile;
    const SortScratch ss = sort_scratch(e->sort_temp, e->scratch_n);
    // keys: slot or ctx_cap (= not walked), ctx_bits + 1 bits: 8-bit digits up
    // to 16 bits, two 9-11-bit digits up to 22 (the wide sort), else 8-bit again
    // 17-19 bits: an 8-bit pass and one wide pass (hybrid); 20-22: two wide
    // passes (profiles/r04/kernel_experiments.md 8)
    const int key_bits = e->ctx_bits + 1;
    const bool big = key_bits > 16 && key_bits <= 2 * kSortWideMaxBits;
    const bool hybrid = big && key_bits <= 8 + kSortWideMaxBits;
    const bool wide = big && !hybrid;
    a.sort_key_bits = key_bits;
    a.sort_hi_bits = hybrid ? key_bits - 8 : 0;
    a.sort_passes = big ? 2 : (key_bits + 7) / 8;
    a.sort_bits = wide ? (key_bits + 1) / 2 : 8;
    a.sort_counts = wide ? ss.wcounts[0] : ss.counts[0];
    // the walk re-zeroes the 8-bit sort's last counts, and the hybrid's first
    // (k_parse's); the wide sort's k_sort_prefix zeroes its own (the walk then
    // clears a prefix table that is rewritten before its next use)
    a.sort_zero = wide ? ss.wprefix : hybrid ? ss.counts[0] : ss.counts[a.sort_passes - 1];
    a.sort_zero_words = ((n + sort_tile_records() - 1u) / sort_tile_records()) * 256u; // tiles of this bundle x 256 digits
    // a small bundle's AES-CM keystream by k_ctr_small (a lane per counter-block
    // pair; the fused kernels only MAC): up to 8192 packets (128 waves: under
    // one wave per SIMD; profiles/r04/kernel_experiments.md 9)
    // Mid-size bundles of engines whose key sets are all AES-CM / NULL cipher +
    // HMAC-SHA1 take the split path (k_ctr_wide + k_mac_wide, srtp_kernels.hip),
    // the rest the fused kernels (with k_ctr_small up to kSmallCtrMax packets).
    const bool wide_ok = e->n_not_wide == 0 && !(e->dbg & SRTP_DEBUG_NO_WIDE);
    const bool split = wide_ok && ((n >= kWideMin && n <= kWideMax) || (e->dbg & SRTP_DEBUG_FORCE_WIDE));
    const bool small = small_path(e, n);
    if (pk_host && !small) return fail(e, SRTP_EINVAL, "direct mode without k_small");
    a.pk_host = small ? pk_host : nullptr;
    a.pk_dev = pk_dev;
    a.pk_bytes = pk_bytes;
    a.small_ctr = split || small ? 2 : n <= kSmallCtrMax ? 1 : 0;
    const int c = e->ctl_cur;
    const size_t nt_max = e->opts.max_transformers;
    a.ctl = e->ctl + c;
    a.e_min = e->e_min + c * nt_max;
    a.ctl_next = e->ctl + (c ^ 1);
    a.e_min_next = e->e_min + (c ^ 1) * nt_max;
    const bool need_ctl = !e->ctl_clean[c];
    const bool need_emin = a.abort_on_error && e->emin_filled[c] < a.n_transformers;
    e->ctl_clean[c] = false; // this bundle's atomics dirty it
    // e_min is written (and the next bundle's reset by k_parse) only by bundles
    // with abort-on-throw; a bundle without it leaves both tables as they are
    if (a.abort_on_error) e->emin_filled[c] = 0u;
    if (need_ctl) HIPCHK(e, hipMemsetAsync(a.ctl, 0, sizeof(BundleCtl), s));
    if (need_emin) HIPCHK(e, hipMemsetAsync(a.e_min, 0x7f, sizeof(int32_t) * a.n_transformers, s));
    if (small) {
        StageTimer t(e, s, a.reverse ? SRTP_STAGE_VERIFY : SRTP_STAGE_PROTECT);
        HIPCHK(e, launch_small(a, s)); // also resets control block c ^ 1 (and e_min c ^ 1)
        e->ctl_clean[c ^ 1] = true;
        if (a.abort_on_error) e->emin_filled[c ^ 1] = a.n_transformers;
        e->ctl_cur = c ^ 1;
        e->n_small++;
    } else {
    // a one-tile bundle is sorted by one workgroup in one launch
    const bool one_tile = n <= sort_tile_records();
    {
        StageTimer t(e, s, SRTP_STAGE_PARSE);
        // also resets control block c ^ 1
        HIPCHK(e, launch_parse(a, s));
    }
    e->ctl_clean[c ^ 1] = true;
    if (a.abort_on_error) e->emin_filled[c ^ 1] = a.n_transformers;
    e->ctl_cur = c ^ 1;
    {
        StageTimer t(e, s, SRTP_STAGE_SORT);
        HIPCHK(e, one_tile ? launch_sort_tile(a, s) : launch_sort(a, ss, s));
    }
    if (a.reverse && a.small_ctr == 2) {
        StageTimer t(e, s, SRTP_STAGE_VERIFY);
        HIPCHK(e, launch_mac_wide(a, s)); // tag check under the ROC guess, no decryption yet
    } else if (a.reverse) {
        StageTimer t(e, s, SRTP_STAGE_VERIFY);
        HIPCHK(e, launch_unprotect(a, s));
        if (a.small_ctr) HIPCHK(e, launch_ctr_small(a, s)); // the speculative decryption
        if (e->n_skein) HIPCHK(e, launch_skein(a, s));
    }
    {
        StageTimer t(e, s, SRTP_STAGE_WALK);
        HIPCHK(e, launch_walk(a, 0, s));
        // second pass: abort-on-throw's limit pass when a packet may throw,
        // else the wave-parallel walk of context chains longer than the
        // first pass's window (returns at once when there are none) -- which a
        // bundle of fewer than kLongMin packets cannot hold: a small bundle
        // without abort-on-throw saves the launch
        if (a.abort_on_error || n >= kLongMin || a.dbg) HIPCHK(e, launch_walk(a, 1, s));
    }
    if (a.reverse && a.small_ctr == 2) {
        StageTimer t(e, s, SRTP_STAGE_DECRYPT);
        HIPCHK(e, launch_ctr_wide(a, s)); // final statuses, decryption under the walk's ROC
    } else if (a.small_ctr == 2) {
        StageTimer t(e, s, SRTP_STAGE_PROTECT);
        HIPCHK(e, launch_ctr_wide(a, s)); // the keystream, then the MAC and trailer
        HIPCHK(e, launch_mac_wide(a, s));
    } else if (a.reverse) {
        StageTimer t(e, s, SRTP_STAGE_DECRYPT);
        HIPCHK(e, launch_unprotect_fix(a, s));
        if (e->n_ext) HIPCHK(e, launch_ext(a, s));
    } else {
        StageTimer t(e, s, SRTP_STAGE_PROTECT);
        if (a.small_ctr) HIPCHK(e, launch_ctr_small(a, s)); // the keystream, then k_protect MACs
        HIPCHK(e, launch_protect(a, s));
        if (e->n_ext) HIPCHK(e, launch_ext(a, s));
        if (e->n_skein) HIPCHK(e, launch_skein(a, s));
    }
    }
    HIPCHK(e, hipEventRecord(dev_event ? e->ev_dev : e->ev_last, s));
    e->last_dev = dev_event;
    e->last_stream = s;
    e->have_last = true;
    e->n_bundles++;
    e->n_packets += n;
    return SRTP_OK;
}

int srtp_transform_device(srtp_engine *e, int32_t reverse, const int32_t *tids, int32_t tid,
                          uint8_t *seg, const uint32_t *off, uint32_t *len, const uint32_t *cap,
                          const uint32_t *flags, int32_t *status, uint32_t n, void *stream) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    // NULL = the device's default (null) stream, ordered with the caller's
    // other default-stream work (torch's default stream is NULL too); callers
    // that want the two directions to overlap pass each engine's own stream
    // (srtp_engine_stream: one hardware queue per engine)
    hipStream_t s = (hipStream_t)stream;
    return transform_locked(e, reverse, tids, tid, seg, off, len, cap, flags, status, n, s, -1, true);
}

// Every packet region [off, off + cap rounded to 16) inside the segment,
// 16-B aligned, cap <= 65535 (the kernels' 16-bit length fields).
static int validate_regions(srtp_engine *e, const uint32_t *off, const uint32_t *cap, uint32_t n,
                            size_t seg_bytes) {
    for (uint32_t i = 0; i < n; i++) {
        if (off[i] % 16 != 0) return fail(e, SRTP_EINVAL, "off[i] must be 16-byte aligned");
        uint64_t end = (uint64_t)off[i] + ((cap[i] + 15u) & ~15u);
        if (cap[i] > 65535u || end > seg_bytes)
            return fail(e, SRTP_EINVAL, "packet region outside the segment");
    }
    return SRTP_OK;
}

int srtp_transform_host(srtp_engine *e, int32_t reverse, const int32_t *tids, int32_t tid,
                        uint8_t *seg, size_t seg_bytes, const uint32_t *off, uint32_t *len,
                        const uint32_t *cap, const uint32_t *flags, int32_t *status, uint32_t n) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (n == 0) return SRTP_OK;
    if (!seg || !off || !len || !cap || !status) return fail(e, SRTP_EINVAL, "null buffer");
    int vr = validate_regions(e, off, cap, n, seg_bytes);
    if (vr != SRTP_OK) return vr;
    GUARD(e);
    hipStream_t s = e->stream;
    size_t need = (seg_bytes + 15) & ~(size_t)15;
    if ((need > e->h_seg_bytes || n > e->h_n) && e->have_last) {
        // the staging buffers may still be in use by an enqueued bundle
        int qrc = quiesce(e);
        if (qrc != SRTP_OK) return qrc;
    }
    if (need > e->h_seg_bytes) {
        dfree(e->h_seg);
        e->h_seg = nullptr;
        HIPCHK(e, hipMalloc(&e->h_seg, need));
        e->h_seg_bytes = need;
    }
    if (n > e->h_n) {
        void *ptrs[] = {e->h_off, e->h_len, e->h_cap, e->h_flags, e->h_status, e->h_tids};
        for (void *p : ptrs) dfree(p);
        HIPCHK(e, dalloc(&e->h_off, n));
        HIPCHK(e, dalloc(&e->h_len, n));
        HIPCHK(e, dalloc(&e->h_cap, n));
        HIPCHK(e, dalloc(&e->h_flags, n));
        HIPCHK(e, dalloc(&e->h_status, n));
        HIPCHK(e, dalloc(&e->h_tids, n));
        e->h_n = n;
    }
    HIPCHK(e, hipMemcpyAsync(e->h_seg, seg, seg_bytes, hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->h_off, off, n * 4ull, hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->h_len, len, n * 4ull, hipMemcpyHostToDevice, s));
    HIPCHK(e, hipMemcpyAsync(e->h_cap, cap, n * 4ull, hipMemcpyHostToDevice, s));
    if (flags) HIPCHK(e, hipMemcpyAsync(e->h_flags, flags, n * 4ull, hipMemcpyHostToDevice, s));
    if (tids) HIPCHK(e, hipMemcpyAsync(e->h_tids, tids, n * 4ull, hipMemcpyHostToDevice, s));
    int rc = transform_locked(e, reverse, tids ? e->h_tids : nullptr, tid, e->h_seg, e->h_off,
                              e->h_len, e->h_cap, flags ? e->h_flags : nullptr, e->h_status, n, s);
    if (rc != SRTP_OK) return rc;
    HIPCHK(e, hipMemcpyAsync(seg, e->h_seg, seg_bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipMemcpyAsync(len, e->h_len, n * 4ull, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipMemcpyAsync(status, e->h_status, n * 4ull, hipMemcpyDeviceToHost, s));
    HIPCHK(e, hipStreamSynchronize(s));
    return SRTP_OK;
}

void *srtp_engine_stream(srtp_engine *e) { return e ? (void *)e->stream : nullptr; }

int srtp_engine_sync(srtp_engine *e, void *stream) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    if (!stream) return quiesce(e); // every bundle of this engine, whatever its stream
    HIPCHK(e, hipStreamSynchronize((hipStream_t)stream));
    return e->have_last && e->last_stream == (hipStream_t)stream ? fence_to_host(e, (hipStream_t)stream) : SRTP_OK;
}

int srtp_get_context_state(srtp_engine *e, int32_t t, uint32_t ssrc, srtp_ctx_state *out) {
    if (!e || !out) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    int qrc = quiesce(e);
    if (qrc != SRTP_OK) return qrc;
    uint64_t key = ((uint64_t)(uint32_t)t << 32) | ssrc;
    uint32_t mask = e->ctx_cap - 1;
    uint32_t h = (uint32_t)mix64_host(key) & mask;
    for (uint32_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        uint64_t k;
        HIPCHK(e, hipMemcpy(&k, e->d_ctx_keys + h, 8, hipMemcpyDeviceToHost));
        if (k == kEmptyKey) return 0;
        if (k != key) continue;
        CtxState s;
        HIPCHK(e, hipMemcpy(&s, e->d_ctx + h, sizeof s, hipMemcpyDeviceToHost));
        KeySet ks;
        HIPCHK(e, hipMemcpy(&ks, e->d_keysets + s.ks, sizeof ks, hipMemcpyDeviceToHost));
        memset(out, 0, sizeof *out);
        out->key_set = s.ks;
        out->replay_window = s.window;
        if (ks.kind == SRTP_KIND_RTP) {
            out->roc = s.a; out->s_l = s.b; out->seq_num_set = (int32_t)(s.flags & 1u);
            out->guessed_roc = s.g;
        } else {
            out->sent_index = s.a; out->received_index = s.b;
        }
        memset(&ks, 0, sizeof ks);
        return 1;
    }
    return 0;
}

static void fill_state(const CtxState &s, const KeySet &ks, srtp_ctx_state *out) {
    memset(out, 0, sizeof *out);
    out->key_set = s.ks;
    out->replay_window = s.window;
    if (ks.kind == SRTP_KIND_RTP) {
        out->roc = s.a; out->s_l = s.b; out->seq_num_set = (int32_t)(s.flags & 1u);
        out->guessed_roc = s.g;
    } else {
        out->sent_index = s.a; out->received_index = s.b;
    }
}

int srtp_export_contexts(srtp_engine *e, int32_t t, uint32_t *ssrcs, srtp_ctx_state *states,
                         uint32_t max, uint32_t *count) {
    if (!e || !count || (max && (!ssrcs || !states))) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (t < 0 || (size_t)t >= e->transformers.size()) return fail(e, SRTP_EINVAL, "bad transformer id");
    GUARD(e);
    int qrc = quiesce(e);
    if (qrc != SRTP_OK) return qrc;
    std::vector<uint64_t> keys(e->ctx_cap);
    std::vector<CtxState> ctx(e->ctx_cap);
    HIPCHK(e, hipMemcpy(keys.data(), e->d_ctx_keys, keys.size() * 8, hipMemcpyDeviceToHost));
    HIPCHK(e, hipMemcpy(ctx.data(), e->d_ctx, ctx.size() * sizeof(CtxState), hipMemcpyDeviceToHost));
    std::vector<KeySet> ks(e->n_keysets);
    if (!ks.empty())
        HIPCHK(e, hipMemcpy(ks.data(), e->d_keysets, ks.size() * sizeof(KeySet), hipMemcpyDeviceToHost));
    uint32_t n = 0;
    for (uint32_t h = 0; h < e->ctx_cap; h++) {
        const uint64_t k = keys[h];
        if (k == kEmptyKey || k == kTombKey || (int32_t)(k >> 32) != t) continue;
        if (n < max) {
            ssrcs[n] = (uint32_t)k;
            fill_state(ctx[h], ks[ctx[h].ks], &states[n]);
        }
        n++;
    }
    for (auto &x : ks) memset(&x, 0, sizeof x);
    *count = n;
    return SRTP_OK;
}

int srtp_set_context_state(srtp_engine *e, int32_t t, uint32_t ssrc, int32_t forward,
                           const srtp_ctx_state *st) {
    if (!e || !st) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (t < 0 || (size_t)t >= e->transformers.size()) return fail(e, SRTP_EINVAL, "bad transformer id");
    const TransformerRec &tr = e->transformers[t];
    if (!tr.alive) return fail(e, SRTP_EINVAL, "transformer closed");
    const int32_t f = forward ? tr.fwd : tr.rev;
    if (f < 0 || !e->factories[f].open) return fail(e, SRTP_EPOLICY, "factory closed");
    CtxState s{};
    s.ks = (uint32_t)(tr.kind == SRTP_KIND_RTP ? e->factories[f].ks_rtp : e->factories[f].ks_rtcp);
    s.window = st->replay_window;
    if (tr.kind == SRTP_KIND_RTP) {
        s.a = st->roc; s.b = st->s_l; s.g = st->guessed_roc; s.flags = st->seq_num_set ? 1u : 0u;
    } else {
        s.a = st->sent_index; s.b = st->received_index;
    }
    s.birth = 0;
    GUARD(e);
    int qrc = quiesce(e);
    if (qrc != SRTP_OK) return qrc;
    const uint64_t key = ((uint64_t)(uint32_t)t << 32) | ssrc;
    const uint32_t mask = e->ctx_cap - 1;
    uint32_t h = (uint32_t)mix64_host(key) & mask, free_slot = kNoSlot;
    for (uint32_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        uint64_t k;
        HIPCHK(e, hipMemcpy(&k, e->d_ctx_keys + h, 8, hipMemcpyDeviceToHost));
        if (k == key) { free_slot = h; break; }
        if (k == kTombKey && free_slot == kNoSlot) free_slot = h; // reuse, but keep probing for key
        if (k == kEmptyKey) { if (free_slot == kNoSlot) free_slot = h; break; }
    }
    if (free_slot == kNoSlot) return fail(e, SRTP_EFULL, "context table full");
    HIPCHK(e, hipMemcpy(e->d_ctx + free_slot, &s, sizeof s, hipMemcpyHostToDevice));
    HIPCHK(e, hipMemcpy(e->d_ctx_keys + free_slot, &key, 8, hipMemcpyHostToDevice));
    return SRTP_OK;
}

// Snapshot / restore of (transformer, SSRC) contexts by key, on the device
// (k_ctx_save / k_ctx_restore): one small kernel and two copies per call.
static int contexts_io(srtp_engine *e, bool restore, uint32_t n, const int32_t *tids,
                       const uint32_t *ssrcs, srtp_ctx_raw *out, const srtp_ctx_raw *in,
                       int32_t *present_out, const int32_t *present_in) {
    static_assert(sizeof(srtp_ctx_raw) == sizeof(CtxState), "srtp_ctx_raw holds one CtxState");
    if (n == 0) return SRTP_OK;
    std::vector<uint64_t> keys(n);
    for (uint32_t i = 0; i < n; i++) keys[i] = ((uint64_t)(uint32_t)tids[i] << 32) | ssrcs[i];
    GUARD(e);
    int rc = quiesce(e);
    if (rc != SRTP_OK) return rc;
    uint64_t *d_keys = nullptr;
    CtxState *d_st = nullptr;
    int32_t *d_pr = nullptr;
    unsigned int *d_fail = nullptr;
    unsigned int failed = 0;
    hipStream_t s = e->stream;
    do {
        if (dalloc(&d_keys, n) != hipSuccess || dalloc(&d_st, n) != hipSuccess ||
            dalloc(&d_pr, n) != hipSuccess || dalloc(&d_fail, 1) != hipSuccess) {
            rc = fail(e, SRTP_ENOMEM, "context snapshot scratch");
            break;
        }
        bool ok = hipMemcpyAsync(d_keys, keys.data(), n * 8ull, hipMemcpyHostToDevice, s) == hipSuccess;
        if (restore) {
            ok = ok && hipMemcpyAsync(d_st, in, n * sizeof(CtxState), hipMemcpyHostToDevice, s) == hipSuccess &&
                 hipMemcpyAsync(d_pr, present_in, n * 4ull, hipMemcpyHostToDevice, s) == hipSuccess &&
                 hipMemsetAsync(d_fail, 0, 4, s) == hipSuccess &&
                 launch_ctx_restore(e->d_ctx_keys, e->d_ctx, e->ctx_cap - 1, d_keys, n, d_st, d_pr, d_fail, s) ==
                     hipSuccess &&
                 hipMemcpyAsync(&failed, d_fail, 4, hipMemcpyDeviceToHost, s) == hipSuccess;
        } else {
            ok = ok && launch_ctx_save(e->d_ctx_keys, e->d_ctx, e->ctx_cap - 1, d_keys, n, d_st, d_pr, s) ==
                           hipSuccess &&
                 hipMemcpyAsync(out, d_st, n * sizeof(CtxState), hipMemcpyDeviceToHost, s) == hipSuccess &&
                 hipMemcpyAsync(present_out, d_pr, n * 4ull, hipMemcpyDeviceToHost, s) == hipSuccess;
        }
        if (!ok || hipStreamSynchronize(s) != hipSuccess) rc = fail(e, SRTP_EDEVICE, "context snapshot");
        else if (failed) rc = fail(e, SRTP_EFULL, "context table full on restore");
    } while (0);
    if (d_st) (void)hipMemsetAsync(d_st, 0, n * sizeof(CtxState), s); // no key material is kept, but no state either
    (void)hipStreamSynchronize(s);
    dfree(d_keys);
    dfree(d_st);
    dfree(d_pr);
    dfree(d_fail);
    return rc;
}

int srtp_contexts_save(srtp_engine *e, uint32_t n, const int32_t *tids, const uint32_t *ssrcs,
                       srtp_ctx_raw *out, int32_t *present) {
    if (!e || (n && (!tids || !ssrcs || !out || !present))) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    return contexts_io(e, false, n, tids, ssrcs, out, nullptr, present, nullptr);
}

int srtp_contexts_restore(srtp_engine *e, uint32_t n, const int32_t *tids, const uint32_t *ssrcs,
                          const srtp_ctx_raw *in, const int32_t *present) {
    if (!e || (n && (!tids || !ssrcs || !in || !present))) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    return contexts_io(e, true, n, tids, ssrcs, nullptr, in, nullptr, present);
}

int64_t srtp_engine_num_contexts(srtp_engine *e) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    int rc = quiesce(e);
    if (rc != SRTP_OK) return rc;
    uint64_t live = 0, tomb = 0;
    rc = count_slots(e, &live, &tomb);
    if (rc != SRTP_OK) return rc;
    return (int64_t)live;
}

int srtp_engine_stats(srtp_engine *e, srtp_stats *out) {
    if (!e || !out) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    int rc = quiesce(e);
    if (rc != SRTP_OK) return rc;
    std::vector<unsigned long long> c((size_t)kCountReplicas * kCtrStride);
    HIPCHK(e, hipMemcpy(c.data(), e->d_counters, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost));
    uint64_t sum[kCtrStride] = {0};
    for (int r = 0; r < kCountReplicas; r++)
        for (int k = 0; k < kCtrStride; k++) sum[k] += c[(size_t)r * kCtrStride + k];
    memset(out, 0, sizeof *out);
    out->bundles = e->n_bundles;
    out->packets = e->n_packets;
    for (int k = 0; k < SRTP_NUM_STATUS; k++) out->status[k] = sum[kCtrStatus + k];
    out->roc_rechecks = sum[kCtrRocRecheck];
    out->repaired = sum[kCtrRepaired];
    out->ctx_overflow = sum[kCtrOverflow];
    rc = count_slots(e, &out->ctx_live, &out->ctx_tombstones);
    if (rc != SRTP_OK) return rc;
    out->ctx_slots = e->ctx_cap;
    out->rehashes = e->n_rehash;
    out->chain_stalls = sum[kCtrChainStall];
    out->long_walked = sum[kCtrLongWalked];
    out->holes = sum[kCtrStatus + kStatusHole];
    out->small_bundles = e->n_small;
    return SRTP_OK;
}

int32_t srtp_device_count(void) {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess ? (int32_t)n : 0;
}

int srtp_engine_set_debug(srtp_engine *e, uint32_t flags) {
    if (!e || (flags & ~(SRTP_DEBUG_FORCE_CHAIN_STALL | SRTP_DEBUG_FORCE_WIDE | SRTP_DEBUG_NO_WIDE | SRTP_DEBUG_NO_SMALL)))
        return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    e->dbg = flags;
    return SRTP_OK;
}

int srtp_engine_set_timing(srtp_engine *e, int32_t enable) {
    if (!e) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    e->timing = enable != 0;
    return SRTP_OK;
}

int srtp_engine_read_timing(srtp_engine *e, double *ms, uint64_t *count) {
    if (!e || !ms || !count) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    for (int i = 0; i < SRTP_NUM_STAGES; i++) { ms[i] = 0.0; count[i] = 0; }
    for (auto &m : e->marks) {
        HIPCHK(e, hipEventSynchronize(m.b));
        float t = 0.f;
        HIPCHK(e, hipEventElapsedTime(&t, m.a, m.b));
        ms[m.stage] += t;
        count[m.stage] += 1;
        e->event_pool.push_back(m.a);
        e->event_pool.push_back(m.b);
    }
    e->marks.clear();
    return SRTP_OK;
}

#ifdef SRTP_STAMPS
// Diagnostic build only (tools/stamps.sh): per-wave stamps of the last
// k_protect (reverse = 0) / k_unprotect (reverse = 1) launch.
int srtp_debug_stamps(srtp_engine *e, int32_t reverse, unsigned long long *out, uint32_t waves) {
    if (!e || !out || !e->d_stamps[reverse ? 1 : 0]) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(e->mu);
    GUARD(e);
    int rc = quiesce(e);
    if (rc != SRTP_OK) return rc;
    HIPCHK(e, hipMemcpy(out, e->d_stamps[reverse ? 1 : 0], (size_t)waves * 8 * 8, hipMemcpyDeviceToHost));
    return SRTP_OK;
}
#endif

int srtp_derive_session_keys(const uint8_t mk[16], const uint8_t ms[14], int32_t rtcp,
                             uint8_t enc[16], uint8_t auth[20], uint8_t salt[14]) {
    if (!mk || !ms || !enc || !auth || !salt) return SRTP_EINVAL;
    derive_session_keys(mk, ms, rtcp != 0, enc, auth, salt);
    return SRTP_OK;
}

int srtp_derive_session_keys_n(const uint8_t *mk, int32_t key_len, const uint8_t ms[14], int32_t rtcp,
                               uint8_t *enc, uint8_t auth[20], uint8_t salt[14]) {
    if (!mk || !ms || !enc || !auth || !salt || (key_len != 16 && key_len != 32)) return SRTP_EINVAL;
    derive_session_keys_n(mk, key_len, ms, rtcp != 0, enc, auth, salt);
    return SRTP_OK;
}

int srtp_derive_session_keys_for(int32_t enc_type, const uint8_t *mk, int32_t key_len,
                                 const uint8_t ms[14], int32_t rtcp, uint8_t *enc, uint8_t auth[20],
                                 uint8_t salt[14]) {
    if (!mk || !ms || !enc || !auth || !salt || (key_len != 16 && key_len != 32)) return SRTP_EINVAL;
    derive_session_keys_cipher(is_twofish(enc_type), mk, key_len, ms, rtcp != 0, enc, auth, salt);
    return SRTP_OK;
}

int srtp_derive_session_keys_auth(int32_t enc_type, const uint8_t *mk, int32_t key_len,
                                  const uint8_t ms[14], int32_t rtcp, uint8_t *enc, uint8_t *auth,
                                  int32_t auth_len, uint8_t salt[14]) {
    if (!mk || !ms || !enc || !auth || !salt || (key_len != 16 && key_len != 32) || auth_len < 1 ||
        auth_len > 64)
        return SRTP_EINVAL;
    derive_session_keys_cipher(is_twofish(enc_type), mk, key_len, ms, rtcp != 0, enc, auth, salt,
                               auth_len);
    return SRTP_OK;
}

int srtp_skein512_mac(const uint8_t *key, int32_t key_len, int32_t out_bits, const uint8_t *msg,
                      size_t n, uint8_t *out) {
    if ((!key && key_len) || (!msg && n) || !out || key_len < 0 || out_bits < 1 || out_bits > 512)
        return SRTP_EINVAL;
    skein512_mac(key, key_len, out_bits, msg, n, out);
    return SRTP_OK;
}

int srtp_block_encrypt(int32_t enc_type, const uint8_t *key, int32_t key_len, const uint8_t in[16],
                       uint8_t out[16]) {
    if (!key || !in || !out) return SRTP_EINVAL;
    if (is_twofish(enc_type)) {
        if (key_len != 16 && key_len != 24 && key_len != 32) return SRTP_EINVAL;
        std::vector<TwofishKeys> t(1);
        twofish_schedule(key, key_len, t[0].K, t[0].T);
        twofish_encrypt_block(t[0].K, t[0].T, in, out);
        t[0] = TwofishKeys{};
        return SRTP_OK;
    }
    if (key_len != 16 && key_len != 32) return SRTP_EINVAL;
    uint32_t rk[60];
    const int nr = aes_expand_le(key, key_len, rk);
    aes_encrypt_block_nr(rk, nr, in, out);
    memset(rk, 0, sizeof rk);
    return SRTP_OK;
}

} // extern "C"

extern "C" {

// ------------------------------------------------- registered host memory
namespace {
std::mutex g_reg_mu;
struct RegRange {
    size_t bytes;
    bool owned; // srtp_host_alloc's (hipHostMalloc) rather than registered caller memory
};
std::map<uintptr_t, RegRange> g_reg; // start -> range, disjoint
} // namespace

int srtp_host_register(void *ptr, size_t bytes) {
    if (!ptr || bytes == 0) return SRTP_EINVAL;
    const uintptr_t a = (uintptr_t)ptr;
    if (a + bytes < a) return SRTP_EINVAL;
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.upper_bound(a);
    if (it != g_reg.end() && it->first < a + bytes) return SRTP_EINVAL;
    if (it != g_reg.begin() && std::prev(it)->first + std::prev(it)->second.bytes > a) return SRTP_EINVAL;
    if (hipHostRegister(ptr, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        return SRTP_EDEVICE;
    }
    g_reg[a] = RegRange{bytes, false};
    return SRTP_OK;
}

int srtp_host_alloc(size_t bytes, void **out) {
    if (!out || bytes == 0) return SRTP_EINVAL;
    *out = nullptr;
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        return SRTP_ENOMEM;
    }
    std::lock_guard<std::mutex> g(g_reg_mu);
    g_reg[(uintptr_t)p] = RegRange{bytes, true};
    *out = p;
    return SRTP_OK;
}

int srtp_host_free(void *ptr) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find((uintptr_t)ptr);
    if (it == g_reg.end() || !it->second.owned) return SRTP_EINVAL;
    g_reg.erase(it);
    return hipHostFree(ptr) == hipSuccess ? SRTP_OK : SRTP_EDEVICE;
}

int srtp_host_unregister(void *ptr) {
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.find((uintptr_t)ptr);
    if (it == g_reg.end() || it->second.owned) return SRTP_EINVAL;
    g_reg.erase(it);
    if (hipHostUnregister(ptr) != hipSuccess) {
        (void)hipGetLastError();
        return SRTP_EDEVICE;
    }
    return SRTP_OK;
}

// The device address of registered host memory p (the range's mapping)
static uint8_t *host_device_ptr(uint8_t *p) {
    uintptr_t start;
    {
        std::lock_guard<std::mutex> g(g_reg_mu);
        auto it = g_reg.upper_bound((uintptr_t)p);
        if (it == g_reg.begin()) return nullptr;
        start = std::prev(it)->first;
    }
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, reinterpret_cast<void *>(start), 0) != hipSuccess || !d) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t *>(d) + ((uintptr_t)p - start);
}

int32_t srtp_host_is_registered(const void *ptr, size_t bytes) {
    const uintptr_t a = (uintptr_t)ptr;
    if (!ptr || a + bytes < a) return 0;
    std::lock_guard<std::mutex> g(g_reg_mu);
    auto it = g_reg.upper_bound(a);
    if (it == g_reg.begin()) return 0;
    --it;
    return a + bytes <= it->first + it->second.bytes ? 1 : 0;
}

} // extern "C"

// ------------------------------------------------------------ host pipeline
struct srtp_pipeline {
    srtp_engine *e = nullptr;
    uint32_t max_n = 0;
    size_t max_seg = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    bool one_stream = false; // SRTP_PIPE_ONE_STREAM: copies on the engine's stream (s_in / s_out not owned)
    bool poll_crowded = false; // SRTP_PIPE_POLL_CROWDED
    std::mutex mu;
    struct Slot {
        srtp_pipeline_slot h{};     // pinned host arrays
        uint8_t *d_seg = nullptr;   // device copies
        uint32_t *d_off = nullptr, *d_len = nullptr, *d_cap = nullptr, *d_flags = nullptr;
        int32_t *d_tids = nullptr, *d_status = nullptr;
        // small bundles: the per-packet arrays packed into one block each way
        // (off | cap | flags | tids | len in, len | status out), so a bundle
        // of a few packets costs two copies in and two out instead of six and
        // three -- each copy's fixed cost, not its bytes, is what a small
        // bundle's round trip pays
        uint32_t *h_pack = nullptr, *d_pack = nullptr;
        uint8_t *m_pack = nullptr; // h_pack's device mapping (k_small's direct mode), or null
        // srtp_pipeline_submit_gather: each packet's offset in the caller's
        // registered segment (pinned host copy, device copy)
        uint32_t *h_src = nullptr, *d_src = nullptr;
        uint32_t packed_n = 0;      // the bundle in flight used the packed layout (its n), else 0
        // tiny bundles (kTinySeg bytes): the segment rides in the packed block
        // too -- one copy each way -- and is copied back to tiny_dst on wait
        uint8_t *tiny_dst = nullptr;
        size_t tiny_off = 0, tiny_bytes = 0;
        hipEvent_t ev_in = nullptr, ev_done = nullptr, ev_out = nullptr;
        bool busy = false;
        int rc = SRTP_OK;           // engine return code of the last submit
    };
    std::vector<Slot> slots;
};

// bundles up to this many packets use the packed copies: one H2D for the
// per-packet arrays and one D2H for lengths + statuses instead of five and
// two -- each separate small copy held the copy stream ~30-80 us, which left
// the dispatcher's 32768-packet chunks' H2D idle ~200 us per chunk
// (profiles/r05/dispatch/)
constexpr uint32_t kPackMax = 1u << 15;
constexpr size_t kOneStreamBytes = (size_t)1 << 20; // bundles up to this size copy on the engine's stream
constexpr size_t kTinySeg = (size_t)64 << 10;       // bundles up to this size: one copy each way

static void pipeline_free(srtp_pipeline *pl) {
    DeviceGuard guard(pl->e->opts.device);
    for (auto &sl : pl->slots) {
        if (sl.busy && sl.ev_out) (void)hipEventSynchronize(sl.ev_out);
        void *hp[] = {sl.h.seg, sl.h.off, sl.h.len, sl.h.cap, sl.h.flags, sl.h.tids, sl.h.status};
        for (void *p : hp)
            if (p) (void)hipHostFree(p);
        if (sl.h_pack) (void)hipHostFree(sl.h_pack);
        if (sl.h_src) (void)hipHostFree(sl.h_src);
        void *dp[] = {sl.d_seg, sl.d_off, sl.d_len, sl.d_cap, sl.d_flags, sl.d_tids, sl.d_status, sl.d_pack,
                      sl.d_src};
        for (void *p : dp) dfree(p);
        hipEvent_t ev[] = {sl.ev_in, sl.ev_done, sl.ev_out};
        for (auto x : ev)
            if (x) (void)hipEventDestroy(x);
    }
    if (pl->s_in && !pl->one_stream) (void)hipStreamDestroy(pl->s_in);
    if (pl->s_out && !pl->one_stream) (void)hipStreamDestroy(pl->s_out);
    delete pl;
}

template <class T> static hipError_t halloc(T **p, size_t count) {
    return hipHostMalloc((void **)p, std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault);
}

int srtp_pipeline_create(srtp_engine *e, uint32_t max_packets, size_t max_seg_bytes,
                         int32_t depth, srtp_pipeline **out) {
    return srtp_pipeline_create_ex(e, max_packets, max_seg_bytes, depth, 0u, out);
}

int srtp_pipeline_create_ex(srtp_engine *e, uint32_t max_packets, size_t max_seg_bytes, int32_t depth,
                            uint32_t flags, srtp_pipeline **out) {
    if (!e || !out || depth < 1 || depth > 16 || max_packets == 0 || max_packets > kRecIdxMask ||
        (flags & ~(uint32_t)(SRTP_PIPE_ONE_STREAM | SRTP_PIPE_POLL_CROWDED)))
        return SRTP_EINVAL;
    *out = nullptr;
    srtp_pipeline *pl = new (std::nothrow) srtp_pipeline();
    if (!pl) return SRTP_ENOMEM;
    pl->e = e;
    pl->max_n = max_packets;
    pl->max_seg = (max_seg_bytes + 15) & ~(size_t)15;
    pl->slots.resize((size_t)depth);
    DeviceGuard guard(e->opts.device);
    pl->one_stream = (flags & SRTP_PIPE_ONE_STREAM) != 0;
    pl->poll_crowded = (flags & SRTP_PIPE_POLL_CROWDED) != 0;
    if (pl->one_stream) pl->s_in = pl->s_out = e->stream;
    bool ok = guard.ok && (pl->one_stream || (hipStreamCreateWithFlags(&pl->s_in, hipStreamNonBlocking) == hipSuccess &&
                                              hipStreamCreateWithFlags(&pl->s_out, hipStreamNonBlocking) == hipSuccess));
    for (auto &sl : pl->slots) {
        if (!ok) break;
        const size_t n = max_packets;
        ok = halloc(&sl.h.seg, pl->max_seg) == hipSuccess && halloc(&sl.h.off, n) == hipSuccess &&
             halloc(&sl.h.len, n) == hipSuccess && halloc(&sl.h.cap, n) == hipSuccess &&
             halloc(&sl.h.flags, n) == hipSuccess && halloc(&sl.h.tids, n) == hipSuccess &&
             halloc(&sl.h.status, n) == hipSuccess &&
             dalloc(&sl.d_seg, pl->max_seg) == hipSuccess && dalloc(&sl.d_off, n) == hipSuccess &&
             dalloc(&sl.d_len, n) == hipSuccess && dalloc(&sl.d_cap, n) == hipSuccess &&
             dalloc(&sl.d_flags, n) == hipSuccess && dalloc(&sl.d_tids, n) == hipSuccess &&
             dalloc(&sl.d_status, n) == hipSuccess &&
             hipHostMalloc((void **)&sl.h_pack, (6 * std::min<size_t>(n, kPackMax) + 4 + kTinySeg / 4) * 4,
                           hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
             dalloc(&sl.d_pack, 6 * std::min<size_t>(n, kPackMax) + 4 + kTinySeg / 4) == hipSuccess &&
             halloc(&sl.h_src, std::min<size_t>(n, kPackMax)) == hipSuccess &&
             dalloc(&sl.d_src, std::min<size_t>(n, kPackMax)) == hipSuccess &&
             hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&sl.ev_out, hipEventDisableTiming) == hipSuccess;
        sl.h.seg_cap = pl->max_seg;
        sl.h.max_packets = max_packets;
        if (ok && hipHostGetDevicePointer((void **)&sl.m_pack, sl.h_pack, 0) != hipSuccess) {
            (void)hipGetLastError();
            sl.m_pack = nullptr; // the copies then
        }
    }
    if (!ok) {
        pipeline_free(pl);
        return SRTP_ENOMEM;
    }
    *out = pl;
    return SRTP_OK;
}

void srtp_pipeline_destroy(srtp_pipeline *pl) {
    if (pl) pipeline_free(pl);
}

int srtp_engine_get_opts(srtp_engine *e, srtp_engine_opts *out) {
    if (!e || !out) return SRTP_EINVAL;
    *out = e->opts;
    return SRTP_OK;
}

int srtp_pipeline_slot_get(srtp_pipeline *pl, int32_t slot, srtp_pipeline_slot *out) {
    if (!pl || !out || slot < 0 || (size_t)slot >= pl->slots.size()) return SRTP_EINVAL;
    *out = pl->slots[(size_t)slot].h;
    return SRTP_OK;
}

// How a pipeline waits for a bundle: hipEventSynchronize, which spins on a
// core -- except that a SRTP_PIPE_POLL_CROWDED pipeline polls hipEventQuery,
// yielding the CPU between polls (sleeping 20 us between polls after the
// first), while more than kSpinWaiters threads are waiting on such
// pipelines: 64 callers each spinning on its own 1-packet bundle took the
// host's cores from the threads enqueueing the next bundles (4.7k calls/s,
// p99 82 ms; polling 12.9k, 4.7 ms; profiles/r04/kernel_experiments.md 7 and
// 10).  Other pipelines (aggregator lanes, dispatcher shards: a few waiters)
// always keep the spin's wake-up.
static std::atomic<int> g_crowd{0};
constexpr int kSpinWaiters = 4;

static int wait_event(hipEvent_t ev, bool crowd) {
    struct Crowd {
        bool on;
        int n;
        explicit Crowd(bool c) : on(c), n(c ? g_crowd.fetch_add(1, std::memory_order_relaxed) + 1 : 0) {}
        ~Crowd() {
            if (on) g_crowd.fetch_sub(1, std::memory_order_relaxed);
        }
    } cr(crowd);
    if (cr.n <= kSpinWaiters) return hipEventSynchronize(ev) == hipSuccess ? 0 : -1;
    bool first = true;
    for (;;) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return 0;
        if (q != hipErrorNotReady) return -1;
        if (first) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
        first = false;
    }
}

static int pipeline_wait_locked(srtp_pipeline *pl, srtp_pipeline::Slot &sl) {
    if (!sl.busy) return SRTP_OK;
    sl.busy = false;
    if (wait_event(sl.ev_out, pl->poll_crowded) != 0) return fail(pl->e, SRTP_EDEVICE, "pipeline D2H");
    if (const uint32_t n = sl.packed_n) { // lengths and statuses to the slot's own arrays
        memcpy(sl.h.len, sl.h_pack + 4 * (size_t)n, n * 4ull);
        memcpy(sl.h.status, sl.h_pack + 5 * (size_t)n, n * 4ull);
        sl.packed_n = 0;
    }
    if (sl.tiny_dst) { // a tiny bundle's segment, back where the caller reads it
        memcpy(sl.tiny_dst, reinterpret_cast<const uint8_t *>(sl.h_pack) + sl.tiny_off, sl.tiny_bytes);
        sl.tiny_dst = nullptr;
    }
    return sl.rc;
}

int srtp_pipeline_submit(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                         int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes) {
    return srtp_pipeline_submit_ex(pl, slot, reverse, use_tids, tid, use_flags, n, seg_bytes, -1);
}

// hseg: the bundle's host segment -- the slot's pinned seg, or registered
// caller memory (srtp_pipeline_submit_host)
static int pipeline_submit(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids, int32_t tid,
                           int32_t use_flags, uint32_t n, size_t seg_bytes, int32_t abort_on_error,
                           uint8_t *hseg) {
    if (!pl || slot < 0 || (size_t)slot >= pl->slots.size()) return SRTP_EINVAL;
    std::lock_guard<std::mutex> gp(pl->mu);
    srtp_pipeline::Slot &sl = pl->slots[(size_t)slot];
    srtp_engine *e = pl->e;
    GUARD(e);
    (void)pipeline_wait_locked(pl, sl); // the slot's previous bundle (its status is the caller's)
    if (n > pl->max_n || seg_bytes > pl->max_seg) return fail(e, SRTP_EINVAL, "bundle exceeds the slot");
    if (n == 0) return SRTP_OK;
    seg_bytes = (seg_bytes + 15) & ~(size_t)15;
    std::lock_guard<std::mutex> g(e->mu);
    int rc = validate_regions(e, sl.h.off, sl.h.cap, n, seg_bytes);
    if (rc != SRTP_OK) return rc;
    if (!use_tids && (tid < 0 || (size_t)tid >= e->transformers.size()))
        return fail(e, SRTP_EINVAL, "bad transformer id");
    // a small bundle's copies go on the engine's stream: their fixed cost, not
    // their bytes, is its round trip, and two cross-stream events add to it
    const bool one = pl->one_stream || seg_bytes <= kOneStreamBytes;
    hipStream_t s = e->stream, si = one ? s : pl->s_in, so = one ? s : pl->s_out;
    const int32_t abort = abort_on_error < 0 ? -1 : (abort_on_error ? 1 : 0);
    if (!hseg) hseg = sl.h.seg;
    // tiny: [off | cap | flags | tids | len | status | segment] in one block
    const bool tiny = n <= kPackMax && seg_bytes <= kTinySeg;
    const size_t tiny_off = (24ull * n + 15) & ~(size_t)15;
    // direct: k_small reads the block from its pinned host copy and writes
    // the results back there itself -- no copy either way
    const bool direct = tiny && sl.m_pack && small_path(e, n);
    uint8_t *d_seg = tiny ? reinterpret_cast<uint8_t *>(sl.d_pack) + tiny_off : sl.d_seg;
    if (!tiny) HIPCHK(e, hipMemcpyAsync(sl.d_seg, hseg, seg_bytes, hipMemcpyHostToDevice, si));
    if (n <= kPackMax) {
        uint32_t *hp = sl.h_pack, *dp = sl.d_pack;
        const size_t n4 = n * 4ull;
        memcpy(hp, sl.h.off, n4);
        memcpy(hp + n, sl.h.cap, n4);
        if (use_flags) memcpy(hp + 2 * (size_t)n, sl.h.flags, n4);
        if (use_tids) memcpy(hp + 3 * (size_t)n, sl.h.tids, n4);
        memcpy(hp + 4 * (size_t)n, sl.h.len, n4);
        if (tiny) {
            memcpy(reinterpret_cast<uint8_t *>(hp) + tiny_off, hseg, seg_bytes);
            if (!direct) HIPCHK(e, hipMemcpyAsync(dp, hp, tiny_off + seg_bytes, hipMemcpyHostToDevice, si));
        } else {
            HIPCHK(e, hipMemcpyAsync(dp, hp, 5 * n4, hipMemcpyHostToDevice, si));
        }
        if (si != s && !direct) {
            HIPCHK(e, hipEventRecord(sl.ev_in, si));
            HIPCHK(e, hipStreamWaitEvent(s, sl.ev_in, 0));
        }
        sl.rc = transform_locked(e, reverse, use_tids ? reinterpret_cast<int32_t *>(dp + 3 * (size_t)n) : nullptr,
                                 tid, d_seg, dp, dp + 4 * (size_t)n, dp + n,
                                 use_flags ? dp + 2 * (size_t)n : nullptr,
                                 reinterpret_cast<int32_t *>(dp + 5 * (size_t)n), n, s, abort, false,
                                 direct ? sl.m_pack : nullptr, reinterpret_cast<uint8_t *>(dp),
                                 direct ? (uint32_t)(tiny_off + seg_bytes) : 0u);
        if (sl.rc != SRTP_OK) return sl.rc;
        if (so != s && !direct) {
            HIPCHK(e, hipEventRecord(sl.ev_done, s));
            HIPCHK(e, hipStreamWaitEvent(so, sl.ev_done, 0));
        }
        if (tiny) { // len | status | segment back in one copy (direct: k_small wrote them)
            if (!direct)
                HIPCHK(e, hipMemcpyAsync(hp + 4 * (size_t)n, dp + 4 * (size_t)n,
                                         tiny_off - 16 * (size_t)n + seg_bytes, hipMemcpyDeviceToHost, so));
            sl.tiny_dst = hseg;
            sl.tiny_off = tiny_off;
            sl.tiny_bytes = seg_bytes;
        } else {
            HIPCHK(e, hipMemcpyAsync(hseg, sl.d_seg, seg_bytes, hipMemcpyDeviceToHost, so));
            HIPCHK(e, hipMemcpyAsync(hp + 4 * (size_t)n, dp + 4 * (size_t)n, 2 * n4, hipMemcpyDeviceToHost, so));
        }
        sl.packed_n = n;
    } else {
        HIPCHK(e, hipMemcpyAsync(sl.d_off, sl.h.off, n * 4ull, hipMemcpyHostToDevice, si));
        HIPCHK(e, hipMemcpyAsync(sl.d_len, sl.h.len, n * 4ull, hipMemcpyHostToDevice, si));
        HIPCHK(e, hipMemcpyAsync(sl.d_cap, sl.h.cap, n * 4ull, hipMemcpyHostToDevice, si));
        if (use_flags) HIPCHK(e, hipMemcpyAsync(sl.d_flags, sl.h.flags, n * 4ull, hipMemcpyHostToDevice, si));
        if (use_tids) HIPCHK(e, hipMemcpyAsync(sl.d_tids, sl.h.tids, n * 4ull, hipMemcpyHostToDevice, si));
        if (si != s) {
            HIPCHK(e, hipEventRecord(sl.ev_in, si));
            HIPCHK(e, hipStreamWaitEvent(s, sl.ev_in, 0));
        }
        sl.rc = transform_locked(e, reverse, use_tids ? sl.d_tids : nullptr, tid, sl.d_seg, sl.d_off,
                                 sl.d_len, sl.d_cap, use_flags ? sl.d_flags : nullptr, sl.d_status, n, s, abort);
        if (sl.rc != SRTP_OK) return sl.rc;
        if (so != s) {
            HIPCHK(e, hipEventRecord(sl.ev_done, s));
            HIPCHK(e, hipStreamWaitEvent(so, sl.ev_done, 0));
        }
        HIPCHK(e, hipMemcpyAsync(hseg, sl.d_seg, seg_bytes, hipMemcpyDeviceToHost, so));
        HIPCHK(e, hipMemcpyAsync(sl.h.len, sl.d_len, n * 4ull, hipMemcpyDeviceToHost, so));
        HIPCHK(e, hipMemcpyAsync(sl.h.status, sl.d_status, n * 4ull, hipMemcpyDeviceToHost, so));
    }
    HIPCHK(e, hipEventRecord(sl.ev_out, so));
    sl.busy = true;
    return SRTP_OK;
}

int srtp_pipeline_submit_ex(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                            int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                            int32_t abort_on_error) {
    return pipeline_submit(pl, slot, reverse, use_tids, tid, use_flags, n, seg_bytes, abort_on_error, nullptr);
}

int srtp_pipeline_submit_host(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                              int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                              int32_t abort_on_error, uint8_t *host_seg) {
    // the D2H writes whole 16-B regions: the registered range must hold them
    if (!host_seg || (n && !srtp_host_is_registered(host_seg, (seg_bytes + 15) & ~(size_t)15)))
        return SRTP_EINVAL;
    return pipeline_submit(pl, slot, reverse, use_tids, tid, use_flags, n, seg_bytes, abort_on_error, host_seg);
}

// The slot's bundle laid out in the slot (off, cap, ...), its packets' regions
// read by the GPU from the caller's registered memory at host_base + src_off[j]
// and written back there afterwards (srtp_mi355x.h).  Packed per-packet arrays
// (n <= kPackMax); the gather runs on the copy-in stream, the scatter on the
// copy-out stream, so one slot's moves overlap another's kernels.
int srtp_pipeline_submit_gather(srtp_pipeline *pl, int32_t slot, int32_t reverse, int32_t use_tids,
                                int32_t tid, int32_t use_flags, uint32_t n, size_t seg_bytes,
                                int32_t abort_on_error, uint8_t *host_base, size_t host_bytes,
                                const uint32_t *src_off) {
    if (!pl || slot < 0 || (size_t)slot >= pl->slots.size() || (n && (!host_base || !src_off)))
        return SRTP_EINVAL;
    if (n > kPackMax || (n && !srtp_host_is_registered(host_base, host_bytes))) return SRTP_EINVAL;
    std::lock_guard<std::mutex> gp(pl->mu);
    srtp_pipeline::Slot &sl = pl->slots[(size_t)slot];
    srtp_engine *e = pl->e;
    GUARD(e);
    (void)pipeline_wait_locked(pl, sl);
    if (n > pl->max_n || seg_bytes > pl->max_seg) return fail(e, SRTP_EINVAL, "bundle exceeds the slot");
    if (n == 0) return SRTP_OK;
    seg_bytes = (seg_bytes + 15) & ~(size_t)15;
    for (uint32_t j = 0; j < n; j++) { // every region inside the registered range, 16-B aligned
        const uint64_t r = ((uint64_t)sl.h.cap[j] + 15u) & ~15ull;
        if (src_off[j] % 16 != 0 || (uint64_t)src_off[j] + r > host_bytes)
            return fail(e, SRTP_EINVAL, "gathered packet region outside the registered segment");
    }
    uint8_t *dhost = host_device_ptr(host_base);
    if (!dhost) return fail(e, SRTP_EDEVICE, "registered segment without a device mapping");
    std::lock_guard<std::mutex> g(e->mu);
    int rc = validate_regions(e, sl.h.off, sl.h.cap, n, seg_bytes);
    if (rc != SRTP_OK) return rc;
    if (!use_tids && (tid < 0 || (size_t)tid >= e->transformers.size()))
        return fail(e, SRTP_EINVAL, "bad transformer id");
    const bool one = pl->one_stream;
    hipStream_t s = e->stream, si = one ? s : pl->s_in, so = one ? s : pl->s_out;
    const int32_t abort = abort_on_error < 0 ? -1 : (abort_on_error ? 1 : 0);
    uint32_t *hp = sl.h_pack, *dp = sl.d_pack;
    const size_t n4 = n * 4ull;
    memcpy(hp, sl.h.off, n4);
    memcpy(hp + n, sl.h.cap, n4);
    if (use_flags) memcpy(hp + 2 * (size_t)n, sl.h.flags, n4);
    if (use_tids) memcpy(hp + 3 * (size_t)n, sl.h.tids, n4);
    memcpy(hp + 4 * (size_t)n, sl.h.len, n4);
    memcpy(sl.h_src, src_off, n4);
    HIPCHK(e, hipMemcpyAsync(dp, hp, 5 * n4, hipMemcpyHostToDevice, si));
    HIPCHK(e, hipMemcpyAsync(sl.d_src, sl.h_src, n4, hipMemcpyHostToDevice, si));
    HIPCHK(e, launch_move_regions(true, sl.d_seg, dp, dp + n, dhost, sl.d_src, n, si));
    if (si != s) {
        HIPCHK(e, hipEventRecord(sl.ev_in, si));
        HIPCHK(e, hipStreamWaitEvent(s, sl.ev_in, 0));
    }
    sl.rc = transform_locked(e, reverse, use_tids ? reinterpret_cast<int32_t *>(dp + 3 * (size_t)n) : nullptr, tid,
                             sl.d_seg, dp, dp + 4 * (size_t)n, dp + n, use_flags ? dp + 2 * (size_t)n : nullptr,
                             reinterpret_cast<int32_t *>(dp + 5 * (size_t)n), n, s, abort);
    if (sl.rc != SRTP_OK) return sl.rc;
    if (so != s) {
        HIPCHK(e, hipEventRecord(sl.ev_done, s));
        HIPCHK(e, hipStreamWaitEvent(so, sl.ev_done, 0));
    }
    HIPCHK(e, launch_move_regions(false, sl.d_seg, dp, dp + n, dhost, sl.d_src, n, so));
    HIPCHK(e, hipMemcpyAsync(hp + 4 * (size_t)n, dp + 4 * (size_t)n, 2 * n4, hipMemcpyDeviceToHost, so));
    sl.packed_n = n;
    HIPCHK(e, hipEventRecord(sl.ev_out, so));
    sl.busy = true;
    return SRTP_OK;
}

int srtp_pipeline_query(srtp_pipeline *pl, int32_t slot) {
    if (!pl || slot < 0 || (size_t)slot >= pl->slots.size()) return SRTP_EINVAL;
    std::lock_guard<std::mutex> gp(pl->mu);
    const srtp_pipeline::Slot &sl = pl->slots[(size_t)slot];
    if (!sl.busy) return 1;
    const hipError_t q = hipEventQuery(sl.ev_out);
    if (q == hipSuccess) return 1;
    return q == hipErrorNotReady ? 0 : fail(pl->e, SRTP_EDEVICE, "pipeline D2H");
}

int srtp_pipeline_wait(srtp_pipeline *pl, int32_t slot) {
    if (!pl || slot < 0 || (size_t)slot >= pl->slots.size()) return SRTP_EINVAL;
    std::lock_guard<std::mutex> gp(pl->mu);
    return pipeline_wait_locked(pl, pl->slots[(size_t)slot]);
}
