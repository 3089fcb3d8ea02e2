// srtp_kernels.h -- launch interface of the gfx950 SRTP kernels (srtp_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "srtp_types.h"

namespace srtp {

constexpr int kSortMaxPass = 4; // 8-bit digits: context tables up to 2^31 slots
// Context chains of at least this many records in a bundle are walked by the
// wave-parallel (speculative) walk, shorter ones lane-serially.
#ifndef SRTP_LONG_MIN
#define SRTP_LONG_MIN 256
#endif
constexpr uint32_t kLongMin = SRTP_LONG_MIN;

// Everything one bundle needs; passed by value to every kernel.
struct BundleArgs {
    // engine tables (HBM resident)
    const KeySet *keysets;
    const ExtKeys *extkeys;  // [keysets] round keys of the k_ext key sets (AES-F8 IV', AES-256)
    const TwofishKeys *tfkeys; // [2 * keysets] Twofish session / F8 IV' keys (null: none yet)
    const SkeinKeys *skkeys;   // [keysets] Skein-512 MAC keys (null: none yet)
    const FactoryRec *factories;
    const TransformerRec *transformers;
    uint64_t *ctx_keys;
    CtxState *ctx;
    uint32_t ctx_mask;     // table capacity - 1 (power of two)
    // [ctx_mask + 1] per context slot: serial + 1 of the last unprotect bundle
    // in which one of the context's RTP packets lay 16384 or more from its
    // bundle-start s_l, or the context had no seqNumSet (k_parse); otherwise
    // its ROC cannot change within the bundle (see k_unprotect)
    uint32_t *far;
    uint32_t n_transformers;
    // caller's bundle
    uint8_t *seg;
    const uint32_t *off;
    uint32_t *len;
    const uint32_t *cap;
    const uint32_t *flags; // may be null
    int32_t *status;
    const int32_t *tids;   // may be null -> tid
    int32_t tid;
    uint32_t n;
    int32_t reverse;
    int32_t check_replay;
    int32_t abort_on_error;
    uint32_t serial;       // bundle serial (context birth stamp)
    uint32_t dbg;          // kDbg* test hooks (srtp_engine_set_debug): 0 in production
    int32_t has_skein;     // the engine has Skein-MAC key sets (the walk's Skein re-check)
    unsigned long long *counters; // [kCountReplicas][kCtrStride] cumulative event counters
    // k_small's direct mode (a tiny pipeline bundle): the packed block
    // [off | cap | flags | tids | len | status | segment] at pk_dev is first
    // read from its pinned host copy pk_host (device-mapped, coherent) and
    // len, status and the packet regions written back there, instead of a
    // copy each way; pk_host null: the block is already in device memory
    const uint8_t *pk_host;
    uint8_t *pk_dev;
    uint32_t pk_bytes;
#ifdef SRTP_STAMPS
    unsigned long long *stamps;   // diagnostic build only: per-wave start / filled / end times
#endif
    // per-bundle scratch
    uint32_t *p_slot;      // [n] context slot of packet p
    uint32_t *sk_in, *sk_out; // [n] sort keys (slot)
    WalkRec *sv_in, *sv_out;  // [n] sort values
    int32_t *w_status;     // [n]
    uint32_t *w_cw;        // [n] guessed ROC / SRTCP index word
    uint32_t *w_len;       // [n] length after processing
    uint32_t *gok;         // [2n] unprotect, per packet p: gok[2p] = g0, the ROC the verify
                           // pass assumed; gok[2p + 1] = auth_ok: bit 0 tag matched under
                           // g0; bit 2: also checked under g0 - 1, bit 1 its result (one
                           // 8-B word, so the walk gathers both with one load)
    uint32_t *mid;         // [5n] unprotect: inner SHA-1 state before the ROC block
    uint32_t *tailc;       // [16n] unprotect: ciphertext of the ROC-carrying 64-B chunk
    uint32_t *spec;        // [n] unprotect: kSpec* summary of k_unprotect (bit 0: decrypted in place under g0)
    uint64_t *tile_link;   // [(n / 256 + 2) * 10] per walk tile: the published part of a long chain
    uint32_t *spos;        // [n] unprotect: each record's position in sort order (the last sort pass)
    uint32_t *lord;        // [n] packets grouped by length class (the sort's first pass), for the crypto kernels
    uint32_t *cls_tile;    // [tiles][33] per sort tile: packets per length class, the class mask
                           // (k_parse; zeroed again by k_walk)
    int32_t *e_min;        // [n_transformers] first throwing packet per transformer
    BundleCtl *ctl_next;   // the next bundle's control block, reset by k_parse
    int32_t *e_min_next;   // the next bundle's e_min, [n_transformers] set to 0x7f7f7f7f by k_parse
    BundleCtl *ctl;
    // radix sort of the walk records (srtp_kernels.hip "radix sort")
    uint32_t *sort_counts; // [tiles][bins] first-digit counts per sort tile, by k_parse
    int32_t sort_passes;   // digits to sort: key width / 8 rounded up, or 2 wide digits
    int32_t sort_bits;     // bits of the first digit (8, or 9-11 for a two-pass wide sort)
    int32_t sort_hi_bits;  // 9-11: an 8-bit first pass, then one wide pass of these bits (0: not)
    int32_t sort_key_bits; // the key's width (slot bits + 1)
    uint32_t *sort_zero;   // the last pass's digit counts, re-zeroed by k_walk
    uint32_t sort_zero_words;
    // a small bundle: the AES-CM keystream of the AES-CM + HMAC-SHA1 packets is
    // applied by k_ctr_small (a lane per counter-block pair), the fused
    // kernels only MAC those packets; 2: the split path (k_ctr_wide + k_mac_wide)
    int32_t small_ctr;
};

// Layout of the sort's scratch (one allocation of sort_temp_bytes(n_max)).
struct SortScratch {
    uint32_t *keys_tmp;
    WalkRec *vals_tmp;
    uint32_t *counts[kSortMaxPass]; // [tiles][256] digit counts per tile and pass (kept zero between uses)
    // the two-pass wide sort (9-11-bit digits, context tables of 2^16-2^21 slots)
    uint32_t *wcounts[2];           // [tiles][2^bits] digit counts per pass (pass 0 kept zero between uses)
    uint32_t *wprefix;              // [tiles][2^bits] per digit, records in earlier tiles
    uint32_t *wtotal;               // [2^bits] records per digit
    uint32_t max_tiles;
};
constexpr int kSortWideMaxBits = 11;

hipError_t launch_parse(const BundleArgs &a, hipStream_t s);
size_t sort_temp_bytes(uint32_t n_max);
uint32_t sort_tile_records(); // records per sort tile (k_parse's class and digit counts, the sort's tiles)
SortScratch sort_scratch(void *temp, uint32_t n_max);
// Stable LSD radix sort of (sk_in, sv_in) by key into (sk_out, sv_out),
// a.sort_passes passes of 8 bits; zeroes the other parity's histograms.
hipError_t launch_sort(const BundleArgs &a, const SortScratch &ss, hipStream_t s);
// the whole sort of a bundle of at most sort_tile_records() packets in one
// workgroup (one launch)
hipError_t launch_sort_tile(const BundleArgs &a, hipStream_t s);
// k_parse + the one-tile sort in one launch (a bundle of at most
// sort_tile_records() packets)
// unprotect: fused tag check + speculative in-place decryption (before the walk)
hipError_t launch_unprotect(const BundleArgs &a, hipStream_t s);
// Engines with Skein-MAC key sets.  Unprotect: those packets' tag check under
// k_unprotect's ROC guess (after k_unprotect, before the walk).  Protect: their
// trailers (after k_ext).
hipError_t launch_skein(const BundleArgs &a, hipStream_t s);
hipError_t launch_walk(const BundleArgs &a, int limit_pass, hipStream_t s);
hipError_t launch_protect(const BundleArgs &a, hipStream_t s);
// BundleArgs::small_ctr: the keystream of the AES-CM + HMAC-SHA1 packets, one
// workgroup per packet -- protect before k_protect, unprotect after k_unprotect
hipError_t launch_ctr_small(const BundleArgs &a, hipStream_t s);
// The split path (BundleArgs::small_ctr == 2): the AES-CM keystream of a
// bundle, lane per counter-block pair (protect: before k_mac_wide; unprotect:
// after the walk, with the final statuses), and the HMAC-SHA1 (protect: MAC,
// trailer and final statuses; unprotect: the tag check before the walk)
hipError_t launch_ctr_wide(const BundleArgs &a, hipStream_t s);
hipError_t launch_mac_wide(const BundleArgs &a, hipStream_t s);
// A bundle of up to kSmallMaxN packets (engines whose key sets are all AES-CM
// or NULL cipher with HMAC-SHA1): parse, sort, (tag check,)
// walk, keystream and (MAC, trailer) in one workgroup and one launch (k_small).
constexpr uint32_t kSmallMaxN = 255u;
hipError_t launch_small(const BundleArgs &a, hipStream_t s);
// Packet regions [doff[j], + cap[j] rounded to 16) of a device segment from /
// to [src[j], ...) of device-mapped host memory (a dispatcher shard's gather of
// an interleaved registered host bundle)
hipError_t launch_move_regions(bool to_device, uint8_t *dseg, const uint32_t *doff, const uint32_t *cap,
                               uint8_t *host, const uint32_t *src, uint32_t n, hipStream_t s);
// unprotect: statuses/lengths out; undo/redo the rare speculation misses (after the walk)
hipError_t launch_unprotect_fix(const BundleArgs &a, hipStream_t s);
// AES-F8 packets after the final statuses: protect (F8 + HMAC + trailer) or
// decryption of the accepted unprotected packets.
hipError_t launch_ext(const BundleArgs &a, hipStream_t s);
hipError_t launch_remove_transformer(uint64_t *ctx_keys, CtxState *ctx, uint32_t cap,
                                     uint32_t tid, hipStream_t s);
// Contexts by key (tid << 32 | ssrc): save -> out[i] / present[i]; restore ->
// create or overwrite (present[i]) or remove (!present[i]); keys distinct.
hipError_t launch_ctx_save(const uint64_t *tab, const CtxState *ctx, uint32_t mask, const uint64_t *keys,
                           uint32_t n, CtxState *out, int32_t *present, hipStream_t s);
hipError_t launch_ctx_restore(uint64_t *tab, CtxState *ctx, uint32_t mask, const uint64_t *keys, uint32_t n,
                              const CtxState *in, const int32_t *present, unsigned int *failed,
                              hipStream_t s);
// out[0] += live contexts, out[1] += tombstones
hipError_t launch_count_contexts(const uint64_t *ctx_keys, uint32_t cap, unsigned long long *out,
                                 hipStream_t s);
// Table rebuild without tombstones: collect the live (key, state) pairs into
// tmp_keys / tmp_ctx (count in *n_live, which starts at 0), then the caller
// resets the key array and re-inserts them.
hipError_t launch_rehash_collect(const uint64_t *ctx_keys, const CtxState *ctx, uint32_t cap,
                                 uint64_t *tmp_keys, CtxState *tmp_ctx, unsigned long long *n_live,
                                 hipStream_t s);
hipError_t launch_rehash_insert(uint64_t *ctx_keys, CtxState *ctx, uint32_t mask,
                                const uint64_t *tmp_keys, const CtxState *tmp_ctx, uint32_t n,
                                hipStream_t s);
// Upload the LE T-table used by the AES rounds (once per device).
hipError_t upload_tables(const uint32_t te0[256]);

} // namespace srtp
