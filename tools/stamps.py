"""Per-wave timing of k_protect / k_unprotect (diagnostic build with
SRTP_STAMPS: libsrtp_stamps.so, built by tools/stamps.sh).

Runs the bench workload (2^18 x 1200-B packets, 10k SSRCs) serially for a few
bundles, then reads each wave's realtime-clock stamps (100 MHz) of the last
launch: entry, after the LDS T-table fill, end; __smid (XCC / SE / CU); and the
shader clock counter (s_memtime) at the same points, for the clock the waves ran at.
Prints the spread of wave start / end times over the launch, per XCC."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("SRTP_MI355X_LIB", os.path.join(ROOT, "tools", "stamps", "libsrtp_stamps.so"))

import torch  # noqa: E402

from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, profile_policies, synth  # noqa: E402
from libjitsi_amd import _native as N  # noqa: E402


def main():
    n, L = 1 << 18, 1200
    L_ = N.lib()
    L_.srtp_debug_stamps.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_uint32]
    eng = SRTPEngine(device=0, max_contexts=1 << 15, max_factories=8, max_transformers=8, max_batch=n)
    pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
    (k, s), = synth.keys(2, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng))
    b = synth.rtp_bundle(n, 10000, L, seed=synth.SEED_BASE + 2)
    dev = torch.device("cuda", 0)
    off = torch.from_numpy(b.off.view(np.int32)).to(dev)
    cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    step = -(-n // 10000)
    base = torch.from_numpy(b.seg).to(dev)
    off64 = off.to(torch.int64)
    for it in range(12):
        seg = base.clone()
        hi, lo = seg[off64 + 2].to(torch.int32), seg[off64 + 3].to(torch.int32)
        q = ((hi << 8) | lo) + it * step
        seg[off64 + 2] = ((q >> 8) & 0xFF).to(torch.uint8)
        seg[off64 + 3] = (q & 0xFF).to(torch.uint8)
        ln = torch.from_numpy(b.length.view(np.int32)).to(dev)
        cur = torch.cuda.current_stream(dev)  # after the torch work that built seg / ln
        eng.transform_device(False, snd.tid, seg, off, ln, cap, st, stream=cur)
        eng.transform_device(True, rcv.tid, seg, off, ln, cap, st, stream=cur)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    waves = n // 64
    out = {}
    for name, rev in (("k_protect", 0), ("k_unprotect", 1)):
        buf = np.zeros(waves * 8, np.uint64)
        N.check(L_.srtp_debug_stamps(eng.h, rev, buf.ctypes.data, waves), eng.h, "stamps")
        t = buf.reshape(waves, 8)
        t0 = t[:, 0].min()
        start = (t[:, 0] - t0) / 100.0  # us
        filled = (t[:, 1] - t0) / 100.0
        end = (t[:, 2] - t0) / 100.0
        smid = t[:, 3].astype(np.int64)
        wg_end = end.reshape(-1, 16).max(axis=1)
        wg_start = start.reshape(-1, 16).min(axis=1)
        r = {"launch_us": float(end.max()),
             "wave_start_us": np.percentile(start, [0, 50, 90, 99, 100]).round(1).tolist(),
             "fill_us_median": float(np.median(filled - start)),
             "wave_end_us": np.percentile(end, [0, 10, 50, 90, 100]).round(1).tolist(),
             "wave_busy_us": np.percentile(end - filled, [0, 10, 50, 90, 100]).round(1).tolist(),
             "wg_end_us_pct": np.percentile(wg_end, [0, 10, 50, 90, 100]).round(1).tolist(),
             "wg_start_us_pct": np.percentile(wg_start, [0, 50, 100]).round(1).tolist(),
             "mean_wave_lifetime_over_launch": float((end - start).mean() / end.max())}
        xcc = (smid >> 6) & 0xF if smid.max() > 63 else smid // 32
        per = {}
        for x in np.unique(xcc):
            m = xcc == x
            per[int(x)] = {"waves": int(m.sum()), "end_median": float(np.median(end[m])),
                           "end_max": float(end[m].max()), "busy_median": float(np.median((end - filled)[m]))}
        r["per_xcc"] = per
        # shader clock over the wave's life / realtime (100 MHz): the clock it ran at
        dclk = (t[:, 6] - t[:, 4]).astype(np.float64)
        dt = (t[:, 2] - t[:, 0]).astype(np.float64) / 100.0  # us
        r["shader_clock_mhz"] = np.percentile(dclk / np.maximum(dt, 1e-3), [0, 50, 100]).round(0).tolist()
        r["smid_distinct"] = int(len(np.unique(smid)))
        out[name] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
