#!/usr/bin/env python3
"""Throughput of every BASELINE.json config on one MI355X, beside the oracle's
CPU restatement of the reference path on the same host (one thread).

bench.py measures configs[1] (the headline); this tool fills BASELINE.md's
per-config table:

  C1  1 SSRC, 160-B (Opus-sized) RTP, protect -> unprotect round trips
  C2  10k SSRCs, 1200-B RTP, protect -> unprotect round trips
  C3  mixed 60-1400-B RTP over 10k SSRCs, unprotect of bundles carrying the C3
      fault mix (1 % tampered, 1 % exact replays, 0.5 % stale replays,
      5 % reordered within 16): tag checks, ROC/index estimation, replay drops
  C4  SRTP + SRTCP over AES_CM_128_HMAC_SHA1_80 / _32 / NULL_HMAC_SHA1_80
      (one sender/receiver pair per profile and kind in one bundle), an SDES
      rekey (new factories on the _80 pair) half-way, round trips
  C5  one GPU's share of 10^6 streams on 8 GPUs (125k SSRCs), and all 10^6 on
      one GPU, 1200-B round trips

GPU: K bundles of 2^18 packets (C1: 2^18 packets of one stream), each with
fresh sequence numbers, staged in HBM; the clock covers the K protects and K
unprotects (wall time, synchronized).  Every status is checked (OK, or the
expected fault drops in C3).  CPU: the oracle (oracle/srtp_oracle.c, the
reference's call structure, `kind: port`) on a 2^14-packet sample of the same
bundles, one thread -- a bounded sample, as bench.py's cpu_baseline.

    python tools/config_bench.py [--configs C1,C2,...] [--bundles K] [--out file.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from libjitsi_amd import (SRTCPTransformer, SRTPContextFactory, SRTPEngine, SRTPTransformer,  # noqa: E402
                          profile_policies, synth)
from libjitsi_amd import _native as N  # noqa: E402
from oracle import oracle as O  # noqa: E402

N_PKT = 1 << 18
SAMPLE = 1 << 14


def opol(p):
    return O.Policy(p.encType, p.encKeyLength, p.authType, p.authKeyLength, p.authTagLength,
                    p.saltKeyLength)


def split(b, k, n):
    return [synth.select(b, np.arange(i * n, (i + 1) * n)) for i in range(k)]


class Dev:
    """A bundle staged in HBM (torch tensors on cuda:0)."""

    def __init__(self, torch, b, tids=None):
        d = torch.device("cuda", 0)
        self.n = b.n
        self.seg = torch.from_numpy(b.seg).to(d)
        self.off = torch.from_numpy(b.off.view(np.int32)).to(d)
        self.len = torch.from_numpy(b.length.view(np.int32)).to(d)
        self.cap = torch.from_numpy(b.cap.view(np.int32)).to(d)
        self.st = torch.empty(b.n, dtype=torch.int32, device=d)
        self.tids = None if tids is None else torch.from_numpy(np.asarray(tids, np.int32)).to(d)

    def run(self, eng, reverse, tid):
        eng.transform_device(reverse, self.tids if self.tids is not None else tid, self.seg, self.off,
                             self.len, self.cap, self.st)

    def host(self):
        return self.seg.cpu().numpy(), self.len.cpu().numpy().view(np.uint32), self.st.cpu().numpy()


def timed(torch, fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def engine(nssrc, n):
    max_ctx = 1 << max(12, (int(1.6 * max(nssrc, 1)) - 1).bit_length())
    return SRTPEngine(device=0, max_contexts=max_ctx, max_factories=64, max_transformers=64, max_batch=n)


def cpu_round_trips(b, pol, keys, n):
    """Oracle protect + unprotect of the first n packets of bundle b, 1 thread."""
    (k, s) = keys
    po = opol(pol[0]), opol(pol[1])
    snd = O.Transformer(O.KIND_RTP, O.Factory(True, k, s, *po), O.Factory(True, k, s, *po))
    rcv = O.Transformer(O.KIND_RTP, O.Factory(False, k, s, *po), O.Factory(False, k, s, *po))
    sb = synth.select(b, np.arange(min(n, b.n)))
    seg, ln = sb.seg.copy(), sb.length.copy()
    t0 = time.perf_counter()
    st1 = O.process(snd, False, seg, sb.off, ln, sb.cap)
    st2 = O.process(rcv, True, seg, sb.off, ln, sb.cap)
    dt = time.perf_counter() - t0
    return {"value": round(sb.n / dt, 1), "unit": "round trips/s", "threads": 1, "kind": "port",
            "sample": f"{sb.n} packets of the same bundle, oracle protect then unprotect",
            "all_ok": bool((st1 == 0).all() and (st2 == 0).all())}


def round_trip_config(torch, name, nssrc, pkt_len, K, pols, seed):
    n = N_PKT
    b = synth.rtp_bundle(K * n, nssrc, pkt_len, seed=seed)
    keys = synth.keys(seed, 1)[0]
    es, er = engine(nssrc, n), engine(nssrc, n)
    snd = SRTPTransformer(SRTPContextFactory(True, *keys, *pols, engine=es))
    rcv = SRTPTransformer(SRTPContextFactory(False, *keys, *pols, engine=er))
    parts = split(b, K, n)
    dev = [Dev(torch, p) for p in parts]
    # warm the kernels on a throwaway pair of engines (their contexts stay out of the timed ones)
    ew = engine(nssrc, n)
    tw = SRTPTransformer(SRTPContextFactory(True, *keys, *pols, engine=ew))
    w = Dev(torch, parts[0])
    w.run(ew, False, tw.tid)
    torch.cuda.synchronize()
    ew.close()
    tp = timed(torch, lambda: [d.run(es, False, snd.tid) for d in dev])
    ok_p = all(int((d.st != 0).sum()) == 0 for d in dev)
    tu = timed(torch, lambda: [d.run(er, True, rcv.tid) for d in dev])
    ok_u = all(int((d.st != 0).sum()) == 0 for d in dev)
    pkts = K * n
    avg_len = float(b.length[:pkts].mean())
    cpu = cpu_round_trips(parts[-1] if nssrc > 1 else parts[0], pols, keys, SAMPLE)
    es.close(); er.close()
    return {"config": name, "ssrcs": nssrc, "pkt_len": pkt_len if isinstance(pkt_len, int) else list(pkt_len),
            "bundles": K, "packets_per_bundle": n,
            "round_trips_per_s": round(pkts / (tp + tu), 1),
            "protect_pps": round(pkts / tp, 1), "unprotect_pps": round(pkts / tu, 1),
            "gbps_algorithmic": round(pkts * 2 * (2 * avg_len + 10) / (tp + tu) / 1e9, 1),
            "all_ok": bool(ok_p and ok_u), "cpu": cpu}


def inject_faults(b, rng, tag_len=10):
    """C3 fault mix (tests/test_gpu_parity.py's inject_faults, vectorised)."""
    n = b.n
    order = np.arange(n)
    sw = np.nonzero(rng.random(n) < 0.05)[0]
    jump = rng.integers(1, 17, len(sw))
    for i, j in zip(sw, np.minimum(n - 1, sw + jump)):
        order[i], order[j] = order[j], order[i]
    r = rng.random(n)
    rep = r < 0.01
    stale = (r >= 0.01) & (r < 0.015) & (np.arange(n) > 200)
    extra = np.where(rep, order, np.where(stale, order[np.maximum(0, np.arange(n) - rng.integers(130, 200, n))], -1))
    out = np.stack([order, extra], 1).reshape(-1)
    out = out[out >= 0]
    fb = synth.select(b, out)
    tam = np.nonzero(rng.random(fb.n) < 0.01)[0]
    L = fb.length[tam].astype(np.int64)
    pos = (rng.random(len(tam)) * L).astype(np.int64)
    fb.seg[fb.off[tam].astype(np.int64) + pos] ^= (1 << rng.integers(0, 8, len(tam))).astype(np.uint8)
    return fb


def config3(torch, K, seed):
    n = N_PKT
    pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
    b = synth.rtp_bundle(K * n, 10000, (60, 1400), seed=seed)
    keys = synth.keys(seed, 1)[0]
    es, er = engine(10000, n), engine(10000, 2 * n)
    snd = SRTPTransformer(SRTPContextFactory(True, *keys, *pols, engine=es))
    rcv = SRTPTransformer(SRTPContextFactory(False, *keys, *pols, engine=er))
    rng = np.random.default_rng(seed)
    # protect through the host path (untimed), then fault the wire bundles
    fb = []
    for p in split(b, K, n):
        seg, ln = p.seg.copy(), p.length.copy()
        st = es.transform_host(False, snd.tid, seg, p.off, ln, p.cap)
        assert (st == 0).all()
        p.seg, p.length = seg, ln
        fb.append(inject_faults(p, rng))
    dev = [Dev(torch, x) for x in fb]
    ew = engine(10000, 2 * n)
    tw = SRTPTransformer(SRTPContextFactory(False, *keys, *pols, engine=ew))
    w = Dev(torch, fb[0])
    w.run(ew, True, tw.tid)
    torch.cuda.synchronize()
    ew.close()
    er.set_timing(True)
    tu = timed(torch, lambda: [d.run(er, True, rcv.tid) for d in dev])
    tm = er.read_timing()
    er.set_timing(False)
    stages = {k: round(v[0] / max(v[1], 1), 4) for k, v in tm.items() if v[1]}
    est = er.stats()
    slow = {k: est[k] for k in ("long_walked", "repaired", "roc_rechecks")}
    stc = np.bincount(np.concatenate([d.st.cpu().numpy() for d in dev]), minlength=N.NUM_STATUS)
    pkts = sum(x.n for x in fb)
    # CPU: the oracle receiver over a sample of the last faulted bundle, after
    # the bundles before it (so its contexts hold the same state)
    po = opol(pols[0]), opol(pols[1])
    ro = O.Transformer(O.KIND_RTP, O.Factory(False, *keys, *po), O.Factory(False, *keys, *po))
    for x in fb[:-1]:
        O.process(ro, True, x.seg.copy(), x.off, x.length.copy(), x.cap)
    sb = synth.select(fb[-1], np.arange(min(SAMPLE, fb[-1].n)))
    seg, ln = sb.seg.copy(), sb.length.copy()
    t0 = time.perf_counter()
    O.process(ro, True, seg, sb.off, ln, sb.cap)
    dt = time.perf_counter() - t0
    es.close(); er.close()
    return {"config": "C3", "ssrcs": 10000, "pkt_len": [60, 1400], "bundles": K,
            "packets": pkts, "unprotect_pps": round(pkts / tu, 1),
            "gbps_algorithmic": round(sum(float((2 * x.length.astype(np.int64) - 10).sum()) for x in fb) / tu / 1e9, 1),
            "statuses": {N.STATUS_NAMES[i]: int(c) for i, c in enumerate(stc) if c},
            "stage_ms_per_bundle": stages, "slow_path_total": slow,
            "cpu": {"value": round(sb.n / dt, 1), "unit": "packets/s (unprotect)", "threads": 1, "kind": "port",
                    "sample": f"{sb.n} packets of the last faulted bundle, oracle unprotect"}}


def config4(torch, K, seed):
    """SRTP + SRTCP over three profiles, one bundle per step mixing them."""
    n = N_PKT
    profiles = ["AES_CM_128_HMAC_SHA1_80", "AES_CM_128_HMAC_SHA1_32", "NULL_HMAC_SHA1_80"]
    es, er = engine(3000, n), engine(3000, n)
    keys = synth.keys(seed, 4)
    snd, rcv, kinds = [], [], []
    for j, prof in enumerate(profiles):
        pols = profile_policies(prof)
        fs = SRTPContextFactory(True, *keys[j], *pols, engine=es)
        fr = SRTPContextFactory(False, *keys[j], *pols, engine=er)
        for cls in (SRTPTransformer, SRTCPTransformer):
            snd.append(cls(fs, fs))
            rcv.append(cls(fr, fr))
            kinds.append(cls)
    # per step: 80 % RTP (60-1400 B over 1000 SSRCs per profile), 20 % RTCP
    rng = np.random.default_rng(seed)
    n_rtp = int(0.8 * n) // 3
    n_rtcp = (n - 3 * n_rtp) // 3
    bundles, tids_s, tids_r = [], [], []
    rtp = [synth.rtp_bundle(K * n_rtp, 1000, (60, 1400), seed=seed + 10 + j) for j in range(3)]
    rtcp = [synth.rtcp_bundle(K * n_rtcp, 1000, seed=seed + 20 + j) for j in range(3)]
    for k in range(K):
        parts, ts, tr = [], [], []
        for j in range(3):
            parts.append(synth.select(rtp[j], np.arange(k * n_rtp, (k + 1) * n_rtp)))
            ts += [snd[2 * j].tid] * n_rtp
            tr += [rcv[2 * j].tid] * n_rtp
            parts.append(synth.select(rtcp[j], np.arange(k * n_rtcp, (k + 1) * n_rtcp)))
            ts += [snd[2 * j + 1].tid] * n_rtcp
            tr += [rcv[2 * j + 1].tid] * n_rtcp
        cb = synth.concat(parts)
        # interleave the six sources, each keeping its own order (a random
        # permutation would reorder a stream past the sender's replay window)
        keys_t = np.concatenate([(np.arange(p.n) + rng.random(p.n)) / p.n for p in parts])
        perm = np.argsort(keys_t, kind="stable")
        bundles.append(synth.select(cb, perm))
        tids_s.append(np.asarray(ts, np.int32)[perm])
        tids_r.append(np.asarray(tr, np.int32)[perm])
    dev_s = [Dev(torch, b, t) for b, t in zip(bundles, tids_s)]
    # the rekey: new SDES factories on the _80 pair (SRTPTransformer.setContextFactory /
    # SRTCPTransformer.updateFactory), half-way through the protects and the unprotects
    pols80 = profile_policies(profiles[0])
    fs2 = SRTPContextFactory(True, *keys[3], *pols80, engine=es)
    fr2 = SRTPContextFactory(False, *keys[3], *pols80, engine=er)

    def protect_all():
        for k, d in enumerate(dev_s):
            if k == K // 2:
                snd[0].setContextFactory(fs2, True)
                snd[1].updateFactory(fs2, True)
            d.run(es, False, None)

    tp = timed(torch, protect_all)
    ok_p = all(int((d.st != 0).sum()) == 0 for d in dev_s)
    for d, t in zip(dev_s, tids_r):
        d.tids = torch.from_numpy(t).to(d.seg.device)

    def unprotect_all():
        for k, d in enumerate(dev_s):
            if k == K // 2:
                rcv[0].setContextFactory(fr2, False)
                rcv[1].updateFactory(fr2, False)
            d.run(er, True, None)

    tu = timed(torch, unprotect_all)
    # NULL-cipher SRTCP writes index 0 into every packet's trailer (SURVEY Q12,
    # SRTCPCryptoContext.java:419-424), so a receiver drops every SRTCP packet
    # of that stream after its first as a replay, as the reference does; all
    # other packets must come back OK
    null_rtcp = rcv[5].tid
    st_u = np.concatenate([d.st.cpu().numpy() for d in dev_s])
    tid_u = np.concatenate(tids_r)
    ok_u = bool((st_u[tid_u != null_rtcp] == 0).all() and
                np.isin(st_u[tid_u == null_rtcp], [N.STATUS_OK, N.STATUS_DROP_REPLAY]).all())
    st_hist = {N.STATUS_NAMES[i]: int(c) for i, c in enumerate(np.bincount(st_u, minlength=N.NUM_STATUS)) if c}
    pkts = sum(b.n for b in bundles)
    # CPU: oracle round trip of a sample of the first bundle (the same six streams)
    ot_s, ot_r = [], []
    for j, prof in enumerate(profiles):
        pols = profile_policies(prof)
        po = opol(pols[0]), opol(pols[1])
        fso, fro = O.Factory(True, *keys[j], *po), O.Factory(False, *keys[j], *po)
        for kind in (O.KIND_RTP, O.KIND_RTCP):
            ot_s.append(O.Transformer(kind, fso, fso))
            ot_r.append(O.Transformer(kind, fro, fro))
    idx = {t.tid: i for i, t in enumerate(snd)}
    sb = synth.select(bundles[0], np.arange(SAMPLE))
    ts = [ot_s[idx[int(t)]] for t in tids_s[0][:SAMPLE]]
    tr = [ot_r[idx[int(t)]] for t in tids_s[0][:SAMPLE]]
    seg, ln = sb.seg.copy(), sb.length.copy()
    t0 = time.perf_counter()
    s1 = O.process(ts, False, seg, sb.off, ln, sb.cap)
    s2 = O.process(tr, True, seg, sb.off, ln, sb.cap)
    dt = time.perf_counter() - t0
    es.close(); er.close()
    return {"config": "C4", "profiles": profiles, "kinds": "SRTP 80 % + SRTCP 20 %", "bundles": K,
            "packets": pkts, "rekey": "SDES factory swap on the _80 SRTP/SRTCP pair after bundle K/2",
            "round_trips_per_s": round(pkts / (tp + tu), 1), "protect_pps": round(pkts / tp, 1),
            "unprotect_pps": round(pkts / tu, 1), "all_ok": bool(ok_p and ok_u),
            "unprotect_statuses": st_hist,
            "note": "all_ok: every protect OK; every unprotect OK except the NULL-cipher SRTCP stream's "
                    "replay drops (index 0 in every trailer, Q12)",
            "cpu": {"value": round(sb.n / dt, 1), "unit": "round trips/s", "threads": 1, "kind": "port",
                    "sample": f"{sb.n} packets of the first bundle, oracle protect then unprotect",
                    "protect_ok": bool((s1 == 0).all()),
                    "unprotect_statuses": {N.STATUS_NAMES[i]: int(c) for i, c in
                                           enumerate(np.bincount(s2, minlength=N.NUM_STATUS)) if c}}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
    ap.add_argument("--bundles", type=int, default=8)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    assert torch.cuda.is_available(), "config_bench needs cuda:0"
    O.build()
    p80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
    res = []
    for c in a.configs.split(","):
        t0 = time.time()
        if c == "C1":
            r = round_trip_config(torch, "C1", 1, 160, a.bundles, p80, 101)
        elif c == "C2":
            r = round_trip_config(torch, "C2", 10000, 1200, a.bundles, p80, 102)
        elif c == "C3":
            r = config3(torch, a.bundles, 103)
        elif c == "C4":
            r = config4(torch, a.bundles, 104)
        elif c == "C5":
            r = round_trip_config(torch, "C5 (125k SSRCs: one GPU's share of 10^6 on 8)", 125000, 1200,
                                  a.bundles, p80, 105)
            res.append(r)
            print(json.dumps(r), flush=True)
            r = round_trip_config(torch, "C5 (10^6 SSRCs on one GPU)", 1000000, 1200, a.bundles, p80, 106)
        else:
            raise SystemExit(f"unknown config {c}")
        r["wall_s"] = round(time.time() - t0, 1)
        res.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
