#!/usr/bin/env python3
"""SRTP protect+unprotect throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], one bundle per GPU per step): 10,000
concurrent SSRCs, fixed 1200-byte video RTP packets, AES_CM_128_HMAC_SHA1_80,
a bundle of 2^18 packets resident in HBM.  One step = protect the bundle with
a sender SRTPTransformer, unprotect it with a separate receiver transformer
(SURVEY Q1).  Each step has its own bundle, staged in HBM before the clock
starts: bundle i is the base bundle with every SSRC's sequence numbers
advanced by i times the packets per SSRC per bundle (fresh packets for the
replay check; ROC wraps happen naturally).

Multi-GPU: one process per GPU (torchrun), contexts sharded by SSRC (each rank
owns its own 10k SSRCs), no collective on the data path ("scaling": "weak").
value = packets protected AND unprotected by all ranks / max-over-ranks time.

Also reported: the dominant kernel's roofline (k_protect, HIP events on the
bundle stream, algorithmic bytes L + (L+T) per packet) and a CPU baseline (the
oracle restatement of the reference's per-packet path, timed on host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
RING = 160  # most distinct bundles staged in HBM (x 319 MB at the default size)
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "SRTP protect+unprotect packets/s + GB/s, 1200B AES_CM_128_HMAC_SHA1_80, 1-8 GPU"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=1 << 18, help="bundle size per GPU")
    ap.add_argument("--ssrcs", type=int, default=10000, help="concurrent SSRCs per GPU")
    ap.add_argument("--len", type=int, default=1200, help="RTP packet length")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cpu_count)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned-host end-to-end leg")
    ap.add_argument("--e2e-bundles", type=int, default=24)
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for the barrier/timing reduction (nccl = RCCL)")
    ap.add_argument("--serial", action="store_true",
                    help="run the receiver on the sender's stream (no overlap between "
                         "step i's unprotect and step i+1's protect)")
    ap.add_argument("--policy", default="AES_CM_128_HMAC_SHA1_80",
                    help="protection profile; 'AES_CM_128_NULL_AUTH' (cipher only) is a "
                         "diagnostic split of the fused kernel, not the headline metric")
    return ap.parse_args()


def cpu_baseline(seconds: float, threads: int, pkt_len: int, ssrcs: int):
    """The oracle (C restatement of SRTPCryptoContext + SRTPCipherCTR + HMAC,
    reference call structure: one 16-B AES call per keystream block, HMAC
    re-keyed per packet) protecting+unprotecting config-2 packets on host
    cores, one sender/receiver transformer pair per thread, sharded by SSRC."""
    from oracle import oracle as O
    from libjitsi_amd import synth
    O.build()
    n = 4096
    per_thread_ssrc = max(1, ssrcs // threads)
    pol = O.Policy(1, 16, 1, 20, 10, 14)
    counts = [0] * threads
    stop = [False]

    def worker(t):
        b = synth.rtp_bundle(n, per_thread_ssrc, pkt_len, seed=synth.SEED_BASE + 2 + 1000 * t)
        (k, s), = synth.keys(2 + t, 1)
        fs = O.Factory(True, k, s, pol, pol, O.MODE_REF)
        fr = O.Factory(False, k, s, pol, pol, O.MODE_REF)
        ts, tr = O.Transformer(O.KIND_RTP, fs, fs), O.Transformer(O.KIND_RTP, fr, fr)
        step = -(-n // per_thread_ssrc)
        o = b.off.astype(np.int64)
        seg = b.seg.copy()
        while not stop[0]:
            ln = b.length.copy()
            st1 = O.process(ts, False, seg, b.off, ln, b.cap)
            st2 = O.process(tr, True, seg, b.off, ln, b.cap)
            assert (st1 == 0).all() and (st2 == 0).all()
            counts[t] += n
            q = ((seg[o + 2].astype(np.int64) << 8) | seg[o + 3]) + step
            seg[o + 2] = ((q >> 8) & 0xFF).astype(np.uint8)
            seg[o + 3] = (q & 0xFF).astype(np.uint8)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    time.sleep(seconds)
    stop[0] = True
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    return sum(counts) / dt, sum(counts), dt


def e2e_leg(b, pols, keys, n, L, local_rank, bundles, depth=3):
    """End-to-end through PCIe (SURVEY.md 8d "end-to-end: pinned host buffers,
    H2D + kernels + D2H"): the same workload's bundles held in pinned host
    slots of an SRTPPipeline, each bundle copied to HBM, processed, copied
    back.  Each slot alternates protect (sender) and unprotect (receiver) of
    its bundle, so its content returns to the original RTP every two bundles;
    the engine runs with checkReplay off (SRTPCryptoContext's config flag) so
    the repeated sequence numbers are processed in full, not dropped.
    Returns directional packets/s (one bundle = one direction) and PCIe GB/s."""
    from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPPipeline, SRTPTransformer
    eng = SRTPEngine(device=local_rank, check_replay=False, max_contexts=1 << 15,
                     max_factories=8, max_transformers=8, max_batch=n)
    k, s = keys
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng))
    nb = len(b.seg)
    pl = SRTPPipeline(eng, max_packets=n, max_seg_bytes=nb, depth=depth)
    for j in range(depth):
        sl = pl.slot(j)
        sl["seg"][:nb] = b.seg
        sl["off"][:n] = b.off
        sl["len"][:n] = b.length
        sl["cap"][:n] = b.cap
    use = [0] * depth

    def submit(i):
        j = i % depth
        rev = use[j] % 2 == 1
        pl.submit(j, rev, n, nb, tid=(rcv if rev else snd).tid)
        use[j] += 1

    warm = 2 * depth
    for i in range(warm):
        submit(i)
    for j in range(depth):
        pl.wait(j)
    t0 = time.perf_counter()
    for i in range(warm, warm + bundles):
        submit(i)
    for j in range(depth):
        pl.wait(j)
    dt = time.perf_counter() - t0
    ok = all(int((pl.slot(j)["status"][:n] != 0).sum()) == 0 for j in range(depth))
    pps = bundles * n / dt
    pcie = bundles * 2 * nb / dt / 1e9
    pl.close()
    return {"directional_pps": round(pps, 1), "round_trip_pps": round(pps / 2, 1),
            "pcie_gbps_h2d_plus_d2h": round(pcie, 2), "bundles": bundles, "depth": depth,
            "all_accepted": ok,
            "note": "pinned host slots -> H2D -> protect or unprotect -> D2H, bundles of the "
                    "same workload; checkReplay off so repeated bundles are processed in full"}


def main():
    args = parse_args()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # SRTP_BENCH_ONE_DEVICE=1 puts every rank on device 0: a rehearsal of the
    # N-rank path on a 1-GPU box (with --backend gloo; RCCL wants distinct GPUs)
    if os.environ.get("SRTP_BENCH_ONE_DEVICE") == "1":
        local_rank = 0
    if world > 1:
        torch.cuda.set_device(local_rank)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local_rank)

    from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, profile_policies, synth

    n, L, nssrc = args.packets, args.len, args.ssrcs
    # rank r owns its own SSRC shard: disjoint SSRC sets, per-GPU contexts only
    b = synth.rtp_bundle(n, nssrc, L, seed=synth.SEED_BASE + 2 + 7919 * rank)
    # context table: >= 1.6x the SSRCs (load <= 0.31 at 10k); its size sets the
    # sort's key width (2^15 slots + the invalid key: 16 bits = two radix passes)
    max_ctx = 1 << max(12, (int(1.6 * nssrc) - 1).bit_length())
    # The sender and the receiver side each get an engine of their own (its own
    # scratch, context table and bundle stream), as a send thread and a receive
    # thread would: step i's unprotect (receiver stream, after step i's protect)
    # overlaps step i+1's protect (sender stream).  --serial: one engine, one
    # stream, every kernel in order.
    eng = SRTPEngine(device=local_rank, max_contexts=max_ctx, max_factories=64,
                     max_transformers=64, max_batch=n)
    eng_r = eng if args.serial else SRTPEngine(device=local_rank, max_contexts=max_ctx,
                                               max_factories=64, max_transformers=64,
                                               max_batch=n)
    (k, s), = synth.keys(2 + rank, 1)
    if args.policy == "AES_CM_128_NULL_AUTH":
        from libjitsi_amd import SRTPPolicy as P
        pols = (P(1, 16, 0, 0, 0, 14),) * 2
    else:
        pols = profile_policies(args.policy)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng_r))

    off = torch.from_numpy(b.off.view(np.int32)).to(dev)
    cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)      # sender statuses
    st_r = torch.empty(n, dtype=torch.int32, device=dev)    # receiver statuses
    off64 = off.to(torch.int64)
    seq_step = -(-n // nssrc)  # packets per SSRC per bundle
    stream = torch.cuda.current_stream(dev)
    stream_r = stream if args.serial else torch.cuda.Stream(dev)

    def advance_seq(seg, k):
        """Advance every packet's RTP sequence number by k bundles' worth."""
        hi, lo = seg[off64 + 2].to(torch.int32), seg[off64 + 3].to(torch.int32)
        q = ((hi << 8) | lo) + k * seq_step
        seg[off64 + 2] = ((q >> 8) & 0xFF).to(torch.uint8)
        seg[off64 + 3] = (q & 0xFF).to(torch.uint8)

    # Every step gets its own bundle, staged in HBM before the clock starts
    # (bundle i = the base bundle with each SSRC's sequence numbers advanced i
    # bundles): the timed region is protect + unprotect only.  A ring of at
    # most RING bundles (RING x 319 MB); a step count beyond it re-sequences a
    # used bundle inside the loop.
    total = args.warmup + args.steps
    ring = min(total, RING)
    base = torch.from_numpy(b.seg).to(dev)
    len0 = torch.from_numpy(b.length.view(np.int32)).to(dev)
    segs, lens = [], []
    for i in range(ring):
        sg = base.clone()
        if i:
            advance_seq(sg, i)
        segs.append(sg)
        lens.append(len0.clone())
    del base
    torch.cuda.synchronize(dev)

    protected = [torch.cuda.Event() for _ in range(ring)]
    received = [None] * ring

    def step(i, serial=args.serial):
        j = i % ring
        if i >= ring:
            if received[j] is not None:
                stream.wait_event(received[j])  # unprotect of step i - ring is done
            advance_seq(segs[j], ring)
        eng.transform_device(False, snd.tid, segs[j], off, lens[j], cap, st, stream=stream)
        rs = stream if serial else stream_r
        if rs is not stream:
            protected[j].record(stream)
            rs.wait_event(protected[j])
        eng_r.transform_device(True, rcv.tid, segs[j], off, lens[j], cap, st_r, stream=rs)
        if rs is not stream:
            received[j] = torch.cuda.Event()
            received[j].record(rs)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    bad = int((st != 0).sum()) + int((st_r != 0).sum())
    if bad:
        hist = torch.bincount(torch.cat([st, st_r]).to(torch.int64), minlength=10).tolist()
        raise SystemExit(f"rank {rank}: {bad} packets not accepted after warmup; status "
                         f"histogram {hist}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.warmup, total):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ok = (int((st != 0).sum()) == 0 and int((st_r != 0).sum()) == 0
          and all(int((x != L).sum()) == 0 for x in lens))
    # Per-stage HIP-event timing (k_protect's launch duration for the roofline)
    # in a separate, untimed pass, serial (one stream, so no stage shares the
    # GPU with the other direction): the event records would otherwise sit
    # between the kernels of the timed steps.
    engines = [eng] if eng_r is eng else [eng, eng_r]
    for e in engines:
        e.set_timing(True)
        e.read_timing()
    for i in range(total, total + min(args.steps, 10)):
        step(i, serial=True)
    torch.cuda.synchronize(dev)
    timing = {}
    for e in engines:
        for key, (ms, cnt) in e.read_timing().items():
            m0, c0 = timing.get(key, (0.0, 0))
            timing[key] = (m0 + ms, c0 + cnt)
        e.set_timing(False)
    ok = ok and int((st != 0).sum()) == 0 and int((st_r != 0).sum()) == 0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    if world > 1:
        if args.backend != "nccl":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max = float(t.item())

    total_pkts = n * args.steps * world
    pps = total_pkts / dt_max
    T = pols[0].authTagLength
    alg_bytes_rt = 2 * (L + (L + T))  # protect L + (L+T), unprotect (L+T) + L
    gbs = pps * alg_bytes_rt / 1e9
    prot_ms, prot_cnt = timing["protect"]
    avg_prot_s = prot_ms / 1e3 / max(prot_cnt, 1)
    achieved = n * (L + (L + T)) / avg_prot_s / 1e9
    stages = {k: (v[0] / max(v[1], 1)) for k, v in timing.items() if v[1]}
    achieved_u = None
    if "verify" in stages and stages["verify"] > 0:
        achieved_u = n * (L + (L + T)) / (stages["verify"] / 1e3) / 1e9

    traffic = traffic_u = util = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("packets") == n and pmc.get("len") == L:
                traffic = pmc.get("k_protect_bytes_per_launch")
                traffic_u = pmc.get("k_unprotect_bytes_per_launch")
                util = pmc.get("k_protect_utilisation")
        except Exception:
            traffic = None

    # achievable HBM bandwidth on this device (plain device-to-device copy of
    # 512 MiB, read + write bytes), reported beside the 8 TB/s spec peak
    copy_gbs = None
    try:
        src = torch.empty(1 << 29, dtype=torch.uint8, device=dev)
        dst = torch.empty_like(src)
        dst.copy_(src)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize(dev)
        copy_gbs = round(5 * 2 * src.numel() / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)
        del src, dst
    except Exception:
        copy_gbs = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        v, cnt, cdt = cpu_baseline(args.cpu_seconds, threads, L, nssrc)
        cpu = {"value": round(v, 1), "unit": "packets/s", "cores": threads, "kind": "port",
               "sample": f"oracle/srtp_oracle.c (reference call structure, OpenSSL 3 AES-ECB per "
                         f"16-B block + HMAC re-keyed per packet): {cnt} packets of {L} B "
                         f"protected+unprotected in {cdt:.1f} s on {threads} threads, "
                         f"4096-packet bundles, {nssrc} SSRCs split across threads",
               "gbps": round(v * alg_bytes_rt / 1e9, 3)}

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e:
        del segs, lens
        torch.cuda.empty_cache()
        e2e = e2e_leg(b, pols, (k, s), n, L, local_rank, args.e2e_bundles)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(pps, 1),
            "unit": "packets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic RTP packets, random payload, seeded keys)",
            "config": {"workload": "configs[1]: 10k concurrent SSRCs x 1200-B RTP, "
                                   "AES_CM_128_HMAC_SHA1_80, protect then unprotect",
                       "packets_per_gpu_per_step": n, "ssrcs_per_gpu": nssrc, "pkt_len": L,
                       "parallelism": f"ssrc-sharded x{world}",
                       "streams": "serial" if args.serial else
                                  "sender + receiver engine, one stream each"},
            "gbps": round(gbs, 2),
            "goodput_gbps": round(pps * L * 2 / 1e9, 2),
            "all_accepted": ok,
            "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            "roofline": {"bound": "hbm", "kernel": "k_protect", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_source": "rocprofv3 FETCH_SIZE/WRITE_SIZE per k_protect launch, "
                                           "profiles/pmc_traffic.json" if traffic else None,
                         "copy_measured_gbps": copy_gbs,
                         "utilisation": util,
                         "algorithmic_bytes_per_launch": n * (L + L + T)},
            "roofline_k_unprotect": None if achieved_u is None else {
                "bound": "hbm", "achieved": round(achieved_u, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved_u / HBM_PEAK_GBS, 4), "traffic": traffic_u,
                "note": "the other dominant kernel (unprotect: tag check + speculative decryption), "
                        "same algorithmic bytes per packet, HIP events of the same serial pass"},
            "cpu_baseline": cpu,
            "e2e": e2e,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
