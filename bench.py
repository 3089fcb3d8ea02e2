#!/usr/bin/env python3
"""SRTP protect+unprotect throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1], one bundle per GPU per step): 10,000
concurrent SSRCs, fixed 1200-byte video RTP packets, AES_CM_128_HMAC_SHA1_80,
bundles of 2^18 packets resident in HBM.  A sender SRTPTransformer protects
bundles and a separate receiver transformer unprotects them, each
on its own engine and HIP stream, as a bridge's send and receive threads do.
Step i protects bundle i and unprotects bundle i-1 (protected the step
before); the two streams join at the end of every step, so a step is always
one protect and one unprotect of 2^18 packets and the timed steps have no
start or end transient.  Every bundle is staged in HBM before the clock
starts: bundle i is the base bundle with every SSRC's sequence numbers
advanced by i times its packets per bundle (fresh packets for the replay
check; ROC wraps happen naturally).  ``--serial``: one engine, one stream,
step i = protect(i) then unprotect(i).

Multi-GPU: one process per GPU (torchrun), contexts sharded by SSRC (each rank
owns its own SSRCs), no collective on the data path ("scaling": "weak").
Without torchrun, ``--gpus N`` starts the N processes itself (rank r on GPU r,
rendezvous on 127.0.0.1), before anything touches a GPU, so no GPU's steps
wait for another's Python; ``SRTP_BENCH_INPROC=1`` drives the N GPUs from this
one process instead (one host thread each, sharing the GIL: the in-process
deployment).  ``SRTP_BENCH_ONE_DEVICE=1`` puts all N on device 0, a rehearsal
on a one-GPU box (with ``--backend gloo`` in process mode).  value = packets protected AND unprotected by all
GPUs / wall time (max over ranks).  The line also reports the host time spent
enqueueing a step, per GPU.

Also reported: the dominant kernel's roofline (HIP events on the bundle
stream, algorithmic bytes L + (L+T) per packet), and a CPU baseline: the
oracle's pinned C timing loop (oracle/oracle_bench.c) in the reference's call
structure and a tuned-OpenSSL variant, on one core and on the box's CPU share.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
RING = 160  # most distinct bundles staged in HBM per GPU (x 319 MB at the default size)
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
    ap.add_argument("--keysets", type=int, default=1,
                    help="sender/receiver transformer pairs, each with its own master key: SSRC s "
                         "belongs to pair s %% K (a bridge's many DTLS sessions in one bundle)")
    ap.add_argument("--zipf", type=float, default=0.0,
                    help="SSRC popularity Zipf exponent (0: round-robin, every SSRC equal)")
    ap.add_argument("--len", type=int, default=1200, help="RTP packet length")
    ap.add_argument("--align", type=int, default=16,
                    help="packet region alignment in the bundle segment (bytes, >= 16)")
    ap.add_argument("--cpu-seconds", type=float, default=3.0,
                    help="CPU baseline: seconds per measurement (4 measurements)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the box's CPU share: min(16, CPUs in the affinity set)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned-host end-to-end leg")
    ap.add_argument("--e2e-bundles", type=int, default=24)
    ap.add_argument("--no-dispatch", action="store_true",
                    help="skip the dispatcher leg (host bundles through srtp_dispatch_transform_host)")
    ap.add_argument("--dispatch-shards", default="",
                    help="comma-separated shard counts of the dispatcher leg (default: 1,2,4 on one "
                         "GPU, else the GPU count)")
    ap.add_argument("--dispatch-bundles", type=int, default=8)
    ap.add_argument("--dispatch-in-process", action="store_true",
                    help="run the whole dispatcher leg in this (torch) process instead of a torch-free child")
    ap.add_argument("--dispatch-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--backend", default="nccl",
                    help="torch.distributed backend for the barrier/timing reduction (nccl = RCCL)")
    ap.add_argument("--serial", action="store_true",
                    help="one engine and stream: step i = protect(i) then unprotect(i)")
    ap.add_argument("--pipe", default="free", choices=["free", "join", "lag1", "lag2"],
                    help="coupling of the sender and receiver streams (see Side.step)")
    ap.add_argument("--events", default="device", choices=["device", "torch"],
                    help="events ordering the two streams: 'device' = device-scope release (no "
                         "system-scope fence: no L2 write-back between the directions), "
                         "'torch' = torch.cuda.Event (system scope)")
    ap.add_argument("--policy", default="AES_CM_128_HMAC_SHA1_80",
                    help="protection profile; 'AES_CM_128_NULL_AUTH' (cipher only) is a "
                         "diagnostic split of the fused kernel, not the headline metric")
    return ap.parse_args()


def cpu_info():
    """Model name and physical core count of the host (lscpu)."""
    info = {"cpu_model": None, "physical_cores": None, "logical_cpus": os.cpu_count()}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=20).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["cpu_model"] = kv.get("Model name")
        if kv.get("Core(s) per socket") and kv.get("Socket(s)"):
            info["physical_cores"] = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
        info["flags_aes_sha"] = {f: f in kv.get("Flags", "").split() for f in ("aes", "sha_ni", "vaes")}
    except Exception:
        pass
    return info


def cpu_baseline(seconds: float, threads: int, L: int, nssrc: int, T: int):
    """The oracle's pinned C loop (oracle/oracle_bench.c): each thread owns a
    sender/receiver transformer pair and its share of the SSRCs, and protects
    then unprotects 4096-packet bundles of L-byte packets.  MODE_REF follows the
    reference's call structure (SRTPCipherCTR.java:68-121: one 16-B AES-ECB call
    per keystream block plus the tail block; BaseSRTPCryptoContext.java:269-278
    with the HMAC re-keyed per packet), MODE_TUNED uses one EVP AES-CTR call per
    packet and a pre-keyed HMAC context."""
    from oracle import oracle as O
    O.build()
    res = {}
    for name, mode in (("ref", O.MODE_REF), ("tuned", O.MODE_TUNED)):
        for tag, th in (("one_core", 1), ("share", threads)):
            n, el = O.bench_round_trips(mode, th, seconds, L, nssrc)
            res[(name, tag)] = (n / el, n, el)
    alg = 2 * (L + (L + T))
    info = cpu_info()

    def obj(name):
        v1, n1, e1 = res[(name, "one_core")]
        vn, nn, en = res[(name, "share")]
        o = {"value": round(vn, 1), "threads": threads, "one_core": round(v1, 1),
             "gbps": round(vn * alg / 1e9, 3), "packets": nn, "seconds": round(en, 2)}
        if info.get("physical_cores"):
            o["per_core_x_physical_cores"] = round(v1 * info["physical_cores"], 1)
        return o

    ref, tuned = obj("ref"), obj("tuned")
    return {"value": ref["value"], "unit": "packets/s", "cores": threads, "threads": threads,
            "kind": "port",
            "sample": f"oracle/oracle_bench.c pinned C loop, {threads} threads (the box's CPU "
                      f"share) and 1 thread, {seconds:.0f} s each: 4096-packet bundles of {L}-B "
                      f"RTP over {nssrc} SSRCs split across threads, protect then unprotect "
                      f"(reference call structure; 'tuned' = EVP AES-CTR per packet + pre-keyed "
                      f"HMAC)",
            "ref": ref, "tuned": tuned, **info,
            "note": "cores = threads used (min(16, the affinity set): the box's CPU share, not "
                    "a count of physical cores); per_core_x_physical_cores is an extrapolation "
                    "of the 1-thread rate to every physical core, not a measurement"}


class E2E:
    """End-to-end through PCIe (SURVEY.md 8d "end-to-end: pinned host buffers,
    H2D + kernels + D2H") on one GPU: the same workload's bundles held in
    pinned host slots of an SRTPPipeline, each bundle copied to HBM,
    processed, copied back.  Each slot alternates protect (sender) and
    unprotect (receiver) of its bundle, so its content returns to the original
    RTP every two bundles; the engine runs with checkReplay off
    (SRTPCryptoContext's config flag) so the repeated sequence numbers are
    processed in full, not dropped.  Several GPUs run it at once (one E2E per
    GPU, started together), which is the PCIe / host-memory bound scaling
    curve of the north star's deployment."""

    def __init__(self, b, pols, keys, n, device, depth=3):
        from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPPipeline, SRTPTransformer
        self.eng = SRTPEngine(device=device, check_replay=False, max_contexts=1 << 15,
                              max_factories=8, max_transformers=8, max_batch=n)
        k, s = keys
        self.snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=self.eng))
        self.rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=self.eng))
        self.nb = nb = len(b.seg)
        self.n, self.depth = n, depth
        self.pl = SRTPPipeline(self.eng, max_packets=n, max_seg_bytes=nb, depth=depth)
        for j in range(depth):
            sl = self.pl.slot(j)
            sl["seg"][:nb] = b.seg
            sl["off"][:n] = b.off
            sl["len"][:n] = b.length
            sl["cap"][:n] = b.cap
        self.use = [0] * depth
        self.i = 0

    def _submit(self):
        j = self.i % self.depth
        rev = self.use[j] % 2 == 1
        self.pl.submit(j, rev, self.n, self.nb, tid=(self.rcv if rev else self.snd).tid)
        self.use[j] += 1
        self.i += 1

    def _drain(self):
        for j in range(self.depth):
            self.pl.wait(j)

    def warm(self):
        for _ in range(2 * self.depth):
            self._submit()
        self._drain()

    def run(self, bundles):
        """(seconds, packets, H2D + D2H bytes, all accepted) of `bundles` bundles."""
        t0 = time.perf_counter()
        for _ in range(bundles):
            self._submit()
        self._drain()
        dt = time.perf_counter() - t0
        ok = all(int((self.pl.slot(j)["status"][:self.n] != 0).sum()) == 0 for j in range(self.depth))
        return dt, bundles * self.n, bundles * 2 * self.nb, ok

    def close(self):
        self.pl.close()
        self.eng.close()


def e2e_summary(dt, pkts, nbytes, ok, n_gpus, bundles, depth):
    pps = pkts / dt
    return {"directional_pps": round(pps, 1), "round_trip_pps": round(pps / 2, 1),
            "pcie_gbps_h2d_plus_d2h": round(nbytes / dt / 1e9, 2), "bundles_per_gpu": bundles,
            "depth": depth, "n_gpus": n_gpus, "all_accepted": ok,
            "note": "pinned host slots -> H2D -> protect or unprotect -> D2H, bundles of the "
                    "same workload, every GPU at once; checkReplay off so repeated bundles are "
                    "processed in full; rates are whole-job (all GPUs)"}


def dispatch_leg(b, pols, keys, n, devices_for, shard_counts, bundles, modes=None):
    """Host bundles through the in-process dispatcher (srtp_dispatch_transform_host):
    the deployment path of one JVM driving every GPU.  For each shard count G
    (devices_for(G) = the device of each shard), protect then unprotect the
    same bundle (checkReplay off), and report packets/s per direction and the
    dispatcher's host time per bundle: plan + split, packing into the shards'
    pinned slots, waiting for the shards (H2D + kernels + D2H), scattering
    back (the last three summed over the shards' worker threads).  Each G runs
    with the bundle in the engine's pinned memory (HostBuffer / srtp_host_alloc,
    key "G": a shard's chunk whose packets lie back to back moves by DMA in
    place, no host copy) and in plain pageable memory (key "G_copy": every
    packet copied into the pinned slots and back); G = 1 also with pageable
    memory registered once (srtp_host_register, key "1_registered"), and with
    two bundles in flight (srtp_dispatch_submit_host, key "G_async")."""
    from libjitsi_amd import (HostBuffer, SRTPContextFactory, SRTPDispatcher, SRTPTransformer,
                              host_register, host_unregister)
    out = {}
    if modes is None:
        modes = [(G, m) for G in shard_counts for m in ("pinned", "async", "copy")] + [(1, "registered")]
    for G, mode in modes:
        d = SRTPDispatcher(devices_for(G), check_replay=False, max_contexts=1 << 15,
                           max_factories=8, max_transformers=8)
        seg = hb = None
        try:
            k, s = keys
            snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=d))
            rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=d))
            ln = b.length.copy()
            if mode in ("pinned", "async"):  # the engine's pinned buffer pool: chunks DMA in place
                hb = HostBuffer(b.seg.nbytes)
                seg = hb.array
                seg[:] = b.seg
            else:
                seg = b.seg.copy()
                if mode == "registered":  # pageable memory registered once
                    host_register(seg)
            for _ in range(2):  # warm: both directions once
                d.transform_host(False, snd.tid, seg, b.off, ln, b.cap)
                d.transform_host(True, rcv.tid, seg, b.off, ln, b.cap)
            if mode == "async":  # a second pinned bundle: one in flight while the other is packed
                hb2 = HostBuffer(b.seg.nbytes)
                hb2.array[:] = b.seg
                bufs = [(seg, ln), (hb2.array, b.length.copy())]
            h0 = d.host_times()
            ok = True
            t0 = time.perf_counter()
            if mode == "async":
                # srtp_dispatch_submit_host / wait_host, two bundles in flight:
                # P(A) P(B) U(A) U(B) ..., each submit after the wait of the
                # previous operation on its buffer (the oldest in flight)
                pending, t_sub, t_wait = [], [], []
                for _ in range(bundles):
                    for rev, t in ((False, snd), (True, rcv)):
                        for sg, l in bufs:
                            if len(pending) == 2:
                                a0 = time.perf_counter()
                                st_w = pending.pop(0).wait()
                                t_wait.append(time.perf_counter() - a0)
                                ok = ok and not st_w.any()
                            a0 = time.perf_counter()
                            pending.append(d.submit_host(rev, t.tid, sg, b.off, l, b.cap))
                            t_sub.append(time.perf_counter() - a0)
                for tk in pending:
                    ok = ok and not tk.wait().any()
                pending = None
                dt = (time.perf_counter() - t0) / 2  # twice the bundles of the other modes
                op_ms = {"submit_ms_p50": round(float(np.median(t_sub)) * 1e3, 3),
                         "submit_ms_max": round(max(t_sub) * 1e3, 3),
                         "wait_ms_p50": round(float(np.median(t_wait)) * 1e3, 3),
                         "wait_ms_max": round(max(t_wait) * 1e3, 3)}
            else:
                for _ in range(bundles):
                    st = d.transform_host(False, snd.tid, seg, b.off, ln, b.cap)
                    st2 = d.transform_host(True, rcv.tid, seg, b.off, ln, b.cap)
                    ok = ok and not st.any() and not st2.any()
                dt = time.perf_counter() - t0
            h1 = d.host_times()
            calls = max(h1["calls"] - h0["calls"], 1)
            per = {k2: round((h1[k2] - h0[k2]) / calls, 3) for k2 in h1 if k2 != "calls"}
            extra = {}
            if mode == "async":
                bufs = None
                hb2.close()
                extra = {"async_ops": op_ms}
            out[str(G) if mode == "pinned" else f"{G}_{mode}"] = {**extra,
                "directional_pps": round(2 * bundles * n / dt, 1),
                "ms_per_bundle": round(dt / (2 * bundles) * 1e3, 3),
                "host_ms_per_bundle": per, "all_accepted": bool(ok),
                "devices": sorted(set(devices_for(G))), "segment": mode}
        finally:
            d.close()
            if mode == "registered" and seg is not None:
                host_unregister(seg)
            if hb is not None:
                seg = None
                hb.close()
    return out


def policies(args):
    from libjitsi_amd import SRTPPolicy, profile_policies
    if args.policy == "AES_CM_128_NULL_AUTH":
        return (SRTPPolicy(1, 16, 0, 0, 0, 14),) * 2
    return profile_policies(args.policy)


def world_devices(args):
    """The devices of a one-process run (--gpus N in-process, or rank 0)."""
    if args.gpus > 1:
        one = os.environ.get("SRTP_BENCH_ONE_DEVICE") == "1"
        return [0] * args.gpus if one else list(range(args.gpus))
    return [0 if os.environ.get("SRTP_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))]


def dispatch_plan(args, devices):
    """Shard counts of the dispatcher leg and the device of each shard."""
    if args.dispatch_shards:
        counts = [int(x) for x in args.dispatch_shards.split(",")]
    else:
        counts = [1, 2, 4] if len(devices) == 1 else [len(devices)]

    def devs_for(G):
        return [devices[i % len(devices)] for i in range(G)]
    return counts, devs_for


def dispatch_child(args) -> int:
    """--dispatch-child: the dispatcher leg in a process that never imports
    torch.  The torch wheel ships its own HIP runtime (ROCm 7.0,
    torch/lib/libamdhip64.so, SONAME libamdhip64.so.7): in a process that
    imported torch first, libsrtp_mi355x binds to it, and the two-in-flight
    dispatcher runs at half its rate there (profiles/r05/dispatch/
    hip_runtime.txt).  A JVM or C host loads /opt/rocm's runtime, as this
    process does.  Started by the bench before it touches a GPU; idle until
    the parent writes "go" (after its own GPU legs), then prints the leg's
    JSON object and exits.  EOF on stdin: exits without touching the GPU."""
    from libjitsi_amd import synth
    pols = policies(args)
    b, _ = shard_bundle(args, 0)
    keys = synth.keys(2, 1)[0]
    counts, devs_for = dispatch_plan(args, world_devices(args))
    if sys.stdin.readline().strip() != "go":
        return 0
    out = dispatch_leg(b, pols, keys, args.packets, devs_for, counts, args.dispatch_bundles)
    with open("/proc/self/maps") as f:
        out["hip_runtime"] = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    out["torch_imported"] = "torch" in sys.modules
    print(json.dumps(out), flush=True)
    return 0


def dispatch_child_result(child):
    """Start the idle --dispatch-child on its leg and collect its JSON."""
    try:
        out, err = child.communicate("go\n", timeout=900)
    except subprocess.TimeoutExpired:
        child.kill()
        child.communicate()
        return {"error": "dispatcher child timed out"}
    lines = [x for x in out.splitlines() if x.startswith("{")]
    if child.returncode != 0 or not lines:
        return {"error": f"dispatcher child exit {child.returncode}: {err.strip()[-400:]}"}
    return json.loads(lines[-1])


class DeviceEvent:
    """A stream-ordering event with a device-scope release
    (hipEventDisableSystemFence): the two directions' streams are on one GPU
    and only its kernels read what the other stream wrote, so the system-scope
    fence a torch.cuda.Event record carries (an L2 write-back and invalidate,
    ~13 us of idle queue per record, profiles/r05/events/) is not needed."""
    _hip = None

    def __init__(self):
        import ctypes
        if DeviceEvent._hip is None:
            h = ctypes.CDLL("libamdhip64.so")
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipStreamWaitEvent.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            DeviceEvent._hip = h
        self.h = ctypes.c_void_p()
        rc = DeviceEvent._hip.hipEventCreateWithFlags(ctypes.byref(self.h), 0x2 | 0x20000000)
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: {rc}")

    def record(self, stream):
        rc = DeviceEvent._hip.hipEventRecord(self.h, stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: {rc}")

    def wait(self, stream):
        rc = DeviceEvent._hip.hipStreamWaitEvent(stream.cuda_stream, self.h, 0)
        if rc != 0:
            raise RuntimeError(f"hipStreamWaitEvent: {rc}")


class TorchEvent:
    """torch.cuda.Event behind DeviceEvent's record / wait."""

    def __init__(self, torch):
        self.ev = torch.cuda.Event()

    def record(self, stream):
        self.ev.record(stream)

    def wait(self, stream):
        stream.wait_event(self.ev)


def shard_bundle(args, shard: int):
    """Shard r's bundle (its own SSRCs) and each packet's stream length."""
    from libjitsi_amd import synth
    n, L, nssrc = args.packets, args.len, args.ssrcs
    seed = synth.SEED_BASE + 2 + 7919 * shard
    if args.zipf > 0:
        b = synth.rtp_bundle_skewed(n, nssrc, L, seed=seed, zipf_s=args.zipf)
        counts = b.meta["counts"]
    else:
        b = synth.rtp_bundle(n, nssrc, L, seed=seed)
        idx = np.arange(n) % nssrc
        counts = np.bincount(idx, minlength=nssrc)[idx]
    return synth.realign(b, args.align), counts


class Side:
    """One GPU's share: a sender engine + stream, a receiver engine + stream,
    and the ring of staged bundles."""

    def __init__(self, torch, device: int, shard: int, args, pols, total: int):
        from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, synth
        self.torch = torch
        dev = self.dev = torch.device("cuda", device)
        n, L, nssrc = args.packets, args.len, args.ssrcs
        b, counts = shard_bundle(args, shard)
        self.b = b
        # max_contexts = the streams, as a deployment sets it: the engine's table
        # is next_pow2(2 x max_contexts) slots (2^15 at 10k: load 0.31; 2^18 at
        # 100k: 0.38), and its size sets the sort's key width (slot bits + 1)
        max_ctx = max(1 << 12, nssrc)
        K = max(1, args.keysets)
        mk = dict(device=device, max_contexts=max_ctx, max_factories=max(64, 2 * K + 8),
                  max_transformers=max(64, 2 * K + 8), max_batch=n)
        self.eng = SRTPEngine(**mk)
        self.eng_r = self.eng if args.serial else SRTPEngine(**mk)
        (k, s), = synth.keys(2 + shard, 1)
        self.keys = (k, s)
        self.snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=self.eng))
        self.rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=self.eng_r))
        self.tid_s, self.tid_r = self.snd.tid, self.rcv.tid
        if K > 1:  # K key sets: per-packet transformer ids (srtp_transform_device tids[])
            ks = synth.keys(1000 + 97 * shard, K - 1)
            snd, rcv = [self.snd], [self.rcv]
            for kk, ss in ks:
                snd.append(SRTPTransformer(SRTPContextFactory(True, kk, ss, *pols, engine=self.eng)))
                rcv.append(SRTPTransformer(SRTPContextFactory(False, kk, ss, *pols, engine=self.eng_r)))
            self._tr_keep = (snd, rcv)
            pair = np.arange(n) % nssrc % K
            ts_np = np.array([t.tid for t in snd], np.int32)[pair]
            tr_np = np.array([t.tid for t in rcv], np.int32)[pair]
        with torch.cuda.device(dev):
            if K > 1:
                self.tid_s = torch.from_numpy(ts_np).to(dev)
                self.tid_r = torch.from_numpy(tr_np).to(dev)
            self.off = torch.from_numpy(b.off.view(np.int32)).to(dev)
            self.cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
            self.st = torch.empty(n, dtype=torch.int32, device=dev)
            self.st_r = torch.empty(n, dtype=torch.int32, device=dev)
            self.off64 = self.off.to(torch.int64)
            self.step_seq = torch.from_numpy(counts.astype(np.int32)).to(dev)
            # each engine's own stream: created with the engine, each gets a
            # hardware queue of its own (two streams made later may share one,
            # which serialises the two directions)
            self.s_a = torch.cuda.ExternalStream(self.eng.stream_ptr, device=dev)
            self.s_b = (self.s_a if args.serial else
                        torch.cuda.ExternalStream(self.eng_r.stream_ptr, device=dev))
            mkev = DeviceEvent if args.events == "device" else (lambda: TorchEvent(torch))
            self.end_a, self.end_b = mkev(), mkev()
            self.ev_b = [mkev() for _ in range(3)]  # receiver step ends (lag modes)
            self.ring = min(total + 1, RING)
            # ring slot j is free again once the unprotect of its last bundle ran
            # (recorded only when the run reuses slots)
            self.reuse = total + 1 > self.ring
            self.ev_free = [mkev() for _ in range(self.ring)] if self.reuse else []
            self.pending = None  # join mode: protected bundle whose unprotect is due
            base = torch.from_numpy(b.seg).to(dev)
            len0 = torch.from_numpy(b.length.view(np.int32)).to(dev)
            self.segs, self.lens = [], []
            for i in range(self.ring):
                sg = base.clone()
                if i:
                    self.advance_seq(sg, i)
                self.segs.append(sg)
                self.lens.append(len0.clone())
            del base
        torch.cuda.synchronize(dev)
        self.serial = args.serial
        self.pipe = args.pipe
        self.n, self.L = n, L

    def advance_seq(self, seg, k):
        """Advance every packet's RTP sequence number by k bundles' worth."""
        o = self.off64
        hi, lo = seg[o + 2].to(self.torch.int32), seg[o + 3].to(self.torch.int32)
        q = ((hi << 8) | lo) + k * self.step_seq
        seg[o + 2] = ((q >> 8) & 0xFF).to(self.torch.uint8)
        seg[o + 3] = (q & 0xFF).to(self.torch.uint8)

    def protect(self, i, stream):
        j = i % self.ring
        if i >= self.ring:  # reuse a staged bundle once its unprotect has run
            self.ev_free[j].wait(stream)
            with self.torch.cuda.stream(stream):
                self.advance_seq(self.segs[j], self.ring)
        self.eng.transform_device(False, self.tid_s, self.segs[j], self.off, self.lens[j],
                                  self.cap, self.st, stream=stream)

    def unprotect(self, i, stream):
        j = i % self.ring
        self.eng_r.transform_device(True, self.tid_r, self.segs[j], self.off, self.lens[j],
                                    self.cap, self.st_r, stream=stream)
        if self.reuse:
            self.ev_free[j].record(stream)

    def step(self, i):
        """free: protect(i) on stream A, unprotect(i) on stream B after it; the
        sender never waits for the receiver (the ring is deep enough).
        lagK: as free, but protect(i) waits until unprotect(i - K) is done.
        join: protect(i) on A beside unprotect(i - 1) on B, both after the
        previous step's join.  Serial: protect(i) then unprotect(i) on one
        stream."""
        if self.serial:
            self.protect(i, self.s_a)
            self.unprotect(i, self.s_a)
            return
        if self.pipe != "join":
            lag = {"free": 0, "lag1": 1, "lag2": 2}[self.pipe]
            if lag and i >= lag:
                self.ev_b[(i - lag) % 3].wait(self.s_a)
            self.protect(i, self.s_a)
            self.end_a.record(self.s_a)
            self.end_a.wait(self.s_b)
            self.unprotect(i, self.s_b)
            if lag:
                self.ev_b[i % 3].record(self.s_b)
            return
        self.end_b.wait(self.s_a)
        self.end_a.wait(self.s_b)
        self.protect(i, self.s_a)
        if self.pending is not None:
            self.unprotect(self.pending, self.s_b)
        self.pending = i
        self.end_a.record(self.s_a)
        self.end_b.record(self.s_b)

    def serial_step(self, i):
        """protect(i) then unprotect(i) on stream A (the stage-timing pass)."""
        self.end_b.wait(self.s_a)
        if self.pending is not None:
            self.unprotect(self.pending, self.s_a)
            self.pending = None
        self.protect(i, self.s_a)
        self.unprotect(i, self.s_a)
        self.end_a.record(self.s_a)

    def finish(self):
        """Unprotect the last protected bundle (join mode), untimed."""
        if self.pending is not None:
            self.end_a.wait(self.s_b)
            self.unprotect(self.pending, self.s_b)
            self.pending = None
        self.torch.cuda.synchronize(self.dev)

    def bad(self):
        return int((self.st != 0).sum()) + int((self.st_r != 0).sum())

    def engines(self):
        return [self.eng] if self.eng_r is self.eng else [self.eng, self.eng_r]


def status_counts(sides):
    """(packets submitted, packets finished OK) over every engine of every GPU
    (srtp_engine_stats), so that every step's statuses are checked, not only
    the last one's."""
    sub = ok = 0
    for sd in sides:
        for e in sd.engines():
            st = e.stats()
            sub += st["packets"]
            ok += st["status"]["OK"]
    return sub, ok


def run_steps(torch, sides, g0, warmup, steps, barrier=None):
    """Warmup then `steps` timed steps on every side.  One side: this thread.
    Several (in-process mode): one host thread per GPU, started together
    behind a barrier.  Returns (t_start, t_end, host seconds spent enqueueing
    the timed steps, per side)."""
    import threading

    def body(i, sd, res):
        torch.cuda.set_device(sd.dev)
        for w in range(warmup):
            sd.step(g0 + w)
        torch.cuda.synchronize(sd.dev)
        if barrier is not None:
            barrier.wait()
        t0 = time.perf_counter()
        enq = 0.0
        for k in range(steps):
            a = time.perf_counter()
            sd.step(g0 + warmup + k)
            enq += time.perf_counter() - a
        torch.cuda.synchronize(sd.dev)
        res[i] = (t0, time.perf_counter(), enq)

    res = [None] * len(sides)
    if len(sides) == 1:
        body(0, sides[0], res)
    else:
        bar = threading.Barrier(len(sides))
        barrier = bar
        th = [threading.Thread(target=body, args=(i, sd, res)) for i, sd in enumerate(sides)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    return min(r[0] for r in res), max(r[1] for r in res), [r[2] for r in res]


def spawn_ranks(n: int) -> int:
    """--gpus N without torchrun: one child process per GPU, started before
    this process touches a GPU (it never does), each a torchrun-style rank on
    127.0.0.1.  Rank 0's stdout (the JSON line) is passed through."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    args = parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1 and os.environ.get("SRTP_BENCH_INPROC") != "1":
        sys.exit(spawn_ranks(args.gpus))
    if args.dispatch_child:
        sys.exit(dispatch_child(args))
    child = None
    if world == 1 and not args.no_dispatch and not args.dispatch_in_process:
        # the dispatcher leg's torch-free process, started before this one
        # touches a GPU (dispatch_child)
        child = subprocess.Popen([sys.executable, os.path.abspath(__file__), "--dispatch-child"] + sys.argv[1:],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                 text=True)
    try:
        return run_bench(args, world, child)
    finally:
        if child is not None and child.poll() is None:
            child.kill()
            child.communicate()


def run_bench(args, world, child):
    import torch
    import torch.distributed as dist

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
        devices = [local_rank]
        mode = "process"
    elif args.gpus > 1:
        # in-process: this process drives every GPU (all on device 0 for a rehearsal)
        devices = world_devices(args)
        mode = "inproc"
    else:
        devices = [local_rank]
        mode = "process"
    n_gpus = world if mode == "process" else len(devices)

    pols = policies(args)
    n, L = args.packets, args.len
    T = pols[0].authTagLength
    n_timing = 40  # serial stage-timing steps (also the GPU's run-in before the warmup)
    total = n_timing + args.warmup + args.steps
    sides = [Side(torch, d, rank if mode == "process" else i, args, pols, total)
             for i, d in enumerate(devices)]
    sd0 = sides[0]
    g = 0  # global step counter: each step has bundles of its own (fresh sequence numbers)
    for sd in sides:  # loads the status-check kernels now, not between passes
        sd.bad()

    # achievable HBM bandwidth on this device (plain device-to-device copy of
    # 512 MiB, read + write bytes), reported beside the 8 TB/s spec peak
    copy_gbs = None
    try:
        with torch.cuda.device(sd0.dev):
            src = torch.empty(1 << 29, dtype=torch.uint8, device=sd0.dev)
            dst = torch.empty_like(src)
            dst.copy_(src)
            torch.cuda.synchronize(sd0.dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                dst.copy_(src)
            e1.record()
            torch.cuda.synchronize(sd0.dev)
            copy_gbs = round(5 * 2 * src.numel() / (e0.elapsed_time(e1) / 1e3) / 1e9, 1)
            del src, dst
    except Exception:
        copy_gbs = None

    # 1. Per-stage HIP-event timing (the roofline kernels' launch durations),
    # untimed, serial on the first GPU (one stream: no stage shares the GPU
    # with the other direction).  It runs right before the warmup, so that the
    # GPU is busy, every kernel is loaded and the clocks are up when it starts.
    engines = [sd0.eng] if sd0.eng_r is sd0.eng else [sd0.eng, sd0.eng_r]
    for e in engines:
        e.set_timing(True)
        e.read_timing()
    for _ in range(n_timing):
        sd0.serial_step(g)
        g += 1
    for sd in sides[1:]:  # the other GPUs warm up the same way (untimed)
        for k in range(n_timing):
            sd.serial_step(k)
    torch.cuda.synchronize(sd0.dev)
    timing = {}
    for e in engines:
        for key, (ms, cnt) in e.read_timing().items():
            m0, c0 = timing.get(key, (0.0, 0))
            timing[key] = (m0 + ms, c0 + cnt)
        e.set_timing(False)
    ok = sd0.bad() == 0

    # 2. Warmup, straight into the timed steps: no host work between them but
    # the synchronisation the timing needs (an idle GPU lowers its clocks, and
    # the first steps after a gap run slow).  Every step's statuses are checked
    # through the engines' counters (before / after), not only the last one's.
    sub0, ok0 = status_counts(sides)
    if world > 1:
        dist.barrier()
    for sd in sides:
        torch.cuda.synchronize(sd.dev)
    if world > 1:
        dist.barrier()
    t_start, t_end, enq = run_steps(torch, sides, g, args.warmup, args.steps)
    if world > 1:
        dist.barrier()
    g += args.warmup + args.steps
    dt = t_end - t_start
    for sd in sides:
        sd.finish()
    sub1, ok1 = status_counts(sides)
    ok = ok and sub1 - sub0 == ok1 - ok0 and sub1 > sub0
    ok = ok and all(sd.bad() == 0 and all(int((x != L).sum()) == 0 for x in sd.lens[:min(g, sd.ring)])
                    for sd in sides)
    enqueue_us = [round(x / args.steps * 1e6, 1) for x in enq]
    t = torch.tensor([dt], dtype=torch.float64, device=sd0.dev)
    if world > 1:
        if args.backend != "nccl":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt_max = float(t.item())
    # slow-path work per bundle over the whole run (run-in, warmup, timed steps)
    slow = {"long_walked": 0, "repaired": 0, "roc_rechecks": 0, "bundles": 0}
    for e in engines:  # the first GPU's engines
        s = e.stats()
        for k in slow:
            slow[k] += s[k]
    slow_per_bundle = {k: round(v / max(slow["bundles"], 1), 1) for k, v in slow.items() if k != "bundles"}

    total_pkts = n * args.steps * n_gpus
    pps = total_pkts / dt_max
    alg_bytes_rt = 2 * (L + (L + T))  # protect L + (L+T), unprotect (L+T) + L
    gbs = pps * alg_bytes_rt / 1e9
    stages = {k: (v[0] / max(v[1], 1)) for k, v in timing.items() if v[1]}
    alg_launch = n * (L + (L + T))

    pmc = {}
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("packets") != n or pmc.get("len") != L:
                pmc = {}
        except Exception:
            pmc = {}
    # the counters are of the build whose kernel sources hash to this; another
    # build's counters are reported as stale (traffic_stale), not as this one's
    from libjitsi_amd._native import kernel_source_sha16
    ksha = kernel_source_sha16()
    pmc_stale = bool(pmc) and pmc.get("kernel_source_sha16") != ksha

    def roofline(stage, kernel, traffic_key, util_key=None):
        if stage not in stages or stages[stage] <= 0:
            return None
        achieved = alg_launch / (stages[stage] / 1e3) / 1e9
        # traffic: HBM bytes per launch from the committed PMC passes, corrected
        # as the guide prescribes (FETCH_SIZE x 2 + WRITE_SIZE, gfx950).  The
        # guide's factor is calibrated for 16-B-per-lane coalesced streams; for
        # these kernels' per-lane 64-B chunk walk it may overstate, and a
        # stand-in calibration (tools/pmc_calib.hip) lands below the in-place
        # floor, so neither is exact: the physical bytes lie between the floor
        # (every payload byte read once, ciphertext + trailer written once) and
        # this figure: traffic_range.
        g = (pmc.get("guide_correction_bytes_per_launch") or {}).get(kernel)
        hdr = 12  # RTP header: read, never rewritten
        floor = n * (L + (L - hdr + T)) if kernel == "k_protect" else n * ((L + T) + (L - hdr))
        r = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
             "traffic": g, "avg_launch_ms": round(stages[stage], 4),
             "algorithmic_bytes_per_launch": alg_launch,
             "copy_measured_gbps": copy_gbs}
        if g:
            r["traffic_source"] = (f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE per {kernel} launch, "
                                   f"FETCH x 2 + WRITE (the guide's gfx950 correction), {pmc.get('source', '')}")
            r["traffic_over_algorithmic"] = round(g / alg_launch, 3)
            r["traffic_range"] = {"floor": floor, "guide_corrected": g,
                                  "pattern_calibrated": pmc.get(traffic_key),
                                  "note": "physical bytes lie in [floor, guide_corrected]; the pattern "
                                          "calibration (tools/pmc_calib.hip) is quoted, not trusted"}
        if util_key and pmc.get(util_key):
            r["utilisation"] = pmc.get(util_key)
        if pmc:
            r["counters_kernel_sha16"] = pmc.get("kernel_source_sha16")
            r["kernel_sha16"] = ksha
            r["traffic_stale"] = pmc_stale
            if pmc_stale:  # counters of another build: quoted, not this build's traffic
                r["traffic_of_other_build"] = r.pop("traffic")
                r["traffic"] = None
        return r

    r_prot = roofline("protect", "k_protect", "k_protect_bytes_per_launch", "k_protect_utilisation")
    r_unp = roofline("verify", "k_unprotect", "k_unprotect_bytes_per_launch", "k_unprotect_utilisation")
    cands = [r for r in (r_prot, r_unp) if r]
    dominant = max(cands, key=lambda r: r["avg_launch_ms"]) if cands else None
    other = [r for r in cands if r is not dominant]

    cpu = None
    if rank == 0 and n_gpus == 1 and not args.no_cpu:
        share = args.cpu_threads or max(1, min(16, len(os.sched_getaffinity(0))))
        cpu = cpu_baseline(args.cpu_seconds, share, L, args.ssrcs, T)

    # 3. The PCIe-inclusive legs (never `value`): every GPU's pinned pipeline at
    # once, and the dispatcher's host-bundle path.
    b0, keys0 = sd0.b, sd0.keys
    del sides, sd0
    torch.cuda.empty_cache()
    e2e = None
    if not args.no_e2e:
        legs = [E2E(b0, pols, keys0, n, d) for d in devices]
        for x in legs:
            x.warm()
        if world > 1:
            dist.barrier()
        if len(legs) == 1:
            res = [legs[0].run(args.e2e_bundles)]
        else:
            import threading
            res = [None] * len(legs)
            bar = threading.Barrier(len(legs))

            def e2e_body(i):
                torch.cuda.set_device(devices[i])
                bar.wait()
                res[i] = legs[i].run(args.e2e_bundles)
            th = [threading.Thread(target=e2e_body, args=(i,)) for i in range(len(legs))]
            for x in th:
                x.start()
            for x in th:
                x.join()
        e_dt = max(r[0] for r in res)
        e_pk = sum(r[1] for r in res)
        e_by = sum(r[2] for r in res)
        e_ok = all(r[3] for r in res)
        if world > 1:
            v = torch.tensor([e_dt, -float(e_ok)], dtype=torch.float64, device=devices[0])
            w = torch.tensor([e_pk, e_by], dtype=torch.float64, device=devices[0])
            if args.backend != "nccl":
                v, w = v.cpu(), w.cpu()
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            dist.all_reduce(w, op=dist.ReduceOp.SUM)
            e_dt, e_ok = float(v[0]), float(v[1]) < 0
            e_pk, e_by = float(w[0]), float(w[1])
        for x in legs:
            x.close()
        e2e = e2e_summary(e_dt, e_pk, e_by, e_ok, n_gpus, args.e2e_bundles, legs[0].depth)
    disp = disp_torch = None
    if rank == 0 and not args.no_dispatch and world == 1:
        counts, devs_for = dispatch_plan(args, devices)
        if child is None:
            disp = dispatch_leg(b0, pols, keys0, n, devs_for, counts, args.dispatch_bundles)
        else:
            # the leg in this process too, one shard: on torch's HIP runtime
            disp_torch = dispatch_leg(b0, pols, keys0, n, devs_for, [1], args.dispatch_bundles,
                                      modes=[(1, "pinned"), (1, "async")])
            disp_torch["note"] = ("this torch process: libsrtp_mi355x on torch's bundled HIP runtime "
                                  "(ROCm 7.0); 'dispatch' ran in a torch-free process on /opt/rocm's")
            disp = dispatch_child_result(child)
            if "error" not in disp:
                disp["process"] = "torch-free child (/opt/rocm HIP runtime, as a JVM or C host)"

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(pps, 1),
            "unit": "packets/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic RTP packets, random payload, seeded keys)",
            "config": {"workload": "configs[1]: 10k concurrent SSRCs x 1200-B RTP, "
                                   "AES_CM_128_HMAC_SHA1_80, protect + unprotect per step",
                       "packets_per_gpu_per_step": n, "ssrcs_per_gpu": args.ssrcs, "pkt_len": L,
                       "region_align": args.align,
                       "ssrc_mix": f"zipf({args.zipf})" if args.zipf > 0 else "round-robin",
                       "keysets": args.keysets,
                       "parallelism": f"ssrc-sharded x{n_gpus} ({'one process per GPU' if mode == 'process' else 'one process, all GPUs'})",
                       "streams": "serial: protect(i), unprotect(i) on one stream" if args.serial else
                                  {"free": "sender + receiver engine, one stream each: unprotect(i) "
                                           "after protect(i), the sender runs ahead",
                                   "join": "sender + receiver engine, one stream each: protect(i) "
                                           "beside unprotect(i-1), joined every step"}.get(
                                      args.pipe, f"sender + receiver engine, {args.pipe}"),
                       "stream_events": args.events},
            "gbps": round(gbs, 2),
            "goodput_gbps": round(pps * L * 2 / 1e9, 2),
            "all_accepted": ok,
            "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            "slow_path_per_bundle": slow_per_bundle,
            "host_enqueue_us_per_step": enqueue_us,
            "roofline": dominant,
            "roofline_other": other[0] if other else None,
            "cpu_baseline": cpu,
            "e2e": e2e,
            "dispatch": disp,
            "dispatch_in_torch_process": disp_torch,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
