"""CPU, world_size 2 (gloo): SSRC-sharded processing equals unsharded
processing.  Each rank takes its SSRC shard of the same bundle (stable order),
protects and unprotects it with its own transformers (the oracle stands in for
the per-GPU engine here), and rank 0 checks the merged statuses, lengths and
bytes against a single-process run of the whole bundle."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from libjitsi_amd import dispatch, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bundle():
    rng = np.random.default_rng(9)
    seq0 = rng.integers(0, 65536, 40).astype(np.uint32)
    seq0[:4] = 65530
    return synth.rtp_bundle(900, 40, (60, 600), seed=synth.SEED_BASE + 5, seq0=seq0)


def _run(O, b, idx=None):
    sub = b if idx is None else synth.select(b, idx)
    pol = O.Policy(1, 16, 1, 20, 10, 14)
    (k, s), = synth.keys(5, 1)
    fs, fr = O.Factory(True, k, s, pol, pol), O.Factory(False, k, s, pol, pol)
    ts, tr = O.Transformer(0, fs, fs), O.Transformer(0, fr, fr)
    seg, ln = sub.seg.copy(), sub.length.copy()
    st1 = O.process(ts, False, seg, sub.off, ln, sub.cap)
    # tamper and replay a little on the wire
    o = sub.off.astype(np.int64)
    hit = ((sub.ssrc.astype(np.int64) + sub.seq) % 13) == 0  # by packet identity, not position
    seg[o[hit] + 30] ^= 1
    st2 = O.process(tr, True, seg, sub.off, ln, sub.cap)
    pk = [seg[sub.off[i]:sub.off[i] + ln[i]].tobytes() for i in range(sub.n)]
    return st1, st2, ln, pk


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    b = _bundle()
    parts = dispatch.split(dispatch.packet_ssrc(b.seg, b.off), world)
    mine = _run(O, b, parts[rank])
    got = [None] * world if rank == 0 else None
    dist.gather_object((parts[rank], mine), got, dst=0)
    if rank == 0:
        ref = _run(O, b)
        n = b.n
        st1 = dispatch.merge([g[1][0] for g in got], [g[0] for g in got], n)
        st2 = dispatch.merge([g[1][1] for g in got], [g[0] for g in got], n)
        ln = dispatch.merge([g[1][2] for g in got], [g[0] for g in got], n)
        pk = [None] * n
        for idx, res in got:
            for j, i in enumerate(idx):
                pk[i] = res[3][j]
        ok = (np.array_equal(st1, ref[0]) and np.array_equal(st2, ref[1])
              and np.array_equal(ln, ref[2]) and pk == ref[3]
              and all(len(g[0]) > 0 for g in got))
        q.put(bool(ok))
    dist.destroy_process_group()


def test_ssrc_sharding_world2(oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


def test_split_is_stable_partition():
    b = _bundle()
    ssrc = dispatch.packet_ssrc(b.seg, b.off)
    parts = dispatch.split(ssrc, 3)
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(b.n))
    for p in parts:
        assert np.all(np.diff(p) > 0)
    for s in np.unique(ssrc):  # every SSRC lives on exactly one shard
        assert len({int(dispatch.shard_of(np.array([s]), 3)[0])}) == 1
