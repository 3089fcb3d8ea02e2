"""CPU, world_size 2 (gloo): SSRC-sharded processing equals unsharded
processing, with the product's own split.

Each rank takes its shard of the same bundle from ``srtp_dispatch_plan`` (the
C++ plan the in-process dispatcher runs, ``libjitsi_amd/csrc/dispatch.cpp``)
and follows the dispatcher's abort-on-throw protocol with its own transformers
(the oracle stands in for the per-GPU engine): snapshot the contexts of the
transformers that could throw, run the whole shard, exchange each
transformer's first throw (all_gather), roll back that transformer's later
packets -- NOT_PROCESSED, original bytes -- and the contexts they touched,
and re-run its earlier packets on those contexts.  That makes
SinglePacketTransformer's abort-on-throw (SinglePacketTransformer.java
:134-155,190-210) hold across shards.  Rank 0 checks the merged statuses,
lengths and bytes against one oracle run of the whole bundle.  The bundle
mixes two transformers, so one transformer's throw must stop only its own
later packets."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from libjitsi_amd import dispatch, synth

NOT_PROCESSED, ERR_MALFORMED = 8, 6


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
    b = synth.rtp_bundle(900, 40, (60, 600), seed=synth.SEED_BASE + 5, seq0=seq0)
    tids = (np.arange(b.n) % 7 == 3).astype(np.int32)  # transformer 1 owns every 7th packet
    # Malformed packets (V=2, X=1, CC=15: the extension length is read from the
    # payload, so getHeaderLength usually runs past the packet and the cipher
    # throws): two of transformer 1's, late in the bundle, and none of 0's.
    o = b.off.astype(np.int64)
    for i in (703, 815):
        assert tids[i] == 1
        b.seg[o[i]] = 0x9F
    return b, tids


def _transformers(O, rank_seed=5):
    pol = O.Policy(1, 16, 1, 20, 10, 14)
    (k, s), = synth.keys(rank_seed, 1)
    out = []
    for _ in range(2):  # two independent streams' sender/receiver pairs
        fs, fr = O.Factory(True, k, s, pol, pol), O.Factory(False, k, s, pol, pol)
        out.append((O.Transformer(0, fs, fs), O.Transformer(0, fr, fr)))
    return out


def _process(O, ts, b, tids, idx, reverse, seg, ln, status):
    """Oracle on the packets idx (bundle order), results written back."""
    if len(idx) == 0:
        return
    sub = synth.select(b, idx)
    for j, i in enumerate(idx):  # current bytes / length of each packet
        sub.seg[sub.off[j]:sub.off[j] + sub.cap[j]] = seg[b.off[i]:b.off[i] + b.cap[i]]
    sl = ln[idx].copy()
    st = O.process([ts[int(tids[i])][1 if reverse else 0] for i in idx], reverse, sub.seg, sub.off,
                   sl, sub.cap)
    for j, i in enumerate(idx):
        seg[b.off[i]:b.off[i] + b.cap[i]] = sub.seg[sub.off[j]:sub.off[j] + sub.cap[j]]
    ln[idx] = sl
    status[idx] = st


def _sharded(O, b, tids, reverse, seg, ln, rank, world, ts):
    shard, may_throw, runs = dispatch.plan(world, seg, b.off, ln, b.cap, kinds=[0, 0], tids=tids,
                                           reverse=reverse)
    status = np.full(b.n, NOT_PROCESSED, np.int32)
    mine = np.nonzero(shard == rank)[0]
    risky = set(tids[may_throw == 1].tolist())
    valid = (ln >= 12) & (ln <= b.cap)

    def key(i):
        o = int(b.off[i])
        return int(tids[i]), int.from_bytes(seg[o + 8:o + 12].tobytes(), "big")

    def tr(t):
        return ts[t][1 if reverse else 0]

    snap, stash = {}, {}
    for i in mine:  # snapshot of the contexts that a rollback may reset
        if int(tids[i]) in risky:
            stash[i] = (seg[b.off[i]:b.off[i] + b.cap[i]].copy(), int(ln[i]))
            if valid[i] and key(i) not in snap:
                snap[key(i)] = tr(key(i)[0]).state(key(i)[1])
    _process(O, ts, b, tids, mine, reverse, seg, ln, status)
    first = {}
    for i in mine:
        if status[i] == ERR_MALFORMED and int(tids[i]) not in first:
            first[int(tids[i])] = int(i)
    allf = [None] * world
    dist.all_gather_object(allf, first)
    e_t = {}
    for f in allf:
        for t, i in f.items():
            e_t[t] = min(i, e_t.get(t, i))
    dirty = set()
    for i in mine:  # roll back the packets after their transformer's first throw
        e = e_t.get(int(tids[i]))
        if e is None or i <= e:
            continue
        if status[i] != NOT_PROCESSED and valid[i]:
            dirty.add(key(i))
        status[i] = NOT_PROCESSED
        seg[b.off[i]:b.off[i] + b.cap[i]], ln[i] = stash[i]
    for t, ssrc in dirty:  # contexts back to their state before the bundle
        if snap[(t, ssrc)] is None:
            tr(t).remove_context(ssrc)
        else:
            tr(t).import_context(ssrc, snap[(t, ssrc)], forward=not reverse)
    rerun = [i for i in mine if int(tids[i]) in e_t and i <= e_t[int(tids[i])] and valid[i]
             and key(i) in dirty]
    for i in rerun:
        seg[b.off[i]:b.off[i] + b.cap[i]], ln[i] = stash[i]
    _process(O, ts, b, tids, np.array(rerun, np.int64), reverse, seg, ln, status)
    return status, shard, runs


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    b, tids = _bundle()
    ts = _transformers(O)
    seg, ln = b.seg.copy(), b.length.copy()
    st1, shard, runs1 = _sharded(O, b, tids, False, seg, ln, rank, world, ts)
    hit = ((b.ssrc.astype(np.int64) + b.seq) % 13) == 0  # tamper a little on the wire
    seg[b.off[hit].astype(np.int64) + 30] ^= 1
    st2, _, _ = _sharded(O, b, tids, True, seg, ln, rank, world, ts)
    mine = np.nonzero(shard == rank)[0]
    got = [None] * world if rank == 0 else None
    dist.gather_object((mine, st1[mine], st2[mine], ln[mine],
                        [seg[b.off[i]:b.off[i] + ln[i]].tobytes() for i in mine]), got, dst=0)
    if rank == 0:
        # one process, whole bundle, per-packet transformers
        tr = _transformers(O)
        sg, l2 = b.seg.copy(), b.length.copy()
        r1 = O.process([tr[t][0] for t in tids], False, sg, b.off, l2, b.cap)
        sg[b.off[hit].astype(np.int64) + 30] ^= 1
        r2 = O.process([tr[t][1] for t in tids], True, sg, b.off, l2, b.cap)
        idx = [g[0] for g in got]
        m1 = dispatch.merge([g[1] for g in got], idx, b.n)
        m2 = dispatch.merge([g[2] for g in got], idx, b.n)
        ml = dispatch.merge([g[3] for g in got], idx, b.n)
        pk = [None] * b.n
        for g in got:
            for j, i in enumerate(g[0]):
                pk[i] = g[4][j]
        ref_pk = [sg[b.off[i]:b.off[i] + l2[i]].tobytes() for i in range(b.n)]
        ok = (np.array_equal(m1, r1) and np.array_equal(m2, r2) and np.array_equal(ml, l2)
              and pk == ref_pk and all(len(i) > 0 for i in idx)
              and (r1 == ERR_MALFORMED).sum() == 1 and (r1 == NOT_PROCESSED).sum() > 0
              and runs1 == 2)
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


def test_plan_is_stable_partition():
    b, tids = _bundle()
    shard, phase, nph = dispatch.plan(3, b.seg, b.off, b.length, b.cap, kinds=[0, 0], tids=tids)
    parts = dispatch.split(shard, 3)
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, np.arange(b.n))
    for p in parts:
        assert np.all(np.diff(p) > 0)
    for s in np.unique(b.ssrc):  # every SSRC lives on exactly one shard
        sh = set(shard[b.ssrc == s].tolist())
        assert sh == {dispatch.shard_of_ssrc(int(s), 3)}
    # the two malformed packets of transformer 1 are the ones that could throw
    assert nph == 2
    assert phase[703] == 1 and phase[815] == 1 and phase.sum() == 2
    # without abort-on-error nothing needs a snapshot
    _, ph0, n0 = dispatch.plan(3, b.seg, b.off, b.length, b.cap, kinds=[0, 0], tids=tids,
                               abort_on_error=False)
    assert n0 == 1 and (ph0 == 0).all()


def test_plan_skip_and_invalid():
    b, _ = _bundle()
    fl = np.zeros(b.n, np.uint32)
    fl[5] = 0x80000000
    ln = b.length.copy()
    ln[6] = 8  # RawPacket.isInvalid: handled by shard 0's engine (DROP_INVALID)
    tids = np.zeros(b.n, np.int32)
    tids[7] = 5  # no such transformer: skipped without an engine
    shard, phase, _ = dispatch.plan(4, b.seg, b.off, ln, b.cap, kinds=[0], tids=tids, flags=fl)
    assert shard[5] == -1 and shard[7] == -1 and shard[6] == 0
