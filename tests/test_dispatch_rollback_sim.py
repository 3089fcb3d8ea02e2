"""CPU: the dispatcher's abort-on-throw rollback (libjitsi_amd/csrc/dispatch.cpp)
replayed with the oracle standing in for each shard's engine, at the scale of
the GPU test test_dispatcher.py::test_dispatch_many_throws_bounded_runs: 50
transformers interleaved over 4 shards, 200 malformed packets, protect then
unprotect (RTP) and short-SRTCP unprotect.  Each shard is its own set of
oracle transformers (its own contexts, as one engine per GPU); the protocol
is the product's: the shard split and may-throw marks from srtp_dispatch_plan,
a context snapshot of the transformers that could throw, one run of every
shard, each transformer's first throw over all shards, rollback of its later
packets (NOT_PROCESSED, original bytes and length) and of the contexts they
touched, and a re-run of its earlier packets on those contexts.  The merged
result must equal one oracle run of the whole bundle
(SinglePacketTransformer.java:134-155,190-210)."""
import numpy as np

from libjitsi_amd import dispatch, synth

NOT_PROCESSED, ERR_MALFORMED = 8, 6
SHARDS, NT = 4, 50


def _transformers(O, kind, sender, k, s, n):
    pol = O.Policy(1, 16, 1, 20, 10, 14)
    f = O.Factory(sender, k, s, pol, pol)
    return [O.Transformer(kind, f, f) for _ in range(n)]


def _run(O, ts, b, tids, idx, reverse, seg, ln, status):
    if len(idx) == 0:
        return
    sub = synth.select(b, idx)
    for j, i in enumerate(idx):
        sub.seg[sub.off[j]:sub.off[j] + sub.cap[j]] = seg[b.off[i]:b.off[i] + b.cap[i]]
    sl = ln[idx].copy()
    st = O.process([ts[int(tids[i])] for i in idx], reverse, sub.seg, sub.off, sl, sub.cap)
    for j, i in enumerate(idx):
        seg[b.off[i]:b.off[i] + b.cap[i]] = sub.seg[sub.off[j]:sub.off[j] + sub.cap[j]]
    ln[idx] = sl
    status[idx] = st


def sharded(O, shard_ts, kind, b, tids, reverse, seg, ln):
    """The dispatcher's protocol over SHARDS oracle 'engines' (shard_ts[s][t])."""
    shard, may_throw, runs = dispatch.plan(SHARDS, seg, b.off, ln, b.cap, kinds=[kind] * NT,
                                           tids=tids, reverse=reverse)
    status = np.zeros(b.n, np.int32)
    valid0 = (ln >= 12) & (ln <= b.cap)
    so = 8 if kind == 0 else 4

    def key(i):
        o = int(b.off[i])
        return int(tids[i]), int.from_bytes(seg[o + so:o + so + 4].tobytes(), "big")

    per = [np.nonzero(shard == s)[0] for s in range(SHARDS)]
    risky = set(tids[may_throw == 1].tolist()) if runs == 2 else set()
    snap, stash = [{} for _ in range(SHARDS)], {}
    for s in range(SHARDS):
        for i in per[s]:
            if int(tids[i]) in risky:
                stash[i] = (seg[b.off[i]:b.off[i] + b.cap[i]].copy(), int(ln[i]))
                if valid0[i] and key(i) not in snap[s]:
                    t, x = key(i)
                    snap[s][(t, x)] = shard_ts[s][t].state(x)
    for s in range(SHARDS):
        _run(O, shard_ts[s], b, tids, per[s], reverse, seg, ln, status)
    e_t = {}
    for i in range(b.n):
        if shard[i] >= 0 and status[i] == ERR_MALFORMED and int(tids[i]) not in e_t:
            e_t[int(tids[i])] = i
    dirty = [set() for _ in range(SHARDS)]
    for i in range(b.n):
        e = e_t.get(int(tids[i]))
        if shard[i] < 0 or e is None or i <= e:
            continue
        if status[i] != NOT_PROCESSED and valid0[i]:
            dirty[shard[i]].add(key(i))
        status[i] = NOT_PROCESSED
        seg[b.off[i]:b.off[i] + b.cap[i]], ln[i] = stash[i]
    n_rerun = 0
    for s in range(SHARDS):
        for t, x in dirty[s]:
            st = snap[s][(t, x)]
            if st is None:
                shard_ts[s][t].remove_context(x)
            else:
                shard_ts[s][t].import_context(x, st, forward=not reverse)
        rr = [i for i in per[s] if int(tids[i]) in e_t and i <= e_t[int(tids[i])] and valid0[i]
              and key(i) in dirty[s]]
        for i in rr:
            seg[b.off[i]:b.off[i] + b.cap[i]], ln[i] = stash[i]
        _run(O, shard_ts[s], b, tids, np.array(rr, np.int64), reverse, seg, ln, status)
        n_rerun += len(rr) > 0
    return status, n_rerun


def _check(O, kind, b, tids, k, s, sender_first=True):
    """Protect (sender) then unprotect (receiver) of b for RTP, or unprotect
    only for SRTCP; sharded vs one oracle."""
    one_s = _transformers(O, kind, True, k, s, NT)
    one_r = _transformers(O, kind, False, k, s, NT)
    sh_s = [_transformers(O, kind, True, k, s, NT) for _ in range(SHARDS)]
    sh_r = [_transformers(O, kind, False, k, s, NT) for _ in range(SHARDS)]
    seg1, ln1 = b.seg.copy(), b.length.copy()
    seg2, ln2 = b.seg.copy(), b.length.copy()
    reruns = 0
    if sender_first:
        st1 = O.process([one_s[t] for t in tids], False, seg1, b.off, ln1, b.cap)
        st2, r = sharded(O, sh_s, kind, b, tids, False, seg2, ln2)
        reruns += r
        assert np.array_equal(st1, st2) and np.array_equal(ln1, ln2) and np.array_equal(seg1, seg2)
        assert (st1 == ERR_MALFORMED).sum() >= 20 and (st1 == NOT_PROCESSED).any()
    st1 = O.process([one_r[t] for t in tids], True, seg1, b.off, ln1, b.cap)
    st2, r = sharded(O, sh_r, kind, b, tids, True, seg2, ln2)
    reruns += r
    bad = np.nonzero(st1 != st2)[0]
    assert len(bad) == 0, (bad[:10], st1[bad[:10]], st2[bad[:10]])
    assert np.array_equal(ln1, ln2) and np.array_equal(seg1, seg2)
    for s in range(SHARDS):  # every context agrees
        for t in range(NT):
            for x in set(int(v) for v in b.ssrc):
                assert one_r[t].state(x) == sh_r[s][t].state(x) or sh_r[s][t].state(x) is None
    return reruns


def test_rollback_protocol_many_throws_rtp(oracle):
    rng = np.random.default_rng(91)
    (k, s), = synth.keys(90, 1)
    b = synth.rtp_bundle(6000, 400, (40, 900), seed=92)
    who = rng.integers(0, NT, b.n)[np.arange(b.n) % 400]
    o = b.off.astype(np.int64)
    for j, i in enumerate(rng.choice(np.arange(200, b.n), 200, replace=False)):
        if j % 2:
            b.seg[o[i]] = 0x9F
        else:
            b.seg[o[i]] = 0x8F
            b.length[i] = 40
    assert _check(oracle, 0, b, who.astype(np.int32), k, s) > 0  # some shard re-ran


def test_rollback_protocol_short_srtcp(oracle):
    rng = np.random.default_rng(93)
    (k, s), = synth.keys(94, 1)
    cb = synth.rtcp_bundle(3000, 200, len_range=(12, 60), seed=93)
    cw = rng.integers(0, NT, cb.n).astype(np.int32)
    _check(oracle, 1, cb, cw, k, s, sender_first=False)
