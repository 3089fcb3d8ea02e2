"""GPU: the in-process multi-GPU dispatcher (srtp_dispatch_*).

One process drives G engines -- one per GPU in production, G engines on
device 0 here when the box has one GPU -- and every bundle is split by SSRC
across them.  Each scenario runs through the dispatcher and through the oracle
on identical bytes and must agree on every status, length, segment byte and
context state (tests/harness.py), exactly as a single engine does: the
dispatcher must be invisible.  Also: calls from a non-main host thread, the
cross-shard abort-on-throw phases, stats summed over shards, and (with >= 2
GPUs) engines on devices 0 and 1 driven from a thread whose current device is
another one.
"""
import threading

import numpy as np
import pytest

from libjitsi_amd import SRTPDispatcher, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

import test_gpu_parity as G
from harness import Twin

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


def _gpus():
    import torch
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


@pytest.fixture(params=[2, 4], ids=["G2", "G4"])
def dtwin(request, oracle):
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    d = SRTPDispatcher([0] * request.param, max_contexts=1 << 15, max_factories=256,
                       max_transformers=1024)
    yield Twin(d)
    d.close()


def test_dispatch_round_trips_and_configs(dtwin):
    """C1 (one SSRC, seq wrap), C2 (1200 B), C3 (faults), C4 (SRTP+SRTCP,
    three profiles, SDES and DTLS rekeys) through the dispatcher."""
    G.test_config1_single_ssrc_160B_with_wrap(dtwin)
    G.test_config2_video_1200B(dtwin)
    G.test_config3_mixed_sizes_unprotect_with_faults(dtwin)
    G.test_config4_srtp_srtcp_mixed_rekey(dtwin)
    G.test_discard_silence_flags_skip_decrypt(dtwin)
    G.test_roc_guess_overturned_by_walk(dtwin)
    G.test_many_transformers_one_bundle(dtwin)
    G.test_factory_close_no_new_contexts(dtwin)
    G.test_capacity_and_skip(dtwin)


def test_dispatch_every_ssrc_lands_on_its_shard(dtwin):
    d = dtwin.engine
    (k, s), = synth.keys(71, 1)
    f = dtwin.factory(True, k, s, *P80)
    t = dtwin.transformer(O.KIND_RTP, f)
    b = synth.rtp_bundle(4000, 300, (60, 800), seed=72)
    dtwin.run(t, False, b.seg, b.off, b.length, b.cap)
    counts = [N.lib().srtp_engine_num_contexts(N.lib().srtp_dispatch_engine(d.h, i))
              for i in range(d.shards)]
    want = np.bincount([d.shard_of(int(x)) for x in b.meta["ssrcs"]], minlength=d.shards)
    assert counts == want.tolist() and min(counts) > 0
    st = d.stats()
    assert st["status"]["OK"] == b.n and st["ctx_live"] == 300


@pytest.mark.parametrize("abort", [True, False])
def test_dispatch_malformed_abort_across_shards(oracle, abort):
    """A throw on one shard aborts the same transformer's later packets on the
    other shards (SinglePacketTransformer.java:134-155); other transformers
    carry on.  Two transformers interleaved, malformed packets in both."""
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    d = SRTPDispatcher([0, 0, 0], abort_on_error=abort, max_contexts=4096, max_factories=64,
                       max_transformers=64)
    try:
        twin = Twin(d)
        (k, s), = synth.keys(12, 1)
        f, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        ts = [twin.transformer(O.KIND_RTP, f), twin.transformer(O.KIND_RTP, f)]
        rs = [twin.transformer(O.KIND_RTP, fr), twin.transformer(O.KIND_RTP, fr)]
        b = synth.rtp_bundle(600, 31, (40, 700), seed=73)
        who = (np.arange(b.n) % 3 == 1).astype(int)
        o = b.off.astype(np.int64)
        for i in (100, 250, 430):  # CC=15 with X: the header length runs past the packet
            b.seg[o[i]] = 0x9F
        b.seg[o[31]] = 0x8F  # CC=15 without X on a 40-B packet: negative payload length
        b.length[31] = 40
        seg, ln, st = twin.run([ts[w] for w in who], False, b.seg, b.off, b.length, b.cap,
                               abort_on_error=abort)
        assert (st == N.STATUS_ERR_MALFORMED).any()
        if abort:
            assert (st == N.STATUS_NOT_PROCESSED).any()
        twin.run([rs[w] for w in who], True, seg, b.off, ln, b.cap, abort_on_error=abort)
        # SRTCP: index offset < 0 throws before auth
        tc = twin.transformer(O.KIND_RTCP, fr)
        cb = synth.rtcp_bundle(40, 6, len_range=(12, 40), seed=74)
        twin.run(tc, True, cb.seg, cb.off, cb.length, cb.cap, abort_on_error=abort)
    finally:
        d.close()


def test_dispatch_from_a_worker_thread(dtwin):
    """The engines are driven from a host thread that is not the one that
    created them (a JVM send or receive thread)."""
    (k, s), = synth.keys(75, 1)
    fs, fr = dtwin.factory(True, k, s, *P80), dtwin.factory(False, k, s, *P80)
    snd, rcv = dtwin.transformer(O.KIND_RTP, fs), dtwin.transformer(O.KIND_RTP, fr)
    b = synth.rtp_bundle(5000, 200, (60, 1400), seed=76)
    err = []

    def body():
        try:
            seg, ln, st = dtwin.run(snd, False, b.seg, b.off, b.length, b.cap)
            dtwin.run(rcv, True, seg, b.off, ln, b.cap)
        except BaseException as e:  # noqa: BLE001 -- re-raised in the main thread
            err.append(e)

    th = threading.Thread(target=body)
    th.start()
    th.join(120)
    assert not th.is_alive()
    if err:
        raise err[0]


def test_dispatch_two_gpus_other_current_device(oracle):
    """Engines on devices 0 and 1, driven from a thread whose current device
    is the last GPU: every allocation and launch must still land on the
    engine's own device (the C ABI's device guard)."""
    n = _gpus()
    if n < 2:
        pytest.skip("needs two GPUs")
    import torch
    d = SRTPDispatcher([0, 1], max_contexts=4096, max_factories=64, max_transformers=64)
    try:
        twin = Twin(d)
        (k, s), = synth.keys(77, 1)
        fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        b = synth.rtp_bundle(3000, 100, (60, 1400), seed=78)
        err = []

        def body():
            try:
                torch.cuda.set_device(n - 1)
                seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
                twin.run(rcv, True, seg, b.off, ln, b.cap)
                assert torch.cuda.current_device() == n - 1
            except BaseException as e:  # noqa: BLE001
                err.append(e)

        th = threading.Thread(target=body)
        th.start()
        th.join(120)
        if err:
            raise err[0]
    finally:
        d.close()


def test_dispatch_many_throws_bounded_runs(oracle):
    """200 packets that throw (or could: malformed headers, short SRTCP)
    spread over 50 transformers interleaved on 4 shards, with abort-on-throw:
    every bundle agrees with the oracle bit for bit, and the dispatcher runs
    each shard at most twice per bundle (the whole bundle, then the rollback
    re-run of the throwing transformers' earlier packets) -- the engines'
    bundle counters bound the GPU round trips, however many packets throw
    (SinglePacketTransformer.java:134-155,190-210)."""
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    shards = 4
    d = SRTPDispatcher([0] * shards, max_contexts=1 << 14, max_factories=256, max_transformers=256)
    try:
        twin = Twin(d)
        rng = np.random.default_rng(91)
        (k, s), = synth.keys(90, 1)
        f, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        nt = 50
        ts = [twin.transformer(O.KIND_RTP, f) for _ in range(nt)]
        rs = [twin.transformer(O.KIND_RTP, fr) for _ in range(nt)]
        b = synth.rtp_bundle(6000, 400, (40, 900), seed=92)
        who = rng.integers(0, nt, b.n)
        # SSRC i % 400 belongs to transformer who[...]: keep each SSRC on one transformer
        who = who[np.arange(b.n) % 400]
        o = b.off.astype(np.int64)
        bad = rng.choice(np.arange(200, b.n), 200, replace=False)
        for j, i in enumerate(bad):
            if j % 2:
                b.seg[o[i]] = 0x9F  # CC=15 with X: the header length runs past the packet
            else:
                b.seg[o[i]] = 0x8F  # CC=15: negative payload length on a short packet
                b.length[i] = 40
        n0 = d.stats()["bundles"]
        seg, ln, st = twin.run([ts[w] for w in who], False, b.seg, b.off, b.length, b.cap)
        n1 = d.stats()["bundles"]
        assert (st == N.STATUS_ERR_MALFORMED).sum() >= 20 and (st == N.STATUS_NOT_PROCESSED).any()
        assert n1 - n0 <= 2 * shards, (n1 - n0)
        # receive side: the wire copy with the throws' transformers' traffic
        twin.run([rs[w] for w in who], True, seg, b.off, ln, b.cap)
        assert d.stats()["bundles"] - n1 <= 2 * shards
        # SRTCP: short packets throw at the index offset before auth (50 transformers)
        cts = [twin.transformer(O.KIND_RTCP, fr) for _ in range(nt)]
        cb = synth.rtcp_bundle(3000, 200, len_range=(12, 60), seed=93)
        cw = rng.integers(0, nt, cb.n)
        n2 = d.stats()["bundles"]
        twin.run([cts[w] for w in cw], True, cb.seg, cb.off, cb.length, cb.cap)
        assert d.stats()["bundles"] - n2 <= 2 * shards
    finally:
        d.close()


class _Registered:
    """The dispatcher with each call's segment registered (srtp_host_register),
    as a caller's long-lived buffer pool would be: a shard's chunk whose packets
    lie back to back is moved by DMA in place, with no host copy."""

    def __init__(self, d):
        self._d = d

    def __getattr__(self, k):
        return getattr(self._d, k)

    def transform_host(self, reverse, tid, seg, *a, **kw):
        from libjitsi_amd import host_is_registered, host_register, host_unregister
        host_register(seg)
        try:
            assert host_is_registered(seg)
            return self._d.transform_host(reverse, tid, seg, *a, **kw)
        finally:
            host_unregister(seg)


@pytest.mark.parametrize("shards", [1, 3])
def test_dispatch_registered_segment_in_place(oracle, shards):
    """Registered segments through 1 shard (every chunk one run: no host copy
    at all) and 3 shards (runs broken by the SSRC split: the copy path), bit
    for bit against the oracle: several chunks per shard, faults, and
    malformed packets whose rollback restores the registered bytes."""
    if _gpus() < 1:
        pytest.skip("no GPU visible")
    d = SRTPDispatcher([0] * shards, max_contexts=1 << 15, max_factories=64, max_transformers=64)
    try:
        twin = Twin(_Registered(d))
        (k, s), = synth.keys(81, 1)
        fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        b = synth.rtp_bundle(70000, 500, (60, 400), seed=82)  # > 2 chunks of 2^15 packets
        seg, ln, st = twin.run(snd, False, b.seg, b.off, b.length, b.cap)
        assert (st == N.STATUS_OK).all()
        seg = seg.copy()
        o = b.off.astype(np.int64)
        seg[o[1000] + 20] ^= 1      # forged
        seg[o[40000] + 30] ^= 0x80  # forged, in a later chunk
        twin.run(rcv, True, seg, b.off, ln, b.cap)
        # throws: a throw aborts its transformer's packets in later chunks too
        # (2^15-packet chunks), and the rollback restores stashed bytes into
        # the registered segment
        b2 = synth.rtp_bundle(40000, 40, (40, 300), seed=83)
        o2 = b2.off.astype(np.int64)
        for i in (200, 20000):
            b2.seg[o2[i]] = 0x9F
        _, _, st2 = twin.run(snd, False, b2.seg, b2.off, b2.length, b2.cap)
        assert (st2 == N.STATUS_ERR_MALFORMED).any() and (st2 == N.STATUS_NOT_PROCESSED).any()
    finally:
        d.close()
