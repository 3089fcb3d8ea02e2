"""GPU: context-state export / import.

A receiver's SRTP and SRTCP contexts are exported from one engine and imported
into a second engine (another GPU in a re-sharded deployment); the second
engine then continues the streams exactly as the first one does -- same
statuses, lengths, plaintext and final state -- including rejecting replays of
packets only the first engine ever saw.
"""
import numpy as np
import pytest

from libjitsi_amd import SRTCPTransformer, SRTPContextFactory, SRTPTransformer, profile_policies, synth

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")


def run(eng, t, reverse, b, seg=None, ln=None):
    seg = (b.seg if seg is None else seg).copy()
    ln = (b.length if ln is None else ln).copy()
    st = eng.transform_host(reverse, t.tid, seg, b.off, ln, b.cap)
    return seg, ln, st


def test_export_import_continues_streams(engine_factory):
    A = engine_factory(max_contexts=4096, max_factories=64, max_transformers=64)
    B = engine_factory(max_contexts=4096, max_factories=64, max_transformers=64)
    (k, s), = synth.keys(61, 1)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *P80, engine=A))
    rcv_a = SRTPTransformer(SRTPContextFactory(False, k, s, *P80, engine=A))
    csnd = SRTCPTransformer(SRTPContextFactory(True, k, s, *P80, engine=A))
    crcv_a = SRTCPTransformer(SRTPContextFactory(False, k, s, *P80, engine=A))
    seq0 = np.array([65500, 100, 40000, 7], np.uint32)
    full = synth.rtp_bundle(400, 4, (60, 1200), seed=62, seq0=seq0)
    rtcp = synth.rtcp_bundle(60, 4, seed=63, ssrcs=full.meta["ssrcs"])
    parts = [synth.select(full, np.arange(i, i + 100)) for i in range(0, 400, 100)]
    cparts = [synth.select(rtcp, np.arange(i, i + 20)) for i in range(0, 60, 20)]
    prot = []
    for part in parts[:2]:  # history only engine A sees
        seg, ln, st = run(A, snd, False, part)
        assert (st == 0).all()
        prot.append((seg, ln))
        _, _, st = run(A, rcv_a, True, part, seg, ln)
        assert (st == 0).all()
    cprot = []
    for part in cparts[:2]:
        seg, ln, st = run(A, csnd, False, part)
        cprot.append((seg, ln))
        _, _, st = run(A, crcv_a, True, part, seg, ln)
        assert (st == 0).all()

    ex = A.export_contexts(rcv_a)
    cex = A.export_contexts(crcv_a)
    assert sorted(ex) == sorted(int(x) for x in full.meta["ssrcs"])
    assert len(cex) == 4
    rcv_b = SRTPTransformer(SRTPContextFactory(False, k, s, *P80, engine=B))
    crcv_b = SRTCPTransformer(SRTPContextFactory(False, k, s, *P80, engine=B))
    for ssrc, stt in ex.items():
        B.import_context(rcv_b, ssrc, stt, forward=False)
    for ssrc, stt in cex.items():
        B.import_context(crcv_b, ssrc, stt, forward=False)
    for ssrc, stt in ex.items():
        got = B.context_state(rcv_b, ssrc)
        for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
            assert got[key] == stt[key]

    # new traffic plus replays of what only A has seen: A and B must agree
    new_seg, new_ln, st = run(A, snd, False, parts[2])
    assert (st == 0).all()
    replay = synth.select(parts[1], np.arange(0, 100, 7))
    rseg = np.zeros_like(replay.seg)
    for j, i in enumerate(range(0, 100, 7)):  # protected bytes of those packets
        o, L = int(parts[1].off[i]), int(prot[1][1][i])
        rseg[replay.off[j]:replay.off[j] + L] = prot[1][0][o:o + L]
    rlen = prot[1][1][np.arange(0, 100, 7)].astype(np.uint32)
    for part, seg, ln in ((parts[2], new_seg, new_ln), (replay, rseg, rlen)):
        sa, la, sta = run(A, rcv_a, True, part, seg, ln)
        sb, lb, stb = run(B, rcv_b, True, part, seg, ln)
        assert (sta == stb).all() and (la == lb).all() and np.array_equal(sa, sb)
    assert (stb == 1).all()  # the replays: DROP_REPLAY on the importing engine too
    cseg, cln, st = run(A, csnd, False, cparts[2])
    sa, la, sta = run(A, crcv_a, True, cparts[2], cseg, cln)
    sb, lb, stb = run(B, crcv_b, True, cparts[2], cseg, cln)
    assert (sta == 0).all() and (sta == stb).all() and np.array_equal(sa, sb)
    for ssrc in ex:
        a, b = A.context_state(rcv_a, ssrc), B.context_state(rcv_b, ssrc)
        for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
            assert a[key] == b[key]
    for ssrc in cex:
        a, b = A.context_state(crcv_a, ssrc), B.context_state(crcv_b, ssrc)
        for key in ("received_index", "replay_window"):
            assert a[key] == b[key]


def test_import_needs_open_factory(engine_factory):
    E = engine_factory(max_contexts=1024, max_factories=16, max_transformers=16)
    (k, s), = synth.keys(64, 1)
    f = SRTPContextFactory(False, k, s, *P80, engine=E)
    t = SRTPTransformer(f)
    f.close()
    with pytest.raises(Exception):
        E.import_context(t, 1234, {"roc": 1, "s_l": 5, "seq_num_set": 1}, forward=False)
