"""GPU: BASELINE configs[4] at its stream count through the sharded path.

10^6 SRTP streams split by SSRC over 8 shards of the in-process dispatcher
(srtp_dispatch_*, one engine per shard: one per GPU on an 8-GPU node, all
eight on device 0 on a one-GPU box).  Contexts are per (transformer, SSRC)
(SRTPTransformer.java:62,152-175), so every shard owns an eighth of them.

Sustained traffic in bundles of 2^18 packets: protect (1200-B packets, 5 %
of the streams starting just below the sequence wrap, so their second packet
wraps the ROC), then the C3 fault mix on the wire (1 % tamper, 1 % exact
replays, 0.5 % stale, 5 % reordered within 16), then unprotect.  Every bundle
is compared with the oracle bit for bit -- every status, length and segment
byte (tests/harness.py) -- and the context state of 1000 sampled streams per
shard is compared at the end.
"""
import numpy as np
import pytest

from libjitsi_amd import SRTPDispatcher, profile_policies, synth
from libjitsi_amd import _native as N
from oracle import oracle as O

from harness import Twin
from test_gpu_parity import inject_faults

pytestmark = pytest.mark.gpu
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
N_SSRC = 1_000_000
SHARDS = 8
BUNDLE = 1 << 18


def test_config5_1m_streams_8_shards(oracle):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    ngpu = torch.cuda.device_count()
    d = SRTPDispatcher([s % ngpu for s in range(SHARDS)], max_contexts=1 << 18, max_factories=16,
                       max_transformers=16, max_batch=1 << 16)
    try:
        twin = Twin(d)
        rng = np.random.default_rng(synth.SEED_BASE + 5)
        seq0 = rng.integers(0, 65536, N_SSRC).astype(np.uint32)
        near = rng.random(N_SSRC) < 0.05
        seq0[near] = 65535  # the stream's second packet wraps the ROC
        n_pkt = 6 * BUNDLE  # every stream once, 57 % of them twice
        b = synth.rtp_bundle(n_pkt, N_SSRC, 1200, seed=synth.SEED_BASE + 5, seq0=seq0)
        (k, s), = synth.keys(5, 1)
        fs, fr = twin.factory(True, k, s, *P80), twin.factory(False, k, s, *P80)
        snd, rcv = twin.transformer(O.KIND_RTP, fs), twin.transformer(O.KIND_RTP, fr)
        ssrcs = b.meta["ssrcs"]
        parts = []
        for j in range(n_pkt // BUNDLE):
            sub = synth.select(b, np.arange(j * BUNDLE, (j + 1) * BUNDLE))
            seg, ln, st = twin.run(snd, False, sub.seg, sub.off, sub.length, sub.cap,
                                   check_state=False)
            assert (st == 0).all()
            sub.seg, sub.length = seg, ln
            parts.append(sub)
        del b
        fb = inject_faults(synth.concat(parts), rng)
        del parts
        n_ok = n_replay = n_auth = 0
        for lo in range(0, fb.n, BUNDLE):
            sub = synth.select(fb, np.arange(lo, min(fb.n, lo + BUNDLE)))
            _, _, st = twin.run(rcv, True, sub.seg, sub.off, sub.length, sub.cap, check_state=False)
            n_ok += int((st == N.STATUS_OK).sum())
            n_replay += int((st == N.STATUS_DROP_REPLAY).sum())
            n_auth += int((st == N.STATUS_DROP_AUTH).sum())
        assert n_ok > 0.97 * n_pkt and n_replay > 0.005 * n_pkt and n_auth > 0.005 * n_pkt
        # every shard holds its share of the contexts, and a sample agrees with the oracle
        counts = [N.lib().srtp_engine_num_contexts(N.lib().srtp_dispatch_engine(d.h, i))
                  for i in range(SHARDS)]
        # sender + receiver transformer per stream, plus the receiver's contexts
        # of SSRCs a header tamper made up (created before the auth check, as
        # SRTPTransformer.java:152-175 does): the oracle holds the same set
        assert sum(counts) == snd.o.num_contexts() + rcv.o.num_contexts()
        assert snd.o.num_contexts() == N_SSRC and rcv.o.num_contexts() >= N_SSRC
        assert min(counts) > 0.9 * 2 * N_SSRC / SHARDS
        by_shard = {}
        for x in ssrcs[:200000]:
            by_shard.setdefault(d.shard_of(int(x)), []).append(int(x))
        for sh, xs in by_shard.items():
            for ssrc in rng.choice(xs, min(len(xs), 1000), replace=False):
                for t in (snd, rcv):
                    so, se = t.o.state(int(ssrc)), d.context_state(t.e, int(ssrc))
                    assert (so is None) == (se is None), (sh, ssrc)
                    if so is not None:
                        for key in ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window"):
                            assert int(so[key]) == int(se[key]), (sh, ssrc, key)
        wrapped = [x for x in ssrcs[near][:2000] if d.context_state(rcv.e, int(x)) and
                   d.context_state(rcv.e, int(x))["roc"] == 1]
        assert wrapped, "no stream wrapped its ROC"
        st = d.stats()
        assert st["chain_stalls"] == 0 and st["status"]["ERR_INTERNAL"] == 0
    finally:
        d.close()
