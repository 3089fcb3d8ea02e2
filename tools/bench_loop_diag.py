"""GPU diagnostic for the bench loop: per-step status histograms + oracle twin."""
import sys, numpy as np, torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, profile_policies, synth
from oracle import oracle as O
n, nssrc, L = 1 << 18, 10000, 1200
b = synth.rtp_bundle(n, nssrc, L, seed=synth.SEED_BASE + 2)
eng = SRTPEngine(max_contexts=1 << 16, max_factories=64, max_transformers=64, max_batch=n)
(k, s), = synth.keys(2, 1)
pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng))
pol = O.Policy(1, 16, 1, 20, 10, 14)
ofs, ofr = O.Factory(True, k, s, pol, pol), O.Factory(False, k, s, pol, pol)
ots, otr = O.Transformer(0, ofs, ofs), O.Transformer(0, ofr, ofr)
seg, ln = b.seg.copy(), b.length.copy()
o = b.off.astype(np.int64)
step = -(-n // nssrc)
for it in range(4):
    sego, lno = seg.copy(), ln.copy()
    st = eng.transform_host(False, snd.tid, seg, b.off, ln, b.cap)
    sto = O.process(ots, False, sego, b.off, lno, b.cap)
    print(it, "protect eng", np.bincount(st, minlength=10), "oracle", np.bincount(sto, minlength=10),
          "seg equal", np.array_equal(seg, sego), flush=True)
    if not np.array_equal(st, sto):
        bad = np.nonzero(st != sto)[0][:5]
        print(" first diffs", bad, st[bad], sto[bad], b.ssrc[bad], [int.from_bytes(seg[o[i]+2:o[i]+4].tobytes(),'big') for i in bad])
    st2 = eng.transform_host(True, rcv.tid, seg, b.off, ln, b.cap)
    st2o = O.process(otr, True, sego, b.off, lno, b.cap)
    print(it, "unprotect eng", np.bincount(st2, minlength=10), "oracle", np.bincount(st2o, minlength=10), flush=True)
    if not np.array_equal(st2, st2o):
        bad = np.nonzero(st2 != st2o)[0][:5]
        print(" first diffs", bad, st2[bad], st2o[bad], b.ssrc[bad])
        for i in bad[:2]:
            print("  eng state", eng.context_state(rcv, int(b.ssrc[i])), "oracle", otr.state(int(b.ssrc[i])))
    q = ((seg[o + 2].astype(np.int64) << 8) | seg[o + 3]) + step
    seg[o + 2] = ((q >> 8) & 0xFF).astype(np.uint8); seg[o + 3] = (q & 0xFF).astype(np.uint8)
