"""Diagnostic: k_unprotect vs k_protect per-bundle time at two packet sizes
under SRTP_DEBUG variants of k_unprotect (0 = normal, 3 = no midstate /
ciphertext-tail stores, 5 = no speculative decryption).  Results of modes 3/5
are wrong by design; only the timings matter."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, %r)
from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, profile_policies, synth
n, nssrc = 1 << 18, 10000
import os
TWO = os.environ.get('PROBE_TWO') == '1'
res = {}
for L in (160, 1200):
    b = synth.rtp_bundle(n, nssrc, L, seed=synth.SEED_BASE + 2)
    eng = SRTPEngine(max_contexts=1 << 17, max_factories=64, max_transformers=64, max_batch=n)
    (k, s), = synth.keys(2, 1)
    pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
    dev = torch.device("cuda", 0)
    off = torch.from_numpy(b.off.view(np.int32)).to(dev); cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
    st = torch.empty(n, dtype=torch.int32, device=dev)
    seg0 = torch.from_numpy(b.seg).to(dev); ln0 = torch.from_numpy(b.length.view(np.int32)).to(dev)
    eng.set_timing(True)
    r = {}
    seq_step = -(-n // nssrc)
    off64 = off.to(torch.int64)
    eng2 = SRTPEngine(max_contexts=1 << 14, max_factories=64, max_transformers=64, max_batch=n) \
        if TWO else eng
    eng2.set_timing(True)
    snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
    rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng2))
    tp, tv = [], []
    for it in range(6):  # one sender / receiver pair, steady state as in bench.py
        seg, ln = seg0.clone(), ln0.clone()
        hi, lo = seg[off64 + 2].to(torch.int32), seg[off64 + 3].to(torch.int32)
        q = ((hi << 8) | lo) + it * seq_step
        seg[off64 + 2] = ((q >> 8) & 0xFF).to(torch.uint8)
        seg[off64 + 3] = (q & 0xFF).to(torch.uint8)
        torch.cuda.synchronize(); eng.read_timing(); eng2.read_timing()
        eng.transform_device(False, snd.tid, seg, off, ln, cap, st)
        torch.cuda.synchronize()
        tp.append(round(eng.read_timing()["protect"][0], 4))
        eng2.transform_device(True, rcv.tid, seg, off, ln, cap, st)
        torch.cuda.synchronize()
        tv.append(round(eng2.read_timing()["verify"][0], 4))
        assert int((st != 0).sum()) == 0, "not all packets accepted"
    r = {"protect_ms": tp, "verify_ms": tv}
    res[L] = r
print(json.dumps(res))
''' % ROOT
for mode, two in (("0", "0"), ("0", "1")):
    env = dict(os.environ, SRTP_DEBUG=mode, PROBE_TWO=two)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print("SRTP_DEBUG=%s two_engines=%s" % (mode, two), out.stdout.strip(), out.stderr.strip()[-300:] if out.returncode else "", flush=True)
