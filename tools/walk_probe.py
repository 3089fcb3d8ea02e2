"""Diagnostic: per-stage engine timings of the bench workload under SRTP_DEBUG
walk variants (0 = normal, 1 = k_walk stages records only, 2 = no walk_one).
Results of modes 1/2 are wrong by design; only the timings matter."""
import os, subprocess, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, json, numpy as np, torch
sys.path.insert(0, %r)
from libjitsi_amd import SRTPContextFactory, SRTPEngine, SRTPTransformer, profile_policies, synth
n, nssrc, L = 1 << 18, 10000, 1200
b = synth.rtp_bundle(n, nssrc, L, seed=synth.SEED_BASE + 2)
eng = SRTPEngine(max_contexts=1 << 16, max_factories=64, max_transformers=64, max_batch=n)
(k, s), = synth.keys(2, 1)
pols = profile_policies("AES_CM_128_HMAC_SHA1_80")
snd = SRTPTransformer(SRTPContextFactory(True, k, s, *pols, engine=eng))
rcv = SRTPTransformer(SRTPContextFactory(False, k, s, *pols, engine=eng))
dev = torch.device("cuda", 0)
off = torch.from_numpy(b.off.view(np.int32)).to(dev); cap = torch.from_numpy(b.cap.view(np.int32)).to(dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
res = {}
for rev in (False, True):
    seg = torch.from_numpy(b.seg).to(dev); ln = torch.from_numpy(b.length.view(np.int32)).to(dev)
    if rev:
        eng.transform_device(False, snd.tid, seg, off, ln, cap, st)
    for it in range(4):
        sg, l2 = seg.clone(), ln.clone()
        torch.cuda.synchronize()
        eng.set_timing(True); eng.read_timing()
        eng.transform_device(rev, (rcv if rev else snd).tid, sg, off, l2, cap, st)
        torch.cuda.synchronize()
        t = eng.read_timing(); eng.set_timing(False)
    res["unprotect" if rev else "protect"] = {k: round(v[0] / max(v[1], 1), 4) for k, v in t.items() if v[1]}
print(json.dumps(res))
''' % ROOT
for mode in ("0", "1", "2"):
    env = dict(os.environ, SRTP_DEBUG=mode)
    out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print("SRTP_DEBUG=%s" % mode, out.stdout.strip(), out.stderr.strip()[-300:] if out.returncode else "")
