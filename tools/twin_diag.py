import os, sys; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'tests'))
import numpy as np
from libjitsi_amd import SRTPEngine, profile_policies, synth
from harness import Twin
from oracle import oracle as O
from test_gpu_parity import malformed_bundle
P80 = profile_policies("AES_CM_128_HMAC_SHA1_80")
eng = SRTPEngine(max_contexts=1024, max_factories=64, max_transformers=64)
def mk(pk):
    caps = np.array([(c + 15) // 16 * 16 for _, c in pk], np.uint32)
    off = np.concatenate([[0], np.cumsum(caps[:-1])]).astype(np.uint32)
    seg = np.zeros(int(caps.sum()), np.uint8)
    ln = np.array([len(p) for p, _ in pk], np.uint32)
    for i, (p, _) in enumerate(pk):
        seg[off[i]:off[i] + len(p)] = np.frombuffer(p, np.uint8)
    return seg, off, ln, caps
pk = malformed_bundle()
for name, sel in [("only0", [0]), ("0and7", [0, 7]), ("all", list(range(len(pk))))]:
    twin = Twin(eng)
    (k, s), = synth.keys(12, 1)
    f = twin.factory(True, k, s, *P80); fr = twin.factory(False, k, s, *P80)
    t = twin.transformer(O.KIND_RTP, f); r = twin.transformer(O.KIND_RTP, fr)
    seg, off, ln, caps = mk([pk[i] for i in sel])
    for rep in range(2):
        for rev, (tt, sg, l) in enumerate([(t, seg, ln)]):
            pass
        try:
            seg2, ln2, st = twin.run(t, False, seg, off, ln, caps, check_state=False)
            print(name, rep, "protect", st, flush=True)
            seg3, ln3, st3 = twin.run(r, True, seg2, off, ln2, caps, check_state=False)
            print(name, rep, "unprotect", st3, flush=True)
        except AssertionError as e:
            print(name, rep, "FAIL", str(e)[:300], flush=True)
