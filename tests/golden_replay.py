"""Replay of the golden fixtures (tests/golden/*.npz, written by
tests/golden/make_golden.py) against one implementation.

A backend provides factory / transformer / set_factory / close_factory /
close_transformer / bundle / state; ``replay`` runs a fixture's operation
script through it and asserts bit equality with the recorded outputs:
per-packet status, length, every byte of the packed segment, and the final
context state of every (transformer, SSRC) pair the fixture touched.
"""
from __future__ import annotations

import glob
import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
STATUS_NAMES = ["OK", "DROP_REPLAY", "DROP_AUTH", "DROP_VERSION", "DROP_NO_CONTEXT",
                "ERR_CAPACITY", "ERR_MALFORMED", "DROP_INVALID", "NOT_PROCESSED", "SKIPPED"]


def fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def load(path):
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return meta, z


def replay(path, backend_cls, **kw):
    meta, z = load(path)
    be = backend_cls(check_replay=meta["check_replay"], abort_on_error=meta["abort_on_error"], **kw)
    try:
        fac, trans, outs = [], [], []
        for op in meta["ops"]:
            kind = op["op"]
            if kind == "factory":
                fac.append(be.factory(op["sender"], bytes.fromhex(op["key"]),
                                      bytes.fromhex(op["salt"]), op["srtp"], op["srtcp"]))
            elif kind == "transformer":
                trans.append(be.transformer(op["kind"], fac[op["fwd"]], fac[op["rev"]]))
            elif kind == "set_factory":
                be.set_factory(trans[op["t"]], fac[op["f"]], op["forward"])
            elif kind == "close_factory":
                be.close_factory(fac[op["f"]])
            elif kind == "close_transformer":
                be.close_transformer(trans[op["t"]])
            elif kind == "bundle":
                j = op["j"]
                p = f"b{j}_"
                seg_in = (outs[int(z[p + "seg_in_from"])] if p + "seg_in_from" in z
                          else z[p + "seg_in"])
                seg = np.array(seg_in, np.uint8, copy=True)
                ln = np.array(z[p + "len_in"], np.uint32, copy=True)
                off, cap, flags = z[p + "off"], z[p + "cap"], z[p + "flags"]
                tids = [trans[t] if t >= 0 else None for t in z[p + "tids"]]
                st = np.asarray(be.bundle(tids, op["reverse"], seg, off, ln, cap, flags), np.int32)
                want_st = z[p + "status"]
                bad = np.nonzero(st != want_st)[0]
                assert len(bad) == 0, (
                    f"{meta['name']} bundle {j}: status differs at {bad[:8].tolist()}: got "
                    f"{[STATUS_NAMES[s] if 0 <= s < len(STATUS_NAMES) else s for s in st[bad[:8]]]} want "
                    f"{[STATUS_NAMES[s] for s in want_st[bad[:8]]]}")
                bad = np.nonzero(ln != z[p + "len_out"])[0]
                assert len(bad) == 0, f"{meta['name']} bundle {j}: length differs at {bad[:8].tolist()}"
                want = z[p + "seg_out"]
                if not np.array_equal(seg, want):
                    d = np.nonzero(seg != want)[0]
                    pk = np.searchsorted(off.astype(np.int64), d[:5], side="right") - 1
                    raise AssertionError(f"{meta['name']} bundle {j}: {len(d)} segment bytes "
                                         f"differ, first at {d[:5].tolist()} (packets {pk.tolist()})")
                outs.append(want)
            else:
                raise ValueError(kind)
        for s in meta["states"]:
            got = be.state(trans[s["t"]], s["ssrc"])
            if s["state"] is None:
                assert got is None, f"{meta['name']}: context (t{s['t']}, {s['ssrc']:#x}) should not exist"
                continue
            assert got is not None, f"{meta['name']}: context (t{s['t']}, {s['ssrc']:#x}) missing"
            for k, v in s["state"].items():
                assert int(got[k]) == v, (f"{meta['name']}: state {k} of (t{s['t']}, "
                                          f"{s['ssrc']:#x}) is {got[k]}, want {v}")
    finally:
        be.finish()
    return meta


class OracleBackend:
    """The C restatement (oracle/srtp_oracle.c)."""

    def __init__(self, check_replay, abort_on_error):
        from oracle import oracle as O
        self.O, self.abort = O, abort_on_error
        O.set_check_replay(check_replay)

    def factory(self, sender, key, salt, p_rtp, p_rtcp):
        return self.O.Factory(sender, key, salt, self.O.Policy(*p_rtp), self.O.Policy(*p_rtcp))

    def transformer(self, kind, f, r):
        return self.O.Transformer(kind, f, r)

    def set_factory(self, t, f, forward):
        t.set_factory(f, forward)

    def close_factory(self, f):
        f.close()

    def close_transformer(self, t):
        t.close()

    def bundle(self, ts, reverse, seg, off, ln, cap, flags):
        return self.O.process(ts, reverse, seg, off, ln, cap, flags, self.abort)

    def state(self, t, ssrc):
        return t.state(ssrc)

    def finish(self):
        self.O.set_check_replay(True)


class PyrefBackend(OracleBackend):
    """The independent pure-Python restatement (oracle/pyref.py)."""

    def __init__(self, check_replay, abort_on_error):
        from oracle import pyref as R
        self.R, self.abort = R, abort_on_error
        R.CHECK_REPLAY[0] = check_replay

    def factory(self, sender, key, salt, p_rtp, p_rtcp):
        return self.R.Factory(sender, key, salt, tuple(p_rtp), tuple(p_rtcp))

    def transformer(self, kind, f, r):
        return self.R.Transformer(kind, f, r)

    def bundle(self, ts, reverse, seg, off, ln, cap, flags):
        return self.R.process(list(ts), reverse, seg, off, ln, cap, flags, self.abort)

    def state(self, t, ssrc):
        c = t.ctx.get(ssrc)
        if c is None:
            return None
        return {"roc": c.roc, "s_l": c.s_l, "seq_num_set": int(c.seq_set),
                "guessed_roc": c.guessed, "sent_index": c.sent, "received_index": c.recv,
                "replay_window": c.window & 0xFFFFFFFFFFFFFFFF}

    def finish(self):
        self.R.CHECK_REPLAY[0] = True


class EngineBackend:
    """The MI355X engine through its C ABI (libjitsi_amd/libsrtp_mi355x.so),
    via the host mirror of the Java API (libjitsi_amd/srtp.py)."""

    def __init__(self, check_replay, abort_on_error, make_engine):
        import libjitsi_amd as J
        self.J = J
        self.eng = make_engine(check_replay=check_replay, abort_on_error=abort_on_error,
                               max_contexts=1 << 12, max_factories=256, max_transformers=256)

    def factory(self, sender, key, salt, p_rtp, p_rtcp):
        P = self.J.SRTPPolicy
        return self.J.SRTPContextFactory(sender, key, salt, P(*p_rtp), P(*p_rtcp), engine=self.eng)

    def transformer(self, kind, f, r):
        cls = self.J.SRTPTransformer if kind == 0 else self.J.SRTCPTransformer
        return cls(f, r)

    def set_factory(self, t, f, forward):
        t._set_factory(f, forward)

    def close_factory(self, f):
        f.close()

    def close_transformer(self, t):
        t.close()

    def bundle(self, ts, reverse, seg, off, ln, cap, flags):
        tids = np.array([t.tid if t is not None else -1 for t in ts], np.int32)
        return self.eng.transform_host(reverse, tids, seg, off, ln, cap, flags)

    def state(self, t, ssrc):
        return self.eng.context_state(t, ssrc)

    def finish(self):
        self.eng.close()
