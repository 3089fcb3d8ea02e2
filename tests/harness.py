"""Paired oracle / MI355X-engine objects for parity tests.

Every factory and transformer is created twice with identical arguments --
once in the C oracle (oracle/srtp_oracle.c, the CPU restatement of the
reference) and once in the engine -- and every bundle is run through both on
identical bytes.  ``run`` asserts that statuses, lengths, the whole packed
segment and the touched contexts' state agree bit for bit.
"""
from __future__ import annotations

import numpy as np

from libjitsi_amd import SRTCPTransformer, SRTPContextFactory, SRTPPolicy, SRTPTransformer
from libjitsi_amd import _native as N
from oracle import oracle as O

STATE_KEYS_RTP = ("roc", "s_l", "seq_num_set", "guessed_roc", "replay_window")
STATE_KEYS_RTCP = ("sent_index", "received_index", "replay_window")


def opol(p: SRTPPolicy) -> O.Policy:
    return O.Policy(p.encType, p.encKeyLength, p.authType, p.authKeyLength, p.authTagLength,
                    p.saltKeyLength)


class TwinFactory:
    def __init__(self, twin, sender, key, salt, srtp_pol, srtcp_pol):
        self.o = O.Factory(sender, key, salt, opol(srtp_pol), opol(srtcp_pol))
        self.e = SRTPContextFactory(sender, key, salt, srtp_pol, srtcp_pol, engine=twin.engine)

    def close(self):
        self.o.close()
        self.e.close()


class TwinTransformer:
    def __init__(self, twin, kind, fwd: TwinFactory, rev: TwinFactory):
        self.kind = kind
        self.o = O.Transformer(kind, fwd.o, rev.o)
        cls = SRTPTransformer if kind == O.KIND_RTP else SRTCPTransformer
        self.e = cls(fwd.e, rev.e)
        self.tid = self.e.tid

    def set_factory(self, f: TwinFactory, forward: bool):
        self.o.set_factory(f.o, forward)
        self.e._set_factory(f.e, forward)

    def close(self):
        self.o.close()
        self.e.close()


class Twin:
    def __init__(self, engine, check_replay=True):
        self.engine = engine
        O.set_check_replay(check_replay)

    def factory(self, sender, key, salt, srtp_pol, srtcp_pol=None):
        return TwinFactory(self, sender, key, salt, srtp_pol, srtcp_pol or srtp_pol)

    def transformer(self, kind, fwd, rev=None):
        return TwinTransformer(self, kind, fwd, rev or fwd)

    def run(self, transformers, reverse, seg, off, length, cap, flags=None, abort_on_error=True,
            check_state=True, ssrc_of=None):
        """Run one bundle through oracle and engine; assert identical results.
        ``transformers``: one TwinTransformer or a list with one per packet.
        Returns (seg, length, status) of the engine run."""
        n = len(off)
        seg_o, len_o = seg.copy(), length.copy()
        seg_e, len_e = seg.copy(), length.copy()
        if isinstance(transformers, TwinTransformer):
            st_o = O.process(transformers.o, reverse, seg_o, off, len_o, cap, flags, abort_on_error)
            st_e = self.engine.transform_host(reverse, transformers.tid, seg_e, off, len_e, cap,
                                              flags)
            per_pkt = [transformers] * n
        else:
            st_o = O.process([t.o if t else None for t in transformers], reverse, seg_o, off,
                             len_o, cap, flags, abort_on_error)
            tids = np.array([t.tid if t else -1 for t in transformers], np.int32)
            st_e = self.engine.transform_host(reverse, tids, seg_e, off, len_e, cap, flags)
            per_pkt = list(transformers)
        bad = np.nonzero(st_o != st_e)[0]
        assert len(bad) == 0, (
            f"status mismatch at {bad[:10].tolist()}: oracle "
            f"{[N.STATUS_NAMES[s] for s in st_o[bad[:10]]]} engine "
            f"{[N.STATUS_NAMES[s] if 0 <= s < N.NUM_STATUS else s for s in st_e[bad[:10]]]}")
        bad = np.nonzero(len_o != len_e)[0]
        assert len(bad) == 0, f"length mismatch at {bad[:10].tolist()}: {len_o[bad[:10]]} vs {len_e[bad[:10]]}"
        if not np.array_equal(seg_o, seg_e):
            diff = np.nonzero(seg_o != seg_e)[0]
            pk = np.searchsorted(off.astype(np.int64), diff[:5], side="right") - 1
            p0 = int(pk[0])
            o0, c0 = int(off[p0]), int(cap[p0])
            raise AssertionError(
                f"segment bytes differ at {diff[:5].tolist()} (packets {pk.tolist()}, status "
                f"{st_o[pk].tolist()}); {len(diff)} bytes in total; reverse={reverse}; packet {p0} "
                f"len in {int(length[p0])} out {int(len_o[p0])}\n in  {seg[o0:o0 + c0].tobytes().hex()}"
                f"\n ora {seg_o[o0:o0 + c0].tobytes().hex()}\n eng {seg_e[o0:o0 + c0].tobytes().hex()}")
        if check_state:
            self.check_states(per_pkt, seg, off, length)
        return seg_e, len_e, st_e

    def check_states(self, per_pkt, seg, off, length):
        seen = set()
        for i, t in enumerate(per_pkt):
            if t is None or length[i] < 12:
                continue
            o = int(off[i])
            so = 8 if t.kind == O.KIND_RTP else 4
            ssrc = int.from_bytes(seg[o + so:o + so + 4].tobytes(), "big")
            if (t.tid, ssrc) in seen:
                continue
            seen.add((t.tid, ssrc))
            so_ = t.o.state(ssrc)
            se_ = self.engine.context_state(t.e, ssrc)
            assert (so_ is None) == (se_ is None), f"context existence differs for ssrc {ssrc:#x}: {so_} {se_}"
            if so_ is None:
                continue
            keys = STATE_KEYS_RTP if t.kind == O.KIND_RTP else STATE_KEYS_RTCP
            for k in keys:
                assert so_[k] == se_[k], f"state {k} differs for ssrc {ssrc:#x}: oracle {so_} engine {se_}"
