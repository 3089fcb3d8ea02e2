"""Golden fixtures (tests/golden/*.npz): recorded SRTP/SRTCP bundles with their
expected ciphertext, tags, statuses, lengths and final context state.

* CPU: the C oracle and the independent Python restatement each reproduce
  every fixture (pins the oracle the GPU parity tests trust).
* GPU: the MI355X engine, through its C ABI, reproduces every fixture bit for
  bit -- the same vectors, no oracle in the loop.
"""
import os

import pytest

from golden_replay import EngineBackend, OracleBackend, PyrefBackend, fixtures, replay

FIXTURES = fixtures()
IDS = [os.path.basename(p)[:-4] for p in FIXTURES]


def test_fixture_set_complete():
    names = set(IDS)
    for need in ("libsrtp_kat", "c1_opus160_wrap", "c2_video1200", "c3_mixed_faults",
                 "c4_srtp_srtcp_rekey", "edge_replay_quirks", "edge_roc_overturn",
                 "edge_malformed_abort", "edge_malformed_noabort", "edge_flags_lifecycle",
                 "edge_check_replay_off", "null_profiles", "sdes_f8"):
        assert need in names, need


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_oracle_reproduces_fixture(path, oracle):
    replay(path, OracleBackend)


@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_pyref_reproduces_fixture(path):
    replay(path, PyrefBackend)


@pytest.mark.gpu
@pytest.mark.parametrize("path", FIXTURES, ids=IDS)
def test_engine_reproduces_fixture(path, engine_factory):
    replay(path, EngineBackend, make_engine=engine_factory)
