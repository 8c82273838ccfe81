"""Host-side model logic (no GPU, no kernel calls): NetMon state sizes for the carry-over
variants (reference src/model.py:380-391) and the fused-DQN-head eligibility rule."""
import importlib

import pytest


def mods():
    return importlib.import_module("graph-marl_amd.model"), importlib.import_module("graph-marl_amd.fused")


@pytest.mark.parametrize("rnn,carry,states", [("lstm", True, 2), ("lstm", False, 4), ("lnlstm", False, 4),
                                              ("gru", True, 1), ("gru", False, 2)])
def test_netmon_state_size(rnn, carry, states):
    M, _ = mods()
    nm = M.NetMon(88, 32, [64, 48], 1, rnn_type=rnn, rnn_carryover=carry)
    assert nm.get_state_size() == 32 * states
    assert nm.get_out_features() == 4 * 32


def test_netmon_no_carryover_needs_an_iteration():
    M, _ = mods()
    with pytest.raises(ValueError):
        M.NetMon(88, 32, [64, 48], 0, rnn_carryover=False)


def test_fused_head_eligibility(monkeypatch):
    """gm_gemm_x3_head takes the last hidden layer + Q head when the layer is <= 256 wide and
    the head <= 4 outputs (split-f16 form only)."""
    M, FU = mods()
    monkeypatch.setattr(FU.L, "GEMM_MODE", "x3")
    assert FU.head_ok(M.Linear(512, 256, act=1), M.Linear(256, 4))
    assert not FU.head_ok(M.Linear(512, 512, act=1), M.Linear(512, 4))   # wider than one tile
    assert not FU.head_ok(M.Linear(512, 256, act=1), M.Linear(256, 5))   # more than 4 heads
    assert not FU.head_ok(M.Linear(512, 256, act=1), M.Linear(256, 4, act=1))
    monkeypatch.setattr(FU.L, "GEMM_MODE", "f32")
    assert not FU.head_ok(M.Linear(512, 256, act=1), M.Linear(256, 4))
