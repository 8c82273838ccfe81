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


def test_dense_to_nbr_max_degree():
    """dense_to_nbr: ascending neighbour ids, -1 padding up to max_degree (the reference's
    _get_neighbor_h zero-pads to max_degree slots, src/model.py:582-595); the computed width
    equals the largest degree."""
    import torch

    M, _ = mods()
    adj = torch.zeros(2, 5, 5)
    for b, edges in enumerate([[(0, 1), (0, 2), (1, 3), (2, 4), (3, 4)], [(0, 4), (1, 2)]]):
        for i, j in edges:
            adj[b, i, j] = adj[b, j, i] = 1.0
    mask = adj + torch.eye(5)
    nbr = M.dense_to_nbr(mask)
    assert nbr.shape == (2, 5, 2) and nbr.dtype == torch.int32
    assert nbr[0, 0].tolist() == [1, 2] and nbr[0, 4].tolist() == [2, 3]
    assert nbr[1, 3].tolist() == [-1, -1] and nbr[1, 4].tolist() == [0, -1]
    wide = M.dense_to_nbr(mask, max_degree=3)
    assert wide.shape == (2, 5, 3)
    assert torch.equal(wide[..., :2], nbr) and (wide[..., 2] == -1).all()
