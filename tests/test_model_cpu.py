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


def test_fold_env_weight_exact_on_routing_rows():
    """fused.fold_env_weight: W x == W' x' for agent rows of the routing observation layout
    (src/env/routing.py:269-315), x' = x without columns N-1 and 2N (gm_obs_buffers.obs_gemm)."""
    import numpy as np
    import torch

    _, FU = mods()
    rng = np.random.RandomState(3)
    for n in (4, 20, 30):
        D = 6 * n + 10
        rows = []
        for _ in range(64):
            o = np.zeros(D)
            now, tgt = rng.randint(n), rng.randint(n)
            o[now] = 1
            o[n + tgt] = 1
            if rng.rand() < 0.5:
                o[2 * n] = 1
                o[2 * n + 1 + rng.randint(n)] = 1
            o[3 * n + 1:3 * n + 4] = rng.rand(3) * 10
            for k in range(3):
                blk = 3 * n + 4 + k * (n + 2)
                o[blk + rng.randint(n)] = 1
                o[blk + n:blk + n + 2] = rng.rand(2)
            rows.append(o)
        x = torch.tensor(np.array(rows))
        keep = [c for c in range(D) if c not in (n - 1, 2 * n)]
        w = torch.tensor(rng.standard_normal((16, D)))
        wf = FU.fold_env_weight(w, n)
        assert wf.shape == (16, D - 2)
        torch.testing.assert_close(x @ w.t(), x[:, keep] @ wf.t(), rtol=1e-12, atol=1e-12)


def test_activation_names_cover_the_elementwise_functionals():
    """--activation-function takes any elementwise torch.nn.functional name (src/main.py:440-441
    getattr(F, name)); each code maps to a GEMM epilogue, the pre-activation ones are flagged; names
    that are not elementwise with defaults are refused."""
    import importlib

    import pytest
    import torch.nn.functional as F

    M = importlib.import_module("graph-marl_amd.model")
    for name, code in M.ACTIVATIONS.items():
        assert hasattr(F, name) and M.act_code(name) == code and M.act_code(getattr(F, name)) == code
        assert M.epi_code(code) in (0, 1, 4, 5, 6, 7) or M.epi_code(code) == M.GM_EPI_BIAS_ACT + code
    assert {n for n, c in M.ACTIVATIONS.items() if c in M.Z_ACTS} == {"gelu", "silu", "mish", "hardswish", "tanhshrink"}
    assert len(set(M.ACTIVATIONS.values())) == len(M.ACTIVATIONS) == 18
    for bad in ("softmax", "glu", "rrelu"):
        with pytest.raises(NotImplementedError):
            M.act_code(bad)
