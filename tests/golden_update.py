"""Loading and checking the reference's golden DQN + NetMon updates (tests/golden/train*.npz,
made by tests/golden/make_golden.py gen_train from src/main.py:832-1022).

Small goldens store every parameter and output in full. Compact goldens (production sizes,
`compact` = 1) store no parameters: the modules are filled from tests/golden/detparams.py with
the golden's `det_seed`, exactly as the generator filled the reference's modules; outputs above
8192 elements are stored at sampled positions plus their row and column sums.
"""
import os
import sys

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
sys.path.insert(0, GOLDEN)
import detparams  # noqa: E402


def arch(g):
    """(rnn_type, agg, K, H, encoder units, DQN units) of a golden update."""
    if "arch" not in g.files:
        return "lstm", "sum", 1, 32, [64, 48], [64, 32]
    r, a, k, h, e, q = str(g["arch"]).split("|")[:6]
    return r, a, int(k), int(h), [int(x) for x in e.split(",")], [int(x) for x in q.split(",")]


def activation(g):
    """--activation-function of a golden update (leaky_relu before the field existed)."""
    parts = str(g["arch"]).split("|") if "arch" in g.files else []
    return parts[6] if len(parts) > 6 else "leaky_relu"


def compact(g):
    return "compact" in g.files and int(g["compact"]) == 1


def _sd(g, prefix):
    return {k[len(prefix):]: torch.as_tensor(g[k]) for k in g.files
            if k.startswith(prefix) and not k.startswith(prefix + "after_") and k != "aux_coeff"}


def build(g, M, dev):
    """(netmon, model, target, node_state0) of a golden update, on dev."""
    rnn, agg, K, H, enc, dq = arch(g)
    nd = g["node_obs"].shape[-1]
    act = activation(g)
    netmon = M.NetMon(nd, H, enc, K, rnn_type=rnn, agg_type=agg, activation=act).to(dev)
    obs_dim = g["agent_obs"].shape[-1] + netmon.get_out_features()
    model = M.DQN(obs_dim, dq, 4, activation=act).to(dev)
    target = M.DQN(obs_dim, dq, 4, activation=act).to(dev)
    B, n = g["node_obs"].shape[1:3]
    if compact(g):
        seed = int(g["det_seed"])
        for prefix, mod in (("netmon.", netmon), ("model.", model)):
            sd = mod.state_dict()
            vals = detparams.det_state_dict(seed, {prefix + k: tuple(v.shape) for k, v in sd.items()})
            mod.load_state_dict({k: torch.as_tensor(vals[prefix + k]) for k in sd})
        target.load_state_dict({k: torch.as_tensor(detparams.det_perturb(seed, "target." + k, v.cpu().numpy()))
                                for k, v in model.state_dict().items()})
        state0 = detparams.det_state(seed, (B, n, netmon.get_state_size()))
    else:
        netmon.load_state_dict(_sd(g, "netmon_"))
        model.load_state_dict(_sd(g, "model_"))
        target.load_state_dict(_sd(g, "target_"))
        state0 = g["node_state0"]
    return netmon, model, target, torch.as_tensor(state0, device=dev)


def weights_np(g):
    """fp64 numpy (NetMon, DQN, target DQN, initial state) weight dicts of a golden update, keyed
    like the reference's state_dicts (for oracle/netmon_ref.py)."""
    if not compact(g):
        W = lambda p: {k[len(p):]: g[k].astype(np.float64) for k in g.files  # noqa: E731
                       if k.startswith(p) and not k.startswith(p + "after_")}
        return W("netmon_"), W("model_"), W("target_"), g["node_state0"].astype(np.float64)
    import importlib

    M = importlib.import_module("graph-marl_amd.model")
    netmon, model, target, state0 = build(g, M, torch.device("cpu"))
    sd = lambda m: {k: v.double().numpy() for k, v in m.state_dict().items()}  # noqa: E731
    return sd(netmon), sd(model), sd(target), state0.double().numpy()


def count_excess(g, key, actual, atol):
    """(elements off by more than atol, elements compared) of actual vs the golden `key` (every
    element, or a compact entry's sampled positions)."""
    a = (actual.detach().cpu().numpy() if torch.is_tensor(actual) else np.asarray(actual)).astype(np.float64)
    if key in g.files:
        return int((np.abs(a - g[key]) > atol).sum()), a.size
    idx = g[key + "__idx"]
    return int((np.abs(a.reshape(-1)[idx] - g[key + "__val"]) > atol).sum()), len(idx)


def check(g, key, actual, atol, rtol, what=""):
    """actual (tensor / array) vs the golden array `key`, elementwise |a - r| <= atol + rtol |r|;
    for a compact entry at its sampled positions, and its row / column sums within the bound the
    elementwise tolerance implies (atol * count + rtol * sum |a|)."""
    a = actual.detach().cpu().numpy() if torch.is_tensor(actual) else np.asarray(actual)
    at = np.broadcast_to(np.asarray(atol, np.float64), a.shape)  # scalar or per-element
    if key in g.files:
        err = np.abs(a.astype(np.float64) - g[key]) - (at + rtol * np.abs(g[key]))
        assert (err <= 0).all(), f"{what or key}: {(err > 0).sum()} elements off, worst excess {err.max()}"
        return
    assert tuple(g[key + "__shape"]) == a.shape, f"{key}: shape {a.shape} vs {tuple(g[key + '__shape'])}"
    idx = g[key + "__idx"]
    ref = g[key + "__val"].astype(np.float64)
    err = np.abs(a.reshape(-1)[idx] - ref) - (at.reshape(-1)[idx] + rtol * np.abs(ref))
    assert (err <= 0).all(), f"{what or key} (sampled): {(err > 0).sum()} elements off, worst excess {err.max()}"
    a64 = a.astype(np.float64)
    rows = a64.reshape(a.shape[0], -1)
    tol = at.reshape(a.shape[0], -1).sum(1) + rtol * np.abs(rows).sum(1)
    err = np.abs(rows.sum(1) - g[key + "__rowsum"])
    assert (err <= tol).all(), f"{what or key}: row sums off by up to {err.max()} (tol {tol[err.argmax()]})"
    if a.ndim == 2:
        tol = at.sum(0) + rtol * np.abs(a64).sum(0)
        err = np.abs(a64.sum(0) - g[key + "__colsum"])
        assert (err <= tol).all(), f"{what or key}: column sums off by up to {err.max()} (tol {tol[err.argmax()]})"

