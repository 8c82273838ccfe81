"""NumPy float64 restatement of NetMon / DQN forward (reference src/model.py,
src/layernormlstm.py). TEST INFRASTRUCTURE ONLY (parity checker).

Weights are passed as a dict of numpy arrays keyed like the reference's
state_dict (e.g. "encode.linear_layers.0.weight", "rnn_obs.weight_ih").
"""
import numpy as np


def leaky_relu(x, slope=0.01):
    return np.where(x >= 0, x, slope * x)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def linear(x, w, b=None):
    y = x @ w.T
    return y if b is None else y + b


def activation(x, name="leaky_relu"):
    """torch.nn.functional activations selectable by --activation-function (src/main.py:440-441)."""
    if name == "leaky_relu":
        return leaky_relu(x)
    if name == "relu":
        return np.maximum(x, 0.0)
    if name == "elu":
        return np.where(x > 0, x, np.expm1(np.minimum(x, 0.0)))
    if name == "tanh":
        return np.tanh(x)
    if name == "sigmoid":
        return sigmoid(x)
    # the rest of the elementwise torch.nn.functional names with their defaults (round 4)
    sp = lambda v: np.where(v > 20.0, v, np.log1p(np.exp(np.minimum(v, 20.0))))  # softplus, threshold 20
    if name == "relu6":
        return np.clip(x, 0.0, 6.0)
    if name == "hardtanh":
        return np.clip(x, -1.0, 1.0)
    if name == "hardsigmoid":
        return np.clip(x + 3.0, 0.0, 6.0) / 6.0
    if name == "selu":
        a, s = 1.6732632423543772848170429916717, 1.0507009873554804934193349852946
        return s * np.where(x > 0, x, a * np.expm1(np.minimum(x, 0.0)))
    if name == "celu":
        return np.where(x > 0, x, np.expm1(np.minimum(x, 0.0)))
    if name == "softsign":
        return x / (1.0 + np.abs(x))
    if name == "logsigmoid":
        return np.minimum(x, 0.0) - np.log1p(np.exp(-np.abs(x)))
    if name == "softplus":
        return sp(x)
    if name == "gelu":
        from scipy.special import erf
        return 0.5 * x * (1.0 + erf(x / np.sqrt(2.0)))
    if name == "silu":
        return x * sigmoid(x)
    if name == "mish":
        return x * np.tanh(sp(x))
    if name == "hardswish":
        return x * np.clip(x + 3.0, 0.0, 6.0) / 6.0
    if name == "tanhshrink":
        return x - np.tanh(x)
    raise ValueError(f"activation {name!r} not restated")


def mlp(x, W, prefix, n_layers, act_on_output=True, act="leaky_relu"):
    """src/model.py:13-42 MLP (activation also on the output by default)."""
    for i in range(n_layers):
        x = linear(x, W[f"{prefix}.linear_layers.{i}.weight"], W[f"{prefix}.linear_layers.{i}.bias"])
        if i < n_layers - 1 or act_on_output:
            x = activation(x, act)
    return x


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * w + b


def lstm_cell(x, h, c, W, p):
    """torch.nn.LSTMCell (gate order i, f, g, o)."""
    g = linear(x, W[p + ".weight_ih"], W[p + ".bias_ih"]) + linear(h, W[p + ".weight_hh"], W[p + ".bias_hh"])
    H = h.shape[-1]
    i, f, gg, o = sigmoid(g[:, :H]), sigmoid(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), sigmoid(g[:, 3 * H:])
    c1 = f * c + i * gg
    return o * np.tanh(c1), c1


def lnlstm_cell(x, h, c, W, p):
    """src/layernormlstm.py:24-42 (LN on input/hidden gate pre-activations and on the cell)."""
    gi = layer_norm(x @ W[p + ".weight_ih"].T, W[p + ".ln_input.weight"], W[p + ".ln_input.bias"])
    gh = layer_norm(h @ W[p + ".weight_hh"].T, W[p + ".ln_hidden.weight"], W[p + ".ln_hidden.bias"])
    g = gi + gh + W[p + ".bias_ih"]
    H = h.shape[-1]
    i, f, gg, o = sigmoid(g[:, :H]), sigmoid(g[:, H:2 * H]), np.tanh(g[:, 2 * H:3 * H]), sigmoid(g[:, 3 * H:])
    c1 = layer_norm(f * c + i * gg, W[p + ".ln_cell.weight"], W[p + ".ln_cell.bias"])
    return o * np.tanh(c1), c1


def gru_cell(x, h, W, p):
    """torch.nn.GRUCell (gate order r, z, n)."""
    gi = linear(x, W[p + ".weight_ih"], W[p + ".bias_ih"])
    gh = linear(h, W[p + ".weight_hh"], W[p + ".bias_hh"])
    H = h.shape[-1]
    r = sigmoid(gi[:, :H] + gh[:, :H])
    z = sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = np.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return (1 - z) * n + z * h


def netmon_forward(W, x, adj, state, rnn="lstm", agg="sum", K=1, n_enc_layers=3, global_h=False, carryover=True,
                   act="leaky_relu", dtype=np.float64):
    """src/model.py:451-622 NetMon.forward with output_neighbor_hidden=True,
    no_agent_mapping=True; global_h adds the --netmon-global readout (mean of h over the
    graph's nodes after h, src/model.py:461-462, 624-627). carryover=False
    (--netmon-rnn-carryover 0, src/model.py:380-391, 536-570): the state is [obs-cell state |
    update-cell state] and the first update iteration continues from the stored update-cell
    state instead of the obs cell's output.

    x [B,N,F], adj [B,N,N] (I+A), state [B,N,S] or None.
    dtype np.float32 with float32 weights: the same formulas in fp32 arithmetic (what an fp32
    implementation of the reference, e.g. its own torch CPU run, computes), to measure fp32's own
    deviation from the fp64 result.
    Returns (out [B,N,4H] ([B,N,5H] with global_h), new_state [B,N,S])."""
    x = np.asarray(x, dtype)
    adj = np.asarray(adj, dtype)
    B, N, _ = x.shape
    H = W["rnn_obs.weight_hh"].shape[-1]
    nc = 1 if rnn == "gru" else 2  # tensors per cell state
    ns = nc * (1 if carryover else 2)
    if state is None:
        state = np.zeros((B, N, ns * H), dtype)
    st = np.asarray(state, dtype).reshape(B * N, ns, H)
    h = mlp(x.reshape(B * N, -1), W, "encode", n_enc_layers, act=act)
    c = None
    if rnn == "lstm":
        h, c = lstm_cell(h, st[:, 0], st[:, 1], W, "rnn_obs")
    elif rnn == "lnlstm":
        h, c = lnlstm_cell(h, st[:, 0], st[:, 1], W, "rnn_obs")
    else:
        h = gru_cell(h, st[:, 0], W, "rnn_obs")
    h0, c0 = h, c
    last_nbr = None
    for it in range(K):
        if it == K - 1:
            last_nbr = h
        M = np.einsum("bij,bjh->bih", adj, h.reshape(B, N, H))
        if agg == "mean":
            M = M / np.maximum(adj.sum(-1), 1)[..., None]
        M = M.reshape(B * N, H)
        hin, cin = h, c
        if not carryover and it == 0:
            hin, cin = st[:, nc], (st[:, nc + 1] if nc == 2 else None)
        if rnn == "lstm":
            h, c = lstm_cell(M, hin, cin, W, "rnn_update")
        elif rnn == "lnlstm":
            h, c = lnlstm_cell(M, hin, cin, W, "rnn_update")
        else:
            h = gru_cell(M, hin, W, "rnn_update")
    if carryover:
        new_state = (np.stack([h, c], 1) if nc == 2 else h).reshape(B, N, -1)
    elif nc == 2:
        new_state = np.stack([h0, c0, h, c], 1).reshape(B, N, -1)
    else:
        # gru without carry-over: the reference stacks (h0[None], h1[None]) into (2, 1, BN, H),
        # and transpose(0, 1) + reshape(B, N, 2H) keeps that component-major order
        # (src/model.py:566-567, 447-449): rows hold [h0 of all nodes | h1 of all nodes]
        new_state = np.concatenate([h0.reshape(-1), h.reshape(-1)]).reshape(B, N, 2 * H)
    # neighbour readout (src/model.py:582-622): neighbours in ascending node id order
    nb = last_nbr.reshape(B, N, H)
    eye = np.eye(N, dtype=bool)[None]
    mask = (adj > 0) & ~eye
    deg = int(mask.sum(-1).max())
    out_n = np.zeros((B, N, deg, H))
    for b in range(B):
        for i in range(N):
            js = np.nonzero(mask[b, i])[0]
            for k, j in enumerate(js):
                out_n[b, i, k] = nb[b, j]
    parts = [h.reshape(B, N, H)]
    if global_h:
        parts.append(np.repeat(h.reshape(B, N, H).mean(1, keepdims=True), N, 1))
    out = np.concatenate(parts + [out_n.reshape(B, N, deg * H)], -1)
    return out, new_state


def to_network_obs(out, node_agent):
    """src/model.py:629-631 output_to_network_obs."""
    return np.einsum("bna,bnf->baf", np.asarray(node_agent, np.float64), out)


def dqn_forward(W, obs, n_layers=2, act="leaky_relu"):
    """src/model.py:187-203 DQN: MLP encoder (activation on output) + linear Q head."""
    h = mlp(np.asarray(obs, np.float64), W, "encoder", n_layers, act=act)
    return linear(h, W["q_net.fc.weight"], W["q_net.fc.bias"])


def weights_from_npz(g, prefix):
    return {k[len(prefix):]: g[k].astype(np.float64) for k in g.files if k.startswith(prefix)}
