"""NumPy float64 restatement of the agent models DGN, DQNR and CommNet (reference
src/model.py:45-184 AttModel/DGN, 653-794 DQNR/CommNet). TEST INFRASTRUCTURE ONLY
(parity checker); pinned by tests/golden/models.npz (generated from the reference).

Weights: dict of numpy arrays keyed like the reference's state_dict.
"""
import numpy as np

from netmon_ref import leaky_relu, linear, lstm_cell, mlp  # noqa: F401


def n_mlp_layers(W, prefix):
    return len([k for k in W if k.startswith(prefix + ".linear_layers.") and k.endswith(".weight")])


def att_layer(W, p, h, adj, heads, dk=16, dv=16):
    """AttModel.forward (src/model.py:86-117): v/k/q = act(linear) per head, scores
    q k^T / sqrt(dk) (returned unmasked), masked_fill(adj == 0, -1e9), softmax, att v + v
    (skip connection), heads concatenated, act(fc_out)."""
    B, A, _ = h.shape
    v = leaky_relu(linear(h, W[p + ".fc_v.weight"], W[p + ".fc_v.bias"])).reshape(B, A, heads, dv).transpose(0, 2, 1, 3)
    q = leaky_relu(linear(h, W[p + ".fc_q.weight"], W[p + ".fc_q.bias"])).reshape(B, A, heads, dk).transpose(0, 2, 1, 3)
    k = leaky_relu(linear(h, W[p + ".fc_k.weight"], W[p + ".fc_k.bias"])).reshape(B, A, heads, dk).transpose(0, 2, 1, 3)
    w = q @ k.transpose(0, 1, 3, 2) * (1.0 / dk ** 0.5)
    att = np.where(adj[:, None] == 0, -1e9, w)
    att = np.exp(att - att.max(-1, keepdims=True))
    att = att / att.sum(-1, keepdims=True)
    out = att @ v + v
    out = out.transpose(0, 2, 1, 3).reshape(B, A, heads * dv)
    return leaky_relu(linear(out, W[p + ".fc_out.weight"], W[p + ".fc_out.bias"])), w


def dgn(W, x, adj, heads):
    """DGN.forward (src/model.py:163-176): Q on [h_enc | h_att1 | ... ]; returns (q, att weights)."""
    h = mlp(x, W, "encoder", n_mlp_layers(W, "encoder"))
    q_in, atts = [h], []
    li = 0
    while f"att_layers.{li}.fc_v.weight" in W:
        h, w = att_layer(W, f"att_layers.{li}", h, adj, heads)
        q_in.append(h)
        atts.append(w)
        li += 1
    return linear(np.concatenate(q_in, -1), W["q_net.fc.weight"], W["q_net.fc.bias"]), atts


def _cell(x, h, c, W):
    """lstm_cell on [B, A, .] arrays (rows flattened)."""
    B, A, H = h.shape
    h1, c1 = lstm_cell(x.reshape(B * A, -1), h.reshape(B * A, H), c.reshape(B * A, H), W, "lstm")
    return h1.reshape(B, A, H), c1.reshape(B, A, H)


def _split_state(state, B, A, H):
    if state is None:
        return np.zeros((B, A, H)), np.zeros((B, A, H))
    return state[..., :H], state[..., H:]


def dqnr(W, x, state):
    """DQNR.forward (src/model.py:741-744): encoder, LSTMCell with the carried agent
    state [h | c] per agent (zeros if None), Q head. Returns (q, new state)."""
    B, A, _ = x.shape
    h = mlp(x, W, "encoder", n_mlp_layers(W, "encoder"))
    H = W["lstm.weight_hh"].shape[1]
    hs, cs = _split_state(state, B, A, H)
    h, c = _cell(h, hs, cs, W)
    return linear(h, W["q_net.fc.weight"], W["q_net.fc.bias"]), np.concatenate([h, c], -1)


def commnet(W, x, adj, state, rounds=2):
    """CommNet.forward (src/model.py:766-794): LSTM on the encoding, then per round the
    hidden states of the other agents in the mask are averaged (self excluded, count
    clamped to 1), added to h, and h is both input and hidden of the next LSTM step."""
    B, A, _ = x.shape
    h = mlp(x, W, "encoder", n_mlp_layers(W, "encoder"))
    H = W["lstm.weight_hh"].shape[1]
    hs, cs = _split_state(state, B, A, H)
    h, c = _cell(h, hs, cs, W)
    mask = adj * (1.0 - np.eye(A))[None]
    cnt = np.maximum(mask.sum(-1, keepdims=True), 1.0)
    for _ in range(rounds):
        h = h + (mask @ h) / cnt
        h, c = _cell(h, h, c, W)
    return linear(h, W["q_net.fc.weight"], W["q_net.fc.bias"]), np.concatenate([h, c], -1)
