"""GPU parity for the NetMon / DQN kernels: each HIP op vs a torch fp32 reference
of the same op, and full NetMon / DQN forward vs the reference's golden outputs.
Tolerance (north star): 1e-5 absolute on GNN/LSTM float outputs."""
import importlib
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import golden_replay as R

pytestmark = pytest.mark.gpu
ATOL = 1e-5


def lib():
    return importlib.import_module("graph-marl_amd._lib")


def model_mod():
    return importlib.import_module("graph-marl_amd.model")


def random_graphs(G, N, deg=3, seed=0):
    """random symmetric 3-regular-ish neighbour tables via the env's own generator"""
    gm = importlib.import_module("graph-marl_amd")
    env = gm.Routing(gm.Network(N, random_topology=True), 4, n_env=G, seed=seed, agent_adjacency=False)
    env.reset_()
    return env.nbr.clone(), env


def dense_adj(nbr, N):
    G = nbr.shape[0]
    m = torch.eye(N, device=nbr.device).repeat(G, 1, 1)
    for k in range(nbr.shape[-1]):
        m.scatter_(2, nbr[..., k:k + 1].long(), 1.0)
    return m


@pytest.mark.parametrize("mode", [0, 1])
def test_mp_aggregate_rows_strided(mode):
    """gm_mp_aggregate_rows on the h half of [h | c] state rows into a strided output equals the
    contiguous gm_mp_aggregate bit for bit (same member order)."""
    M = model_mod()
    L = M.L
    G, N, H = 64, 20, 128
    nbr, _ = random_graphs(G, N)
    st = torch.randn(G * N, 2 * H, device="cuda")
    out = torch.full((G * N, H + 4), float("nan"), device="cuda")
    L.check(L.lib().gm_mp_aggregate_rows(st.data_ptr(), 2 * H, nbr.data_ptr(), G, N, nbr.shape[-1], H, mode,
                                         out.data_ptr(), H + 4, L.stream_ptr()))
    ref = M.mp_aggregate(st[:, :H].contiguous(), nbr, mode)
    assert torch.equal(out[:, :H], ref)
    assert torch.isnan(out[:, H:]).all()  # nothing written past the row's H columns


@pytest.mark.parametrize("mode", [0, 1])
def test_mp_aggregate_fwd_bwd(mode):
    M = model_mod()
    G, N, H = 64, 20, 128
    nbr, _ = random_graphs(G, N)
    h = torch.randn(G * N, H, device="cuda", requires_grad=True)
    out = M.mp_aggregate(h, nbr, mode)
    adj = dense_adj(nbr, N)
    ref = torch.bmm(adj, h.detach().view(G, N, H))
    if mode == 1:
        ref = ref / adj.sum(-1, keepdim=True).clamp(min=1)
    torch.testing.assert_close(out.view(G, N, H), ref, atol=ATOL, rtol=0)
    g = torch.randn_like(out)
    out.backward(g)
    h2 = h.detach().clone().requires_grad_(True)
    r2 = torch.bmm(adj, h2.view(G, N, H))
    if mode == 1:
        r2 = r2 / adj.sum(-1, keepdim=True).clamp(min=1)
    r2.backward(g.view(G, N, H))
    torch.testing.assert_close(h.grad, h2.grad, atol=ATOL, rtol=0)


@pytest.mark.parametrize("G,N,A", [(32, 20, 20), (16, 100, None), (8, 128, None), (8, 64, None), (12, 40, 64)])
def test_readout_fwd_bwd_with_agent_map(G, N, A):
    """A = None: every node reads out (no agent map, the SL task: up to 128 rows per graph in the
    bitmask backward)."""
    M = model_mod()
    H = 128
    nbr, _ = random_graphs(G, N, seed=3)
    hf = torch.randn(G * N, H, device="cuda", requires_grad=True)
    hp = torch.randn(G * N, H, device="cuda", requires_grad=True)
    if A is None:
        A = N
        an = torch.arange(N, device="cuda", dtype=torch.int32).repeat(G, 1)
        out = M.netmon_readout(hf, hp, nbr, None).view(G, A, 4 * H)
    else:
        an = torch.randint(0, N, (G, A), device="cuda", dtype=torch.int32)
        out = None
    if out is None:
        out = M.netmon_readout(hf, hp, nbr, an).view(G, A, 4 * H)
    nb = hp.detach().view(G, N, H)
    parts = [torch.gather(hf.detach().view(G, N, H), 1, an.long().unsqueeze(-1).expand(-1, -1, H))]
    for k in range(3):
        idx = torch.gather(nbr[..., k], 1, an.long())
        parts.append(torch.gather(nb, 1, idx.long().unsqueeze(-1).expand(-1, -1, H)))
    ref = torch.cat(parts, -1)
    torch.testing.assert_close(out, ref, atol=0, rtol=0)
    g = torch.randn_like(out)
    out.backward(g)
    hf2, hp2 = hf.detach().clone().requires_grad_(True), hp.detach().clone().requires_grad_(True)
    parts = [torch.gather(hf2.view(G, N, H), 1, an.long().unsqueeze(-1).expand(-1, -1, H))]
    for k in range(3):
        idx = torch.gather(nbr[..., k], 1, an.long())
        parts.append(torch.gather(hp2.view(G, N, H), 1, idx.long().unsqueeze(-1).expand(-1, -1, H)))
    torch.cat(parts, -1).backward(g)
    torch.testing.assert_close(hf.grad, hf2.grad, atol=ATOL, rtol=0)
    torch.testing.assert_close(hp.grad, hp2.grad, atol=ATOL, rtol=0)


def test_lstm_pointwise_fwd_bwd():
    M = model_mod()
    m, H = 4096, 128
    gates = torch.randn(m, 4 * H, device="cuda", requires_grad=True)
    c = torch.randn(m, H, device="cuda", requires_grad=True)
    h1, c1 = M._LSTMPointwise.apply(gates, c)
    g2, cc = gates.detach().clone().requires_grad_(True), c.detach().clone().requires_grad_(True)
    i, f, gg, o = g2.chunk(4, 1)
    rc = torch.sigmoid(f) * cc + torch.sigmoid(i) * torch.tanh(gg)
    rh = torch.sigmoid(o) * torch.tanh(rc)
    torch.testing.assert_close(h1, rh, atol=ATOL, rtol=0)
    torch.testing.assert_close(c1, rc, atol=ATOL, rtol=0)
    a, b = torch.randn_like(h1), torch.randn_like(c1)
    (h1 * a + c1 * b).sum().backward()
    (rh * a + rc * b).sum().backward()
    torch.testing.assert_close(gates.grad, g2.grad, atol=ATOL, rtol=0)
    torch.testing.assert_close(c.grad, cc.grad, atol=ATOL, rtol=0)


@pytest.mark.parametrize("shape", [(81920, 512, 88), (4096, 512, 642), (1000, 256, 512), (777, 128, 256),
                                   (81920, 4, 256), (33, 40, 30), (5, 3, 7)])
@pytest.mark.parametrize("act", [0, 1])
def test_linear_f32_vs_torch(shape, act):
    M = model_mod()
    m, n, k = shape
    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device="cuda")
    w = torch.randn(n, k, device="cuda") / k ** 0.5
    b = torch.randn(n, device="cuda")
    lin = M.Linear(k, n, act=act).cuda()
    with torch.no_grad():
        lin.weight.copy_(w)
        lin.bias.copy_(b)
        y = lin(x)
    ref = torch.nn.functional.linear(x.double(), w.double(), b.double())
    if act:
        ref = F.leaky_relu(ref)
    err = (y.double() - ref).abs().max().item()
    assert err < 2e-5 * max(1.0, k ** 0.5 / 8), err


def test_linear_strided_rows_and_grad():
    """rows inside a wider buffer (the joint observation layout) + autograd."""
    M = model_mod()
    buf = torch.zeros(2048, 644, device="cuda")
    buf[:, :642] = torch.randn(2048, 642, device="cuda")
    lin = M.Linear(642, 512, act=1).cuda()
    x = buf[:, :642]
    y = lin(x)
    ref = F.leaky_relu(F.linear(x, lin.weight, lin.bias))
    torch.testing.assert_close(y, ref, atol=1e-4, rtol=1e-5)
    xr = torch.randn(300, 642, device="cuda", requires_grad=True)
    y = lin(xr)
    y.pow(2).sum().backward()
    gw, gx = lin.weight.grad.clone(), xr.grad.clone()
    lin.weight.grad = None
    xr2 = xr.detach().clone().requires_grad_(True)
    F.leaky_relu(F.linear(xr2, lin.weight, lin.bias)).pow(2).sum().backward()
    torch.testing.assert_close(gw, lin.weight.grad, atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(gx, xr2.grad, atol=1e-4, rtol=1e-4)


def _load(module, g, prefix):
    sd = {k[len(prefix):]: torch.as_tensor(g[k]) for k in g.files if k.startswith(prefix)}
    missing, unexpected = module.load_state_dict(sd, strict=True), None
    return module


@pytest.mark.parametrize("vi", range(6))
def test_netmon_forward_vs_reference_golden(vi):
    M = model_mod()
    g = np.load(f"{R.GOLDEN}/netmon.npz")
    rnn, agg, K, H, enc = g["variants"][vi].split("|")
    enc = [int(e) for e in enc.split(",")]
    nm = M.NetMon(g["node_obs"].shape[-1], int(H), enc, int(K), rnn_type=rnn, agg_type=agg).cuda()
    _load(nm, g, f"v{vi}_w_")
    nm.state = None
    with torch.no_grad():
        for t in range(3):
            x = torch.as_tensor(g["node_obs"][t], device="cuda")
            m = torch.as_tensor(g["node_adj"][t], device="cuda")
            na = torch.as_tensor(g["node_agent"][t], device="cuda")
            h = nm(x, m, na, no_agent_mapping=True)
            np.testing.assert_allclose(h.cpu().numpy(), g[f"v{vi}_h_{t}"], atol=ATOL, rtol=0)
            np.testing.assert_allclose(nm.state.cpu().numpy(), g[f"v{vi}_state_{t}"], atol=ATOL, rtol=0)
            mapped = M.NetMon.output_to_network_obs(h, na)
            np.testing.assert_allclose(mapped.cpu().numpy(), g[f"v{vi}_mapped_{t}"], atol=ATOL, rtol=0)


def test_netmon_fast_path_matches_dense_api():
    """forward_graph with (nbr, agent_node) == forward with the reference's dense inputs."""
    M = model_mod()
    G, N, A = 64, 20, 20
    nbr, env = random_graphs(G, N, seed=11)
    torch.manual_seed(0)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1).cuda()
    x = torch.rand(G, N, 4 * N + 8, device="cuda")
    an = torch.randint(0, N, (G, A), device="cuda", dtype=torch.int32)
    na = torch.zeros(G, N, A, device="cuda").scatter_(1, an.long().unsqueeze(1), 1.0)
    with torch.no_grad():
        nm.state = None
        a = nm.forward_graph(x, nbr, an)
        nm.state = None
        b = nm(x, dense_adj(nbr, N), na)
    torch.testing.assert_close(a, b, atol=0, rtol=0)


def test_dqn_forward_vs_reference_golden():
    M = model_mod()
    g = np.load(f"{R.GOLDEN}/netmon.npz")
    obs = torch.as_tensor(g["dqn_obs"], device="cuda")
    dqn = M.DQN(obs.shape[-1], [512, 256], 4).cuda()
    _load(dqn, g, "dqn_w_")
    with torch.no_grad():
        q = dqn(obs)
    np.testing.assert_allclose(q.cpu().numpy(), g["dqn_q"], atol=ATOL, rtol=0)


def test_netmon_global_readout_vs_reference_golden():
    """--netmon-global (src/model.py:458-469, 624-627): [h | node mean of h | neighbour h]
    mapped to agents, over 3 steps with carried state, vs the reference."""
    import importlib

    import numpy as np
    import torch

    M = importlib.import_module("graph-marl_amd.model")
    g = np.load(os.path.join(R.GOLDEN, "netmon_global.npz"))
    for vi, K in enumerate((1, 2)):
        nm = M.NetMon(g["node_obs"].shape[-1], 32, [64, 48], K, output_global_hidden=True).cuda()
        nm.load_state_dict({k[len(f"v{vi}_w_"):]: torch.as_tensor(g[k]) for k in g.files if k.startswith(f"v{vi}_w_")})
        assert nm.get_out_features() == int(g[f"v{vi}_out_features"])
        nm.state = None
        for t in range(3):
            with torch.no_grad():
                mapped = nm(torch.as_tensor(g["node_obs"][t], device="cuda"),
                            torch.as_tensor(g["node_adj"][t], device="cuda"),
                            torch.as_tensor(g["node_agent"][t], device="cuda"))
            np.testing.assert_allclose(mapped.cpu().numpy(), g[f"v{vi}_mapped_{t}"], atol=1e-5, rtol=0)
            np.testing.assert_allclose(nm.state.cpu().numpy(), g[f"v{vi}_state_{t}"], atol=1e-5, rtol=0)


def test_netmon_no_carryover_vs_reference_golden():
    """--netmon-rnn-carryover 0 (src/model.py:380-391, 536-570) for lstm / lnlstm / gru, K = 1, 2:
    agent-mapped readout and the doubled state (incl. the reference's component-major gru
    layout) over 3 carried steps vs the reference; the NetMon wrapper takes the unfused path."""
    import importlib

    import numpy as np
    import torch

    M = importlib.import_module("graph-marl_amd.model")
    g = np.load(os.path.join(R.GOLDEN, "netmon_nocarry.npz"))
    for vi, v in enumerate(g["variants"]):
        rnn, K = str(v).split(":")
        nm = M.NetMon(g["node_obs"].shape[-1], 32, [64, 48], int(K), rnn_type=rnn, rnn_carryover=False).cuda()
        nm.load_state_dict({k[len(f"v{vi}_w_"):]: torch.as_tensor(g[k]) for k in g.files if k.startswith(f"v{vi}_w_")})
        assert nm.get_state_size() == int(g[f"v{vi}_state_size"])
        nm.state = None
        for t in range(3):
            with torch.no_grad():
                mapped = nm(torch.as_tensor(g["node_obs"][t], device="cuda"),
                            torch.as_tensor(g["node_adj"][t], device="cuda"),
                            torch.as_tensor(g["node_agent"][t], device="cuda"))
            np.testing.assert_allclose(mapped.cpu().numpy(), g[f"v{vi}_mapped_{t}"], atol=1e-5, rtol=0)
            np.testing.assert_allclose(nm.state.cpu().numpy(), g[f"v{vi}_state_{t}"], atol=1e-5, rtol=0)


@pytest.mark.parametrize("mode", [0, 1])
def test_mp_aggregate_degree3_missing_neighbours(mode):
    """The degree-3 aggregate kernel (round 5: members in ascending id order by a sorting network) with
    neighbour tables as dense_to_nbr writes them for graphs of degree <= 3 (ascending ids, -1 padding):
    bit for bit the fp32 sum over {n} u nbr(n) in ascending id order (the reference bmm's (I + A) order),
    divided by the member count for mean."""
    M = model_mod()
    G, N, H = 16, 20, 128
    g = torch.Generator().manual_seed(mode)
    adj = torch.zeros(G, N, N, dtype=torch.int8)
    for b in range(G):
        for n in range(N):
            k = int(torch.randint(0, 4, (1,), generator=g))
            for v in torch.randperm(N, generator=g)[:k].tolist():
                if v != n:
                    adj[b, n, v] = 1
    nbr = torch.full((G, N, 3), -1, dtype=torch.int32)
    for b in range(G):
        for n in range(N):
            ids = torch.nonzero(adj[b, n]).flatten()[:3]
            nbr[b, n, :len(ids)] = ids.int()
    nbr = nbr.cuda()
    h = torch.randn(G * N, H, device="cuda")
    out = M.mp_aggregate(h, nbr, mode)
    hv = h.view(G, N, H)
    ref = torch.empty_like(hv)
    for b in range(G):
        for n in range(N):
            mem = sorted([n] + [v for v in nbr[b, n].tolist() if v >= 0])
            acc = hv[b, mem[0]].clone()
            for v in mem[1:]:
                acc = acc + hv[b, v]
            # tensor divisor: torch divides by a Python scalar as a multiply by its reciprocal on the GPU
            ref[b, n] = acc / torch.full_like(acc, float(len(mem))) if mode == 1 else acc
    assert torch.equal(out.view(G, N, H), ref)
