import importlib, sys, numpy as np, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle")
import netmon_ref
gm = importlib.import_module("graph-marl_amd"); M = importlib.import_module("graph-marl_amd.model")
FU = importlib.import_module("graph-marl_amd.fused"); L = gm._lib
N, A, B = 20, 20, 64
for form in ("x3", "f32"):
    L.GEMM_MODE = form
    env = gm.Routing(gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS), A, n_env=B, seed=5, obs_extra=512, agent_adjacency=False)
    torch.manual_seed(1)
    nm = M.NetMon(4 * N + 8, 128, [512, 256], 1, rnn_type="lnlstm").cuda()
    env.reset_()
    Wn = {k: v.detach().double().cpu().numpy() for k, v in nm.state_dict().items()}
    adj = env.get_nodes_adjacency().float().cpu().numpy()
    x = env.node_obs
    st0 = torch.randn(B, N, 256, device="cuda") * 0.5
    with torch.no_grad():
        sf, _ = FU.netmon_step(nm, x, env.nbr, st0.clone())
        sf = sf.clone()
        nm.state = st0.clone()
        nm.forward_graph(x, env.nbr, env.agent_node)
        su = nm.state.clone()
    _, s64 = netmon_ref.netmon_forward(Wn, x.cpu().numpy(), adj, st0.cpu().numpy(), "lnlstm", "sum", 1)
    print(form, "fused vs fp64", np.abs(sf.cpu().numpy() - s64).max(), "unfused vs fp64", np.abs(su.cpu().numpy() - s64).max(),
          "fused vs unfused", (sf - su).abs().max().item())
