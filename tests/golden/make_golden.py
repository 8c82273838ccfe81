#!/usr/bin/env python3
"""Generate golden vectors by importing the *reference* implementation.

This script runs ONLY in the build container (where /root/reference exists). It
imports the reference's Python modules (read-only, never copied) and records
inputs/outputs as small .npz fixtures under tests/golden/. The fixtures are data
(inputs and expected outputs); the reference source itself never ships.

Missing third-party packages that the reference imports but never calls on the
hot path (gymnasium.spaces.Discrete, torch_geometric names, tensorboard) are
replaced by tiny stubs written to a temporary directory.

Usage:  python tests/golden/make_golden.py [--ref /root/reference/src]
"""
import argparse
import copy
import hashlib
import os
import sys
import tempfile
import textwrap

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import detparams  # noqa: E402


def write_stubs(root):
    files = {
        "gymnasium/__init__.py": "",
        "gymnasium/spaces.py": textwrap.dedent(
            """
            import numpy as np
            class Discrete:
                def __init__(self, n, start=0):
                    self.n = n
                    self.start = start
                def sample(self):
                    return self.start + np.random.randint(self.n)
            """
        ),
        "torch_geometric/__init__.py": "",
        "torch_geometric/nn/__init__.py": textwrap.dedent(
            """
            class _Missing:
                def __init__(self, *a, **k):
                    raise ImportError("torch_geometric is not installed")
            GCNConv = SAGEConv = AntiSymmetricConv = GraphSAGE = _Missing
            """
        ),
        "torch_geometric/nn/summary.py": "def summary(model, *a, **k):\n    return 'summary'\n",
        "torch_geometric/utils/__init__.py": textwrap.dedent(
            """
            def dense_to_sparse(*a, **k):
                raise ImportError("torch_geometric is not installed")
            """
        ),
    }
    for rel, txt in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(txt)


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---------------------------------------------------------------------------
# RNG goldens (numpy legacy MT19937 as the reference uses it)
# ---------------------------------------------------------------------------
def gen_rng(out):
    seeds = [0, 1, 42, 476, 923430603, 2**32 - 1]
    d = {"seeds": np.array(seeds, dtype=np.uint64)}
    for s in seeds:
        rs = np.random.RandomState(s)
        d[f"key_{s}"] = rs.get_state()[1].astype(np.uint32)
        rs = np.random.RandomState(s)
        d[f"raw_{s}"] = rs.randint(0, 2**32, size=1500, dtype=np.uint64).astype(np.uint32)
        rs = np.random.RandomState(s)
        # the exact call pattern of Routing.reset_packet for N=20
        mix = []
        for _ in range(100):
            mix.append(float(rs.randint(20)))
            mix.append(float(rs.randint(20)))
            mix.append(rs.random())
        d[f"packet20_{s}"] = np.array(mix, dtype=np.float64)
        rs = np.random.RandomState(s)
        d[f"randint31_{s}"] = np.array([rs.randint(2**31 - 1) for _ in range(64)], dtype=np.int64)
        rs = np.random.RandomState(s)
        eg = []
        for _ in range(40):
            eg.append(rs.randint(4, size=20).astype(np.float64))
            eg.append(rs.rand(20))
        d[f"egreedy_{s}"] = np.stack(eg)
        rs = np.random.RandomState(s)
        d[f"randint_n_{s}"] = np.array(
            [rs.randint(n) for n in [1, 2, 3, 5, 7, 10, 13, 20, 33, 50, 64, 100, 1000] * 20],
            dtype=np.int64,
        )
    np.savez_compressed(out, **d)


# ---------------------------------------------------------------------------
# Topology goldens
# ---------------------------------------------------------------------------
def topo_record(net):
    n = net.n_nodes
    pos = np.array([[nd.x, nd.y] for nd in net.nodes], dtype=np.float64)
    edges = np.array([[e.start, e.end, e.length] for e in net.edges], dtype=np.int64)
    node_edges = np.array([nd.edges for nd in net.nodes], dtype=np.int64)
    neighbors = np.array([nd.neighbors for nd in net.nodes], dtype=np.int64)
    apsp = np.array(
        [[net.shortest_paths_weights[i][j] for j in range(n)] for i in range(n)], dtype=np.int64
    )
    return dict(
        seed=int(net.current_topology_seed),
        repetitions=int(net.repetitions),
        pos=pos,
        edges=edges,
        node_edges=node_edges,
        neighbors=neighbors,
        apsp=apsp,
        adj=net.adj_matrix.astype(np.int8),
    )


def gen_topology(out, Network, EVAL_SEEDS):
    d = {}
    # random topologies drawn through the main stream (training path), EVAL_SEEDS excluded
    for n, main_seed, count in [(10, 11, 24), (20, 12, 24), (30, 13, 12), (40, 14, 12), (50, 15, 12), (100, 16, 6)]:
        np.random.seed(main_seed)
        net = Network(n_nodes=n, random_topology=True, excluded_seeds=EVAL_SEEDS)
        recs = []
        for _ in range(count):
            net.reset()
            recs.append(topo_record(net))
        # main stream position after the resets: next raw draws
        post = np.random.randint(0, 2**32, size=4, dtype=np.uint64).astype(np.uint32)
        key = f"rand_n{n}"
        d[key + "_main_seed"] = np.int64(main_seed)
        d[key + "_post_raw"] = post
        for k in ["seed", "repetitions"]:
            d[key + "_" + k] = np.array([r[k] for r in recs], dtype=np.int64)
        for k in ["pos", "edges", "node_edges", "neighbors", "apsp", "adj"]:
            d[key + "_" + k] = np.stack([r[k] for r in recs])
    # fixed seeds
    for s in [476, 923430603] + list(EVAL_SEEDS[:30]):
        net = Network(n_nodes=20, random_topology=False, topology_init_seed=s)
        np.random.seed(0)
        net.reset()
        r = topo_record(net)
        for k, v in r.items():
            d[f"fixed_{s}_{k}"] = np.asarray(v)
    d["fixed_seeds"] = np.array([476, 923430603] + list(EVAL_SEEDS[:30]), dtype=np.int64)
    # build_seed_list (used for --num-topologies-train and EVAL_SEEDS)
    for n, init, cnt in [(20, 476, 40), (20, 1234, 16), (10, 99, 16), (50, 7, 8)]:
        net = Network(n_nodes=n, random_topology=True, n_random_seeds=cnt, topology_init_seed=init)
        d[f"seedlist_n{n}_i{init}"] = np.array(net.seeds, dtype=np.int64)
    np.savez_compressed(out, **d)


# ---------------------------------------------------------------------------
# Environment traces
# ---------------------------------------------------------------------------
ENV_CONFIGS = [
    # name, n_nodes, n_data, topology mode, topo arg, congestion, action mask, ttl, env seed, steps, episode steps, egreedy eps (None = tape)
    dict(name="fixed476", n=20, a=20, mode="fixed", topo=476, cong=True, mask=False, ttl=0, seed=0, T=300, ep=300, eps=None),
    dict(name="fixed923", n=20, a=20, mode="fixed", topo=923430603, cong=True, mask=False, ttl=0, seed=7, T=300, ep=300, eps=None),
    dict(name="rand20", n=20, a=20, mode="random", topo=476, cong=True, mask=False, ttl=0, seed=3, T=200, ep=50, eps=None),
    dict(name="rand10_nocong", n=10, a=30, mode="random", topo=476, cong=False, mask=False, ttl=0, seed=5, T=150, ep=50, eps=None),
    dict(name="rand50", n=50, a=20, mode="random", topo=476, cong=True, mask=False, ttl=0, seed=9, T=100, ep=50, eps=None),
    dict(name="fixed476_ttl_mask", n=20, a=20, mode="fixed", topo=476, cong=True, mask=True, ttl=10, seed=1, T=200, ep=100, eps=None),
    dict(name="list5", n=20, a=20, mode="list", topo=1234, cong=True, mask=False, ttl=0, seed=2, T=120, ep=20, eps=None),
    dict(name="evalseq", n=20, a=20, mode="sequential", topo=476, cong=True, mask=False, ttl=0, seed=4, T=100, ep=20, eps=None),
    dict(name="egreedy_rand20", n=20, a=20, mode="random", topo=476, cong=True, mask=False, ttl=0, seed=11, T=150, ep=50, eps=0.3),
    dict(name="fixed476_a1", n=20, a=1, mode="fixed", topo=476, cong=True, mask=False, ttl=0, seed=13, T=60, ep=60, eps=None),
    # observation variants 2 (k neighbours) and 3 (global), src/env/routing.py:268-358
    dict(name="fixed476_var2", n=20, a=20, mode="fixed", topo=476, cong=True, mask=False, ttl=0, seed=17, T=80, ep=40, eps=None, var=2),
    dict(name="rand10_var3", n=10, a=12, mode="random", topo=476, cong=True, mask=False, ttl=0, seed=19, T=60, ep=20, eps=None, var=3),
]
FULL_STEPS = (0, 1, 2, 3, 26, 52)  # snapshot indices with full arrays


def gen_env(out_dir, Network, Routing, EVAL_SEEDS, names=None):
    """Per config: a snapshot stream. Snapshot 0 is the initial reset; then every
    env.step(t) appends a snapshot, and an episode reset (episode_steps reached)
    appends another snapshot with kind=1 right after the step's snapshot."""
    for cfg in ENV_CONFIGS:
        if names and cfg["name"] not in names:
            continue
        n, a = cfg["n"], cfg["a"]
        if cfg["mode"] == "fixed":
            net = Network(n_nodes=n, random_topology=False, topology_init_seed=cfg["topo"])
        elif cfg["mode"] == "random":
            net = Network(n_nodes=n, random_topology=True, topology_init_seed=cfg["topo"], excluded_seeds=EVAL_SEEDS)
        elif cfg["mode"] == "list":
            net = Network(n_nodes=n, random_topology=True, n_random_seeds=5, topology_init_seed=cfg["topo"], excluded_seeds=EVAL_SEEDS)
        elif cfg["mode"] == "sequential":
            net = Network(n_nodes=n, random_topology=True, provided_seeds=list(EVAL_SEEDS[:8]), sequential_topology_seeds=True)
        else:
            raise ValueError(cfg["mode"])
        env = Routing(net, a, cfg.get("var", 1), enable_congestion=cfg["cong"], enable_action_mask=cfg["mask"],
                      ttl=cfg["ttl"])
        tape_rng = np.random.RandomState(1000 + cfg["seed"])
        np.random.seed(cfg["seed"])
        snap_keys = ["kind", "step", "now", "target", "edge", "time", "ttl", "size", "start", "spw", "visited",
                     "agent_steps", "loads", "topo_seed", "action_mask", "obs_sha", "nodeobs_sha", "adj_sha",
                     "nodeagent_sha"]
        step_keys = ["reward", "done", "actions", "q", "info_looped", "info_throughput", "info_dropped",
                     "info_blocked", "info_ndelays", "info_narrived"]
        rec = {k: [] for k in snap_keys + step_keys}
        lists = {"delays": [], "delays_arrived": [], "spr": []}
        full = {}
        topo = []
        final_info = []

        def snap(kind, t, obs, adj):
            E = len(env.network.edges)
            si = len(rec["kind"])
            rec["kind"].append(kind)
            rec["step"].append(t)
            rec["now"].append([p.now for p in env.data])
            rec["target"].append([p.target for p in env.data])
            rec["edge"].append([p.edge for p in env.data])
            rec["time"].append([p.time for p in env.data])
            rec["ttl"].append([p.ttl for p in env.data])
            rec["size"].append([p.size for p in env.data])
            rec["start"].append([p.start for p in env.data])
            rec["spw"].append([p.shortest_path_weight for p in env.data])
            rec["visited"].append([sum(1 << v for v in p.visited_nodes) for p in env.data])
            rec["agent_steps"].append(env.agent_steps.copy())
            loads = np.zeros(3 * n // 2, dtype=np.float64)
            loads[:E] = [float(e.load) for e in env.network.edges]
            rec["loads"].append(loads)
            rec["topo_seed"].append(int(env.network.current_topology_seed))
            rec["action_mask"].append(env.action_mask.astype(np.int8).copy())
            nobs = env.get_node_observation()
            nagent = env.get_node_agent_matrix()
            rec["obs_sha"].append(sha(obs.astype(np.float32)))
            rec["nodeobs_sha"].append(sha(nobs.astype(np.float32)))
            rec["adj_sha"].append(sha(adj.astype(np.int8)))
            rec["nodeagent_sha"].append(sha(nagent.astype(np.int8)))
            if si in FULL_STEPS:
                full[f"obs_{si}"] = obs.astype(np.float32)
                full[f"nodeobs_{si}"] = nobs.astype(np.float32)
                full[f"adj_{si}"] = adj.astype(np.int8)
                full[f"nodeagent_{si}"] = nagent.astype(np.int8)
            if kind == 1:
                r = topo_record(env.network)
                r["aux"] = env.get_node_aux()
                topo.append(r)

        obs, adj = env.reset()
        snap(1, 0, obs, adj)
        ep_step = 0
        for t in range(1, cfg["T"] + 1):
            if cfg["eps"] is None:
                act = tape_rng.randint(4, size=a)
                q = np.zeros((a, 4), dtype=np.float32)
            else:
                q = tape_rng.standard_normal((a, 4)).astype(np.float32)
                ra = np.random.randint(4, size=a)
                rf = np.random.rand(a) < cfg["eps"]
                act = np.argmax(q, axis=-1) * ~rf + rf * ra
            rec["q"].append(q)
            rec["actions"].append(np.asarray(act, dtype=np.int64))
            obs, adj, reward, done, info = env.step(act)
            rec["reward"].append(reward.copy())
            rec["done"].append(done.astype(np.int8))
            rec["info_looped"].append(float(info["looped"]))
            rec["info_throughput"].append(int(info["throughput"]))
            rec["info_dropped"].append(int(info["dropped"]))
            rec["info_blocked"].append(int(info["blocked"]))
            rec["info_ndelays"].append(len(info["delays"]))
            rec["info_narrived"].append(len(info["delays_arrived"]))
            for k in lists:
                lists[k].extend([float(x) for x in info[k]])
            snap(0, t, obs, adj)
            ep_step += 1
            if ep_step >= cfg["ep"]:
                fi = env.get_final_info({"delays": []})
                final_info.append([float(x) for x in fi["delays"]] + [-1.0])
                obs, adj = env.reset()
                ep_step = 0
                snap(1, t, obs, adj)

        d = {}
        for k, v in rec.items():
            if k.endswith("_sha"):
                d[k] = np.array(v)
            elif k == "visited":
                d[k] = np.array(v, dtype=np.uint64)
            elif k in ("size", "loads", "agent_steps", "info_looped"):
                d[k] = np.array(v, dtype=np.float64)
            elif k in ("reward", "q"):
                d[k] = np.array(v, dtype=np.float32)
            else:
                d[k] = np.array(v, dtype=np.int64)
        for k, v in lists.items():
            d["list_" + k] = np.array(v, dtype=np.float64)
        d["final_delays"] = np.array(sum(final_info, []), dtype=np.float64)
        for k, v in full.items():
            d["full_" + k] = v
        for i, r in enumerate(topo):
            for k in ["seed", "edges", "node_edges", "apsp", "adj", "aux"]:
                d[f"topo{i}_{k}"] = np.asarray(r[k])
        d["n_topo"] = np.int64(len(topo))
        for k, v in cfg.items():
            d[f"cfg_{k}"] = np.array(-1 if v is None else v)
        np.savez_compressed(os.path.join(out_dir, f"env_{cfg['name']}.npz"), **d)
        print("env", cfg["name"], "done", flush=True)


# ---------------------------------------------------------------------------
# NetMon / DQN / training-step goldens
# ---------------------------------------------------------------------------
def collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, steps, seed, aux=None):
    """node obs / adj / node-agent for B independent envs over `steps` consecutive steps
    (aux: a list that receives get_node_aux() per step, src/env/routing.py:237-254)."""
    obs_l, adj_l, na_l, aobs_l = [], [], [], []
    rng = np.random.RandomState(seed + 77)
    envs = []
    for b in range(B):
        np.random.seed(seed + b)
        net = Network(n_nodes=n, random_topology=True, excluded_seeds=EVAL_SEEDS)
        env = Routing(net, a, 1)
        env.reset()
        envs.append(env)
    for t in range(steps):
        o, ad, na, ao = [], [], [], []
        for env in envs:
            o.append(env.get_node_observation())
            ad.append(env.get_nodes_adjacency().astype(np.float32))
            na.append(env.get_node_agent_matrix().astype(np.float32))
            ao.append(env._get_observation())
            if aux is not None:
                aux.append(np.asarray(env.get_node_aux(), np.float32))
            env.step(rng.randint(4, size=a))
        obs_l.append(np.stack(o))
        adj_l.append(np.stack(ad))
        na_l.append(np.stack(na))
        aobs_l.append(np.stack(ao))
    return np.stack(obs_l), np.stack(adj_l), np.stack(na_l), np.stack(aobs_l)


def sd_to_npz(prefix, sd, d):
    for k, v in sd.items():
        d[f"{prefix}{k}"] = v.detach().cpu().numpy().copy()  # copy: params are updated in place later


def gen_netmon(out, Network, Routing, EVAL_SEEDS, NetMon, DQN):
    import torch
    import torch.nn.functional as F

    d = {}
    n, a, B, steps = 20, 20, 4, 3
    node_obs, node_adj, node_agent, agent_obs = collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, steps, 100)
    d["node_obs"], d["node_adj"], d["node_agent"], d["agent_obs"] = node_obs, node_adj, node_agent, agent_obs
    # variant 0 is the production configuration (H=128, encoder 512,256); the rest use
    # small dimensions to keep the fixture small (the kernels are dimension-generic)
    variants = [
        ("lstm", "sum", 1, 128, (512, 256)), ("lstm", "sum", 3, 32, (64, 48)),
        ("lstm", "mean", 2, 32, (64, 48)), ("lnlstm", "sum", 1, 32, (64, 48)),
        ("lnlstm", "mean", 3, 32, (64, 48)), ("gru", "sum", 2, 32, (64, 48)),
    ]
    d["variants"] = np.array([f"{r}|{g}|{k}|{h}|{e[0]},{e[1]}" for r, g, k, h, e in variants])
    for vi, (rnn, agg, K, H, enc) in enumerate(variants):
        torch.manual_seed(vi)
        nm = NetMon(node_obs.shape[-1], H, list(enc), K, F.leaky_relu, rnn_type=rnn,
                    rnn_carryover=True, agg_type=agg, output_neighbor_hidden=True,
                    output_global_hidden=False)
        nm.eval()
        sd_to_npz(f"v{vi}_w_", nm.state_dict(), d)
        nm.state = None
        with torch.no_grad():
            for t in range(steps):
                x = torch.tensor(node_obs[t])
                m = torch.tensor(node_adj[t])
                na = torch.tensor(node_agent[t])
                state_in = None if nm.state is None else nm.state.clone()
                h = nm(x, m, na, no_agent_mapping=True)
                mapped = NetMon.output_to_network_obs(h, na)
                d[f"v{vi}_h_{t}"] = h.numpy()
                d[f"v{vi}_mapped_{t}"] = mapped.numpy()
                d[f"v{vi}_state_{t}"] = nm.state.numpy()
                if state_in is not None:
                    d[f"v{vi}_statein_{t}"] = state_in.numpy()
    # DQN policy network on the joint observation (agent obs ++ NetMon graph obs)
    torch.manual_seed(42)
    joint = np.concatenate([agent_obs[0], d["v0_mapped_0"]], axis=-1).astype(np.float32)
    dqn = DQN(joint.shape[-1], [512, 256], 4, F.leaky_relu)
    sd_to_npz("dqn_w_", dqn.state_dict(), d)
    with torch.no_grad():
        q = dqn(torch.tensor(joint), None)
    d["dqn_obs"] = joint
    d["dqn_q"] = q.numpy()
    np.savez_compressed(out, **d)


def gen_netmon_global(out, Network, Routing, EVAL_SEEDS, NetMon):
    """NetMon with --netmon-global (src/model.py:451-474, 624-627): readout [h | mean_nodes(h) |
    neighbour h], mapped to agents; 3 steps with carried state, K = 1 and 2."""
    import torch
    import torch.nn.functional as F

    d = {}
    n, a, B, steps = 20, 20, 4, 3
    node_obs, node_adj, node_agent, _ = collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, steps, 200)
    d["node_obs"], d["node_adj"], d["node_agent"] = node_obs, node_adj, node_agent
    for vi, K in enumerate((1, 2)):
        torch.manual_seed(50 + vi)
        nm = NetMon(node_obs.shape[-1], 32, [64, 48], K, F.leaky_relu, rnn_type="lstm", rnn_carryover=True,
                    agg_type="sum", output_neighbor_hidden=True, output_global_hidden=True)
        nm.eval()
        sd_to_npz(f"v{vi}_w_", nm.state_dict(), d)
        d[f"v{vi}_out_features"] = np.int64(nm.get_out_features())
        nm.state = None
        with torch.no_grad():
            for t in range(steps):
                mapped = nm(torch.tensor(node_obs[t]), torch.tensor(node_adj[t]), torch.tensor(node_agent[t]))
                d[f"v{vi}_mapped_{t}"] = mapped.numpy()
                d[f"v{vi}_state_{t}"] = nm.state.numpy()
    np.savez_compressed(out, **d)
    print("netmon_global done", flush=True)


def gen_netmon_nocarry(out, Network, Routing, EVAL_SEEDS, NetMon):
    """NetMon with --netmon-rnn-carryover 0 (src/model.py:380-391, 536-570): the state holds the
    obs cell's and the update cell's outputs, the first update iteration continues from the
    previous step's update-cell state; 3 steps with carried state, lstm / lnlstm / gru, K = 1, 2."""
    import torch
    import torch.nn.functional as F

    d = {}
    n, a, B, steps = 20, 20, 4, 3
    node_obs, node_adj, node_agent, _ = collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, steps, 300)
    d["node_obs"], d["node_adj"], d["node_agent"] = node_obs, node_adj, node_agent
    variants = [("lstm", 1), ("lstm", 2), ("lnlstm", 1), ("gru", 2)]
    d["variants"] = np.array([f"{r}:{k}" for r, k in variants])
    for vi, (rnn, K) in enumerate(variants):
        torch.manual_seed(70 + vi)
        nm = NetMon(node_obs.shape[-1], 32, [64, 48], K, F.leaky_relu, rnn_type=rnn, rnn_carryover=False,
                    agg_type="sum", output_neighbor_hidden=True, output_global_hidden=False)
        nm.eval()
        sd_to_npz(f"v{vi}_w_", nm.state_dict(), d)
        d[f"v{vi}_state_size"] = np.int64(nm.get_state_size())
        nm.state = None
        with torch.no_grad():
            for t in range(steps):
                mapped = nm(torch.tensor(node_obs[t]), torch.tensor(node_adj[t]), torch.tensor(node_agent[t]))
                d[f"v{vi}_mapped_{t}"] = mapped.numpy()
                d[f"v{vi}_state_{t}"] = nm.state.numpy()
    np.savez_compressed(out, **d)
    print("netmon_nocarry done", flush=True)


def gen_models(out, Network, Routing, EVAL_SEEDS, DGN, DQNR, CommNet):
    """DGN / DQNR / CommNet forwards (src/model.py:45-184, 653-794) on real routing agent
    observations and agent adjacency: Q, attention weights, recurrent agent states over a
    3-step sequence (state carried, done agents reset like src/main.py:712-716)."""
    import torch
    import torch.nn.functional as F

    d = {}
    n, a, B, steps = 20, 20, 4, 3
    obs_l, adj_l, done_l = [], [], []
    envs = []
    for b in range(B):
        net = Network(n_nodes=n, random_topology=True, topology_init_seed=476, excluded_seeds=EVAL_SEEDS)
        env = Routing(net, a, 1)
        np.random.seed(300 + b)
        envs.append((env, env.reset()))
    rs = np.random.RandomState(5)
    for t in range(steps):
        ob, ad, dn = [], [], []
        for b, (env, (o, g)) in enumerate(envs):
            ob.append(o.astype(np.float32))
            ad.append(g.astype(np.float32))
            o2, g2, r, done, _ = env.step(rs.randint(4, size=a))
            dn.append(done)
            envs[b] = (env, (o2, g2))
        obs_l.append(np.stack(ob))
        adj_l.append(np.stack(ad))
        done_l.append(np.stack(dn))
    d["obs"], d["adj"], d["done"] = np.stack(obs_l), np.stack(adj_l), np.stack(done_l).astype(np.int8)
    D = d["obs"].shape[-1]
    models = [
        ("dgn", lambda: DGN(D, [512, 256], 4, 8, 2, F.leaky_relu)),
        ("dgn_small", lambda: DGN(D, [64], 4, 3, 1, F.leaky_relu)),
        ("dqnr", lambda: DQNR(D, [128, 64], 4, F.leaky_relu)),
        ("commnet", lambda: CommNet(D, [128, 64], 4, 2, F.leaky_relu)),
    ]
    for mi, (name, make) in enumerate(models):
        torch.manual_seed(70 + mi)
        m = make()
        m.eval()
        sd_to_npz(f"{name}_w_", m.state_dict(), d)
        last_state = None
        with torch.no_grad():
            for t in range(steps):
                if hasattr(m, "state"):
                    m.state = last_state
                    if last_state is not None:
                        d[f"{name}_statein_{t}"] = last_state.numpy().copy()
                q = m(torch.tensor(d["obs"][t]), torch.tensor(d["adj"][t]))
                d[f"{name}_q_{t}"] = q.numpy()
                if hasattr(m, "att_weights"):
                    for li, w in enumerate(m.att_weights):
                        d[f"{name}_att{li}_{t}"] = w.numpy()
                if hasattr(m, "state"):
                    d[f"{name}_state_{t}"] = m.state.numpy().copy()
                    last_state = m.state * ~torch.tensor(d["done"][t], dtype=torch.bool).view(B, -1, 1)
    np.savez_compressed(out, **d)
    print("models done", flush=True)


def _store(d, key, arr, compact, seed):
    """Full array, or (compact, > 8192 elements) values at sample_index + row and column sums."""
    arr = np.asarray(arr)
    if not compact or arr.size <= 8192:
        d[key] = arr.copy()
        return
    import zlib

    idx = detparams.sample_index(arr.size, 4096, (seed + zlib.crc32(key.encode())) & 0x7FFFFFFF)
    d[key + "__idx"] = idx
    d[key + "__val"] = arr.reshape(-1)[idx].copy()
    d[key + "__shape"] = np.array(arr.shape, np.int64)
    a64 = arr.astype(np.float64)
    d[key + "__rowsum"] = a64.reshape(arr.shape[0], -1).sum(1)
    if arr.ndim == 2:
        d[key + "__colsum"] = a64.sum(0)


def gen_train(out, Network, Routing, EVAL_SEEDS, NetMon, DQN, interpolate_model, aux_coeff=0.0, MLP=None,
              rnn_type="lstm", agg="sum", K=1, H=32, enc=(64, 48), dqn_hidden=(64, 32), B=3, L=3, compact=False,
              det_seed=0, act="leaky_relu"):
    """One DQN+NetMon update exactly as src/main.py:832-1022 performs it (sequence replay);
    aux_coeff > 0 adds the NetMon aux head and loss (src/main.py:586-594, 868-875, 996-1000).
    rnn_type / agg / K / H / enc / dqn_hidden select the architecture (src/model.py:451-631,
    src/layernormlstm.py). compact (production sizes): parameters, target perturbation and the
    initial NetMon state come from detparams (regenerated by the tests, not stored); gradients and
    updated parameters above 8192 elements are stored at 4096 sampled positions plus their row and
    column sums (_store)."""
    import torch
    import torch.nn.functional as F
    import torch.optim as optim

    d = {}
    n, a = 20, 20
    aux_l = [] if aux_coeff > 0 else None
    node_obs, node_adj, node_agent, agent_obs = collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, L + 1, 200,
                                                                     aux=aux_l)
    rng = np.random.RandomState(5)
    torch.manual_seed(3)
    act_fn = getattr(F, act)  # src/main.py:440-441
    netmon = NetMon(node_obs.shape[-1], H, list(enc), K, act_fn, rnn_type=rnn_type,
                    rnn_carryover=True, agg_type=agg, output_neighbor_hidden=True)
    obs_dim = agent_obs.shape[-1] + netmon.get_out_features()
    model = DQN(obs_dim, list(dqn_hidden), 4, act_fn)
    d["arch"] = np.array(f"{rnn_type}|{agg}|{K}|{H}|{enc[0]},{enc[1]}|{dqn_hidden[0]},{dqn_hidden[1]}|{act}")
    if compact:
        with torch.no_grad():
            for prefix, mod in (("netmon.", netmon), ("model.", model)):
                sd = mod.state_dict()
                vals = detparams.det_state_dict(det_seed, {prefix + k: v.shape for k, v in sd.items()})
                mod.load_state_dict({k: torch.tensor(vals[prefix + k]) for k in sd})
        d["compact"] = np.int64(1)
        d["det_seed"] = np.int64(det_seed)
    model_tar = copy.deepcopy(model)
    # perturb target so that it differs from the online model
    with torch.no_grad():
        if compact:
            sd = model_tar.state_dict()
            model_tar.load_state_dict({k: torch.tensor(detparams.det_perturb(det_seed, "target." + k, v.numpy()))
                                       for k, v in sd.items()})
        else:
            for p in model_tar.parameters():
                p.add_(0.01 * torch.randn_like(p))
    if not compact:
        sd_to_npz("netmon_", netmon.state_dict(), d)
        sd_to_npz("model_", model.state_dict(), d)
        sd_to_npz("target_", model_tar.state_dict(), d)
    aux_model = None
    if aux_coeff > 0:
        S = netmon.get_state_size()
        aux_model = MLP(S, (S, n), F.leaky_relu, activation_on_output=False)
        sd_to_npz("aux_", aux_model.state_dict(), d)
        node_aux = np.stack(aux_l).reshape(L + 1, B, n, n)
        d["node_aux"] = node_aux
        d["aux_coeff"] = np.float64(aux_coeff)
    if compact:
        node_state0 = detparams.det_state(det_seed, (B, n, netmon.get_state_size()))
    else:
        node_state0 = (0.1 * rng.standard_normal((B, n, netmon.get_state_size()))).astype(np.float32)
    actions = rng.randint(4, size=(L, B, a))
    reward = rng.choice(np.array([0.0, -0.2, 10.0, -10.0, 9.8], dtype=np.float32), size=(L, B, a)).astype(np.float32)
    done = rng.rand(L, B, a) < 0.1
    episode_done = rng.rand(L, B) < 0.3
    d.update(node_obs=node_obs, node_adj=node_adj.astype(np.int8), node_agent=node_agent.astype(np.int8),
             agent_obs=agent_obs, actions=actions.astype(np.int8), reward=reward, done=done.astype(np.int8),
             episode_done=episode_done.astype(np.int8))
    if not compact:
        d["node_state0"] = node_state0
    gamma, lr, tau = 0.9, 1e-3, 0.01
    d["gamma"], d["lr"], d["tau"] = np.float64(gamma), np.float64(lr), np.float64(tau)
    parameters = list(model.parameters()) + list(netmon.parameters())
    if aux_model is not None:
        parameters = parameters + list(aux_model.parameters())
    optimizer = optim.AdamW(parameters, lr=lr)
    netmon.train()
    model.train()
    loss_q = torch.zeros(1)
    loss_aux = torch.zeros(1)
    for t in range(L):
        obs = np.concatenate([agent_obs[t], np.zeros((B, a, netmon.get_out_features()), np.float32)], -1)
        next_obs = np.concatenate([agent_obs[t + 1], np.zeros((B, a, netmon.get_out_features()), np.float32)], -1)
        obs = torch.tensor(obs)
        next_obs = torch.tensor(next_obs)
        if t == 0:
            netmon.state = torch.tensor(node_state0)
        else:
            netmon.state = last_netmon_state * (~last_ep_done).view(-1, 1, 1)  # noqa: F821
        network_obs = netmon(torch.tensor(node_obs[t]), torch.tensor(node_adj[t]), torch.tensor(node_agent[t]))
        if aux_model is not None:
            aux_prediction = aux_model(netmon.state)
            loss_aux = loss_aux + torch.mean((aux_prediction - torch.tensor(node_aux[t])) ** 2) / L
        obs[:, :, -network_obs.shape[-1]:] = network_obs
        last_netmon_state = netmon.state
        last_ep_done = torch.tensor(episode_done[t])
        q_values = model(obs, None)
        with torch.no_grad():
            nno = netmon(torch.tensor(node_obs[t + 1]), torch.tensor(node_adj[t + 1]), torch.tensor(node_agent[t + 1]))
            next_obs[:, :, -nno.shape[-1]:] = nno
            next_q = model_tar(next_obs, None)
            next_q_max = next_q.max(dim=2)[0]
        tgt = torch.tensor(reward[t]) + (~torch.tensor(done[t])) * gamma * next_q_max
        q_target = torch.scatter(q_values.detach(), -1, torch.tensor(actions[t]).unsqueeze(-1), tgt.unsqueeze(-1))
        loss_q = loss_q + torch.mean((q_values - q_target).pow(2)) / L
        d[f"q_{t}"] = q_values.detach().numpy()
        d[f"qtarget_{t}"] = q_target.numpy()
    optimizer.zero_grad()
    loss = loss_q + aux_coeff * loss_aux if aux_model is not None else loss_q
    loss.backward()
    d["loss"] = loss.detach().numpy()
    if aux_model is not None:
        d["loss_aux"] = loss_aux.detach().numpy()
    names = [f"model_{k}" for k, _ in model.named_parameters()] + [f"netmon_{k}" for k, _ in netmon.named_parameters()]
    if aux_model is not None:
        names += [f"aux_{k}" for k, _ in aux_model.named_parameters()]
    for nm_, p in zip(names, parameters):
        _store(d, "grad_raw_" + nm_, p.grad.detach().numpy(), compact, det_seed)
    torch.nn.utils.clip_grad_value_(parameters, 0.5)
    total_norm = torch.nn.utils.clip_grad_norm_(parameters, 1.0)
    d["clip_total_norm"] = np.float64(total_norm.item())
    for nm_, p in zip(names, parameters):
        _store(d, "grad_clip_" + nm_, p.grad.detach().numpy(), compact, det_seed)
    optimizer.step()
    for nm_, p in zip(names, parameters):
        _store(d, "param_after_" + nm_, p.detach().numpy(), compact, det_seed)
    interpolate_model(model, model_tar, tau, model_tar)
    for k, v in model_tar.state_dict().items():
        _store(d, "target_after_" + k, v.detach().numpy(), compact, det_seed)
    d["param_names"] = np.array(names)
    np.savez_compressed(out, **d)
    print(os.path.basename(out), "done", flush=True)


def gen_train_models(out, Network, Routing, EVAL_SEEDS, DGN, DQNR, CommNet, interpolate_model, name, att_coeff=0.0,
                     B=4, L=3, n=20, a=20, seed=400):
    """One update of a non-default model (src/main.py:840-1026 with netmon None, src/model.py:45-184,
    653-794) on real routing agent observations and agent adjacency: DGN with the attention-KL
    regulariser (att_coeff, src/main.py:920-954: the target model runs on the next observation, its
    attention weights are the KL target), DQNR / CommNet with the agent state loaded from the replayed
    start state at t = 0 (src/main.py:847-849), handed to the target model (899-902) and masked by done /
    episode_done after it (956-964). Records q, q_target, loss (and loss_q / loss_att), the raw and
    clipped gradients, the AdamW step and the soft target update, like gen_train."""
    import torch
    import torch.nn.functional as F
    import torch.optim as optim

    d = {}
    obs_l, adj_l = [], []
    envs = []
    for b in range(B):
        net = Network(n_nodes=n, random_topology=True, topology_init_seed=476, excluded_seeds=EVAL_SEEDS)
        env = Routing(net, a, 1)
        np.random.seed(seed + b)
        envs.append((env, env.reset()))
    rs = np.random.RandomState(seed)
    for t in range(L + 1):
        ob, ad = [], []
        for b, (env, (o, g)) in enumerate(envs):
            ob.append(o.astype(np.float32))
            ad.append(g.astype(np.float32))
            o2, g2, _, _, _ = env.step(rs.randint(4, size=a))
            envs[b] = (env, (o2, g2))
        obs_l.append(np.stack(ob))
        adj_l.append(np.stack(ad))
    agent_obs, agent_adj = np.stack(obs_l), np.stack(adj_l)
    D = agent_obs.shape[-1]
    act_fn = F.leaky_relu
    torch.manual_seed(seed + 1)
    make = {"dgn": lambda: DGN(D, [64, 48], 4, 4, 2, act_fn),
            "dqnr": lambda: DQNR(D, [64, 48], 4, act_fn),
            "commnet": lambda: CommNet(D, [64, 48], 4, 2, act_fn)}[name]
    model = make()
    model_tar = copy.deepcopy(model)
    with torch.no_grad():  # DGN: the attention query / key weights perturbed more, so that the KL is not ~0
        for k, p in model_tar.named_parameters():
            p.add_((0.3 if att_coeff > 0 and ("fc_q" in k or "fc_k" in k) else 0.01) * torch.randn_like(p))
    sd_to_npz("model_", model.state_dict(), d)
    sd_to_npz("target_", model_tar.state_dict(), d)
    rng = np.random.RandomState(seed + 2)
    has_state = hasattr(model, "state")
    if has_state:
        d["agent_state0"] = (0.1 * rng.standard_normal((B, a, model.get_state_len()))).astype(np.float32)
    actions = rng.randint(4, size=(L, B, a))
    reward = rng.choice(np.array([0.0, -0.2, 10.0, -10.0, 9.8], dtype=np.float32), size=(L, B, a)).astype(np.float32)
    done = rng.rand(L, B, a) < 0.15
    episode_done = rng.rand(L, B) < 0.3
    d.update(agent_obs=agent_obs, agent_adj=agent_adj.astype(np.int8), actions=actions.astype(np.int8), reward=reward,
             done=done.astype(np.int8), episode_done=episode_done.astype(np.int8))
    gamma, lr, tau = 0.9, 1e-3, 0.01
    d["gamma"], d["lr"], d["tau"], d["att_coeff"] = np.float64(gamma), np.float64(lr), np.float64(tau), np.float64(att_coeff)
    d["arch_model"] = np.array(name)
    parameters = list(model.parameters())
    optimizer = optim.AdamW(parameters, lr=lr)
    model.train()
    loss_q = torch.zeros(1)
    loss_att = torch.zeros(1)
    for t in range(L):
        obs, adj = torch.tensor(agent_obs[t]), torch.tensor(agent_adj[t])
        next_obs, next_adj = torch.tensor(agent_obs[t + 1]), torch.tensor(agent_adj[t + 1])
        bdone, bep = torch.tensor(done[t]), torch.tensor(episode_done[t])
        if has_state and t == 0:
            model.state = torch.tensor(d["agent_state0"])
        q_values = model(obs, adj)
        with torch.no_grad():
            if has_state:
                model_tar.state = model.state.detach()
            next_q = model_tar(next_obs, next_adj)
            next_q_max = next_q.max(dim=2)[0]
        if has_state:
            state_mask = ~bdone * (~bep).view(-1, 1)
            model.state = model.state * state_mask.unsqueeze(-1)
        tgt = torch.tensor(reward[t]) + (~bdone) * gamma * next_q_max
        q_target = torch.scatter(q_values.detach(), -1, torch.tensor(actions[t]).long().unsqueeze(-1),
                                 tgt.unsqueeze(-1))
        loss_q = loss_q + torch.mean((q_values - q_target).pow(2)) / L
        if hasattr(model, "att_weights") and att_coeff > 0:
            attention = F.log_softmax(torch.stack(model.att_weights), dim=-1)
            target_attention = F.softmax(torch.stack(model_tar.att_weights), dim=-1)
            shape = attention.shape
            kl = F.kl_div(attention.view(-1, a), target_attention.view(-1, a), reduction="none").view(shape)
            kl = kl.transpose(0, -2).transpose(0, 1).sum(dim=(-1, -2, -3))
            kl = (kl * ~bdone).sum() / torch.clamp((~bdone).sum(), min=1)
            loss_att = loss_att + kl / L
        d[f"q_{t}"] = q_values.detach().numpy()
        d[f"qtarget_{t}"] = q_target.numpy()
    loss = loss_q + att_coeff * loss_att
    optimizer.zero_grad()
    names = [f"model_{k}" for k, _ in model.named_parameters()]
    if att_coeff > 0:  # the regulariser's own gradient, so that its sign and scale are pinned apart from the TD term
        ga = torch.autograd.grad(att_coeff * loss_att.sum(), parameters, retain_graph=True, allow_unused=True)
        for nm_, g_ in zip(names, ga):
            d["grad_att_" + nm_] = (torch.zeros_like(p) if g_ is None else g_).detach().numpy().copy()
    loss.backward()
    d["loss"], d["loss_q"], d["loss_att"] = loss.detach().numpy(), loss_q.detach().numpy(), loss_att.detach().numpy()
    for nm_, p in zip(names, parameters):
        d["grad_raw_" + nm_] = p.grad.detach().numpy().copy()
    torch.nn.utils.clip_grad_value_(parameters, 0.5)
    d["clip_total_norm"] = np.float64(torch.nn.utils.clip_grad_norm_(parameters, 1.0).item())
    for nm_, p in zip(names, parameters):
        d["grad_clip_" + nm_] = p.grad.detach().numpy().copy()
    optimizer.step()
    for nm_, p in zip(names, parameters):
        d["param_after_" + nm_] = p.detach().numpy().copy()
    interpolate_model(model, model_tar, tau, model_tar)
    for k, v in model_tar.state_dict().items():
        d["target_after_" + k] = v.detach().numpy().copy()
    d["param_names"] = np.array(names)
    np.savez_compressed(out, **d)
    print(os.path.basename(out), "done", flush=True)


# ---------------------------------------------------------------------------
# SimpleEnvironment traces (src/env/simple_environment.py) with EpsilonGreedy
# draws (src/policy.py:44-50) on the same global stream
# ---------------------------------------------------------------------------
SIMPLE_CONFIGS = [(0, 1, 1), (1, 1, 0), (42, 3, 1), (7, 2, 1), (123, 1, 1), (5, 3, 0)]


def simple_snapshot(env):
    score = np.array([r.score for r in env.router], np.int32)
    redge = np.full((3, 2), -1, np.int32)
    for i, r in enumerate(env.router):
        for k, e in enumerate(r.edge):
            redge[i, k] = int(e)
    ends = np.array([[e.start, e.end] for e in env.edges], np.int32)
    return score, redge, ends, np.int32(env.start_node)


def gen_simple(out, SimpleEnvironment):
    d = {"configs": np.array(SIMPLE_CONFIGS, np.int64)}
    T, eps = 40, 0.5
    for ci, (seed, env_var, rt) in enumerate(SIMPLE_CONFIGS):
        np.random.seed(seed)
        env = SimpleEnvironment(env_var=env_var, random_topology=bool(rt))
        qrng = np.random.RandomState(1000 + seed)
        rec = {k: [] for k in ("reset", "q", "act", "obs", "reward", "score", "redge", "ends", "start",
                               "node_obs", "node_adj", "node_agent")}
        for t in range(T):
            if t % 3 == 0:
                obs, adj = env.reset()
                rec["reset"].append(1)
            else:
                rec["reset"].append(0)
            sc, re_, en, st = simple_snapshot(env)
            rec["score"].append(sc)
            rec["redge"].append(re_)
            rec["ends"].append(en)
            rec["start"].append(st)
            rec["node_obs"].append(env.get_node_observation())
            rec["node_adj"].append(env.get_nodes_adjacency().copy())
            rec["node_agent"].append(env.get_node_agent_matrix())
            q = qrng.standard_normal((1, 2)).astype(np.float32)
            random_actions = np.random.randint(2, size=1)
            random_filter = np.random.rand(1) < eps
            act = np.argmax(q, axis=-1) * ~random_filter + random_filter * random_actions
            obs, adj, reward, done, info = env.step(act)
            assert done[0]
            rec["q"].append(q)
            rec["act"].append(act.astype(np.int32))
            rec["obs"].append(np.asarray(obs, np.float32))
            rec["reward"].append(np.asarray(reward, np.float32))
        for k, v in rec.items():
            d[f"c{ci}_{k}"] = np.array(v)
    np.savez_compressed(out, **d)
    print("simple:", out)


# ---------------------------------------------------------------------------
# ShortestPath heuristic (src/policy.py:90-139): networkx first hops and traces
# ---------------------------------------------------------------------------
def first_hops(net):
    n = net.n_nodes
    f = np.zeros((n, n), np.int32)
    for i in range(n):
        for j in range(n):
            f[i, j] = i if i == j else net.shortest_paths[i][j][1]
    return f


def gen_shortest(out, Network, Routing, EVAL_SEEDS, ShortestPath):
    d = {}
    nets = []
    for s in [476, 923430603] + list(EVAL_SEEDS[:30]):
        net = Network(n_nodes=20, random_topology=False, topology_init_seed=s)
        net.reset()
        nets.append(net)
    for n, main_seed, count in [(10, 21, 8), (50, 22, 6), (64, 23, 4)]:
        np.random.seed(main_seed)
        net = Network(n_nodes=n, random_topology=True, excluded_seeds=EVAL_SEEDS)
        for _ in range(count):
            net.reset()
            nets.append(copy.deepcopy(net))
    for i, net in enumerate(nets):
        d[f"t{i}_edges"] = np.array([[e.start, e.end, e.length] for e in net.edges], np.int64)
        d[f"t{i}_first"] = first_hops(net)
    d["n_tables"] = np.int64(len(nets))

    class _Args:
        pass

    for name, mode, seed, T, ep in [("fixed476", "fixed", 0, 100, 100), ("rand20", "random", 3, 100, 25)]:
        if mode == "fixed":
            net = Network(n_nodes=20, random_topology=False, topology_init_seed=476)
        else:
            net = Network(n_nodes=20, random_topology=True, topology_init_seed=476, excluded_seeds=EVAL_SEEDS)
        env = Routing(net, 20, 1, enable_congestion=True, enable_action_mask=False, ttl=0)
        pol = ShortestPath(env, None, 4, _Args())
        np.random.seed(seed)
        env.reset()
        acts, rews = [], []
        for t in range(T):
            a = pol(None, None)
            _, _, r, _, _ = env.step(a)
            acts.append(np.asarray(a, np.int32))
            rews.append(np.asarray(r, np.float32))
            if (t + 1) % ep == 0:
                env.reset()
        d[f"trace_{name}_actions"] = np.stack(acts)
        d[f"trace_{name}_reward"] = np.stack(rews)
        d[f"trace_{name}_cfg"] = np.array([seed, T, ep], np.int64)
    np.savez_compressed(out, **d)
    print("shortest:", out)


# ---------------------------------------------------------------------------
# Evaluation reducer (src/eval.py) with the ShortestPath policy on EVAL_SEEDS, set up
# like `main.py --eval --policy=heuristic` (src/main.py:409-575), and the CLI flags
# ---------------------------------------------------------------------------
EVAL_CONFIGS = [(0, 6, 40, 20, 20), (5, 4, 60, 20, 12), (9, 3, 30, 20, 8)]  # seed, episodes, steps, N, A


def gen_eval(out, Network, Routing, EVAL_SEEDS, ShortestPath, evaluate):
    d = {"configs": np.array(EVAL_CONFIGS, np.int64)}

    class _Args:
        pass

    for ci, (seed, episodes, steps, n, a) in enumerate(EVAL_CONFIGS):
        np.random.seed(seed)
        net = Network(n_nodes=n, random_topology=True, n_random_seeds=0, topology_init_seed=476,
                      excluded_seeds=EVAL_SEEDS)
        env = Routing(net, a, 1, enable_congestion=True, enable_action_mask=False, ttl=0)
        env.reset()  # reset_and_get_sizes
        pol = ShortestPath(env, None, 4, _Args())
        env.network.seeds = EVAL_SEEDS
        env.network.sequential_topology_seeds = True
        m = evaluate(env, pol, episodes, steps, True)
        keys = sorted(m)
        d[f"c{ci}_keys"] = np.array(keys)
        d[f"c{ci}_values"] = np.array([float(m[k]) for k in keys], np.float64)
    np.savez_compressed(out, **d)
    print("eval:", out)


def gen_cli_flags(out, ref):
    import json
    import re

    src = open(os.path.join(ref, "main.py")).read()
    flags = sorted(set(re.findall(r'add_argument\(\s*"(--[a-z0-9-]+)"', src)))
    with open(out, "w") as f:
        json.dump(flags, f, indent=1)
    print("cli flags:", len(flags))


# ---------------------------------------------------------------------------
# Supervised shortest-path task (src/sl.py): samples and one NetMonSL update
# ---------------------------------------------------------------------------
def gen_sl(out, Network, Routing, EVAL_SEEDS, NetMon, n=20, seeds=None, H=32, enc=(64, 48)):
    """n = 20: small NetMon (H 32, encoder 64,48) on 8 EVAL_SEEDS graphs; n = 100 (BASELINE
    config 5): the CLI-default NetMon (H 128, encoder 512,256) on 4 valid 100-node seeds."""
    import torch
    import torch.nn as nn
    import torch.nn.functional as F

    d = {}
    # get_sl_sample (src/sl.py:174-218) on graphs from fixed seeds
    seeds = list(EVAL_SEEDS[100:108]) if seeds is None else [int(x) for x in seeds]
    net = Network(n, random_topology=True, sequential_topology_seeds=True, provided_seeds=seeds)
    env = Routing(net, 20, 1)
    np.random.seed(5)
    env.reset()
    obs, adj, labels, targets_all = [], [], [], []
    for s in range(len(seeds)):
        if s > 0:
            env.reset()
        n = env.get_num_nodes()
        lab = np.zeros(n, np.int64)
        ta = np.zeros((n, n), np.float32)
        for v in range(n):
            for w in range(n):
                ta[v, w] = env.network.shortest_paths_weights[v][w]
            p0 = env.network.shortest_paths[v][0]
            if len(p0) > 1:
                for e_idx, e in enumerate(env.network.nodes[v].edges):
                    if env.network.edges[e].get_other_node(v) == p0[1]:
                        lab[v] = e_idx + 1
                        break
        obs.append(env.get_node_observation())
        adj.append(env.get_nodes_adjacency().astype(np.float32))
        labels.append(lab)
        targets_all.append(ta)
    d["seeds"] = np.array(seeds, np.int64)
    d["node_obs"] = np.stack(obs)
    d["node_adj"] = np.stack(adj)
    d["labels"] = np.stack(labels)
    d["targets_all"] = np.stack(targets_all)
    # NetMonSL (src/sl.py:132-168) = reference NetMon + 3 nn.Linear heads; one train
    # iteration (src/sl.py:360-424) with seq_len 2, regression-all loss
    torch.manual_seed(3)
    netmon = NetMon(4 * n + 8, H, list(enc), 1, activation_fn=F.leaky_relu, rnn_type="lstm", rnn_carryover=True,
                    agg_type="sum", output_neighbor_hidden=True, output_global_hidden=False)
    heads = [nn.Linear(netmon.get_out_features(), k) for k in (4, 1, n)]
    params = list(netmon.parameters()) + [p for h in heads for p in h.parameters()]
    names = [f"netmon.{k}" for k, _ in netmon.named_parameters()] + \
        [f"{hn}.{k}" for hn, h in zip(("linear", "linear_reg", "linear_reg_all"), heads) for k, _ in h.named_parameters()]
    for nme, p in zip(names, params):
        d["w_" + nme] = p.detach().numpy().copy()
    x = torch.tensor(d["node_obs"])
    a = torch.tensor(d["node_adj"])
    eye = torch.eye(n).repeat(x.shape[0], 1, 1)
    tgt = torch.tensor(d["targets_all"])
    netmon.state = None
    seq = []
    for t in range(2):
        feats = netmon(x, a, eye)
        pred_all = heads[2](feats)
        d[f"pred_all_{t}"] = pred_all.detach().numpy().copy()
        seq.append(F.mse_loss(pred_all, tgt))
    total = torch.mean(torch.stack(seq))
    total.backward()
    d["loss"] = np.float64(total.item())
    for nme, p in zip(names, params):
        d["g_" + nme] = (p.grad.numpy().copy() if p.grad is not None else np.zeros(p.shape, np.float32))
    d["param_names"] = np.array(names)
    d["config"] = np.array([n, H, enc[0], enc[1]], np.int64)
    np.savez_compressed(out, **d)
    print("sl:", out)


def gen_sl_prod(out, Network, NetMon, n=100, graphs=328, det_seed=31, topo_seed=17):
    """BASELINE config 5 at its production tiles: the CLI-default NetMon (H 128,
    encoder 512,256, K 1, lstm, sum) on `graphs` valid random 100-node topologies (328 x 100 = 32 800 node
    rows per GEMM: the LDS-DMA k_gemm3g forms), one train iteration of src/sl.py:360-424 with seq_len 2
    and the regression-all loss. Stored compactly like train_prod: the topology seeds (drawn by the
    reference's own _create_valid_network from np.random.seed(topo_seed), EVAL_SEEDS excluded) and
    their neighbour tables; node features, parameters and the initial state regenerated from detparams
    (not stored); targets (the reference's APSP weights), predictions and gradients at sampled
    positions plus row / column sums (_store)."""
    import torch
    import torch.nn as nn
    import torch.nn.functional as F

    from env.constants import EVAL_SEEDS

    d = {}
    np.random.seed(topo_seed)
    net = Network(n, random_topology=True, excluded_seeds=list(EVAL_SEEDS))
    seeds, adj, ta = [], [], []
    for g in range(graphs):
        net.reset()
        seeds.append(net.current_topology_seed)
        adj.append(net.get_nodes_adjacency().astype(np.float32))  # I + A, as gen_sl passes it
        t = np.zeros((n, n), np.float32)
        for v in range(n):
            for w in range(n):
                t[v, w] = net.shortest_paths_weights[v][w]
        ta.append(t)
    a = np.stack(adj)
    d["seeds"] = np.array(seeds, np.int64)
    nbr = np.full((graphs, n, 3), -1, np.int16)
    for g in range(graphs):
        for v in range(n):
            nb = [w for w in np.nonzero(a[g, v])[0] if w != v]
            nbr[g, v, :len(nb)] = nb
    d["nbr"] = nbr
    targets_all = np.stack(ta)
    x = detparams.det_tensor(det_seed, "node_obs", (graphs, n, 4 * n + 8))  # U(-1/sqrt(fan), ..) scaled below
    x = (x * np.sqrt(4 * n + 8)).astype(np.float32)  # U(-1, 1) node features
    torch.manual_seed(3)
    netmon = NetMon(4 * n + 8, 128, [512, 256], 1, activation_fn=F.leaky_relu, rnn_type="lstm", rnn_carryover=True,
                    agg_type="sum", output_neighbor_hidden=True, output_global_hidden=False)
    heads = [nn.Linear(netmon.get_out_features(), k) for k in (4, 1, n)]
    names = [f"netmon.{k}" for k, _ in netmon.named_parameters()] + \
        [f"{hn}.{k}" for hn, h in zip(("linear", "linear_reg", "linear_reg_all"), heads) for k, _ in h.named_parameters()]
    params = list(netmon.parameters()) + [p for h in heads for p in h.parameters()]
    with torch.no_grad():
        for nme, p in zip(names, params):
            p.copy_(torch.tensor(detparams.det_tensor(det_seed, nme, p.shape)))
    xt = torch.tensor(x)
    at = torch.tensor(a)
    eye = torch.eye(n).repeat(graphs, 1, 1)
    tgt = torch.tensor(targets_all)
    netmon.state = None
    seq = []
    for t in range(2):
        feats = netmon(xt, at, eye)
        pred_all = heads[2](feats)
        _store(d, f"pred_all_{t}", pred_all.detach().numpy().reshape(graphs * n, n), True, det_seed)
        seq.append(F.mse_loss(pred_all, tgt))
    total = torch.mean(torch.stack(seq))
    total.backward()
    d["loss"] = np.float64(total.item())
    _store(d, "targets_all", targets_all.reshape(graphs * n, n), True, det_seed)
    for nme, p in zip(names, params):
        _store(d, "g_" + nme, p.grad.numpy() if p.grad is not None else np.zeros(p.shape, np.float32), True, det_seed)
    d["param_names"] = np.array(names)
    d["config"] = np.array([n, 128, 512, 256, graphs, det_seed], np.int64)
    np.savez_compressed(out, **d)
    print("sl_prod:", out, flush=True)


def gen_replay(out, ReplayBuffer):
    """ReplayBuffer sampling indices (src/replaybuffer.py:101-130): transitions t = 0, 1, ...
    inserted in order (obs = t), then a script of get_batch calls (uniform and sequence) with
    interleaved inserts, including ring wrap-around; the yielded TransitionBatch.indices of
    every call are recorded in call order."""
    d = {}
    scripts = {
        # name: (seed, buffer_size, [("add", n) | ("get", batch, seq_len)])
        "a": (7, 64, [("add", 40), ("get", 32, 1), ("get", 17, 1), ("get", 16, 8), ("get", 5, 3), ("add", 60),
                      ("get", 32, 1), ("get", 33, 8), ("get", 1, 2), ("get", 32, 0)]),
        "b": (0, 1000, [("add", 523), ("get", 4096, 8), ("get", 3, 1), ("add", 900), ("get", 2049, 8),
                        ("get", 4097, 1)]),
        "c": (123456789, 10, [("add", 9), ("get", 7, 8), ("get", 5, 1), ("add", 3), ("get", 6, 2)]),
    }
    for name, (seed, size, script) in scripts.items():
        rb = ReplayBuffer(seed, size, 2, 3, 0)
        t = 0
        calls = []
        for op in script:
            if op[0] == "add":
                for _ in range(op[1]):
                    z2 = np.zeros((2, 2), bool)
                    rb.add(np.full((2, 3), t, np.float32), np.zeros(2, np.int8), np.zeros(2, np.float32),
                           np.zeros((2, 3), np.float32), z2, z2, np.zeros(2, bool), False, np.zeros((1, 2, 0)),
                           np.zeros((0, 0)), np.zeros((0, 0)), np.zeros((0, 0)), np.zeros((0, 0), bool),
                           np.zeros((0, 2), bool), np.zeros((0, 0)), np.zeros((0, 0), bool), np.zeros((0, 2), bool))
                    t += 1
            else:
                idx = [np.asarray(b.idx, np.int64) for b in rb.get_batch(op[1], "cpu", sequence_length=op[2])]
                calls.append(np.stack(idx))
        d[f"{name}_seed"] = np.int64(seed)
        d[f"{name}_size"] = np.int64(size)
        d[f"{name}_script"] = np.array([[0, op[1], 0] if op[0] == "add" else [1, op[1], op[2]] for op in script],
                                       np.int64)
        for i, c in enumerate(calls):
            d[f"{name}_idx{i}"] = c
        st = rb._random_generator.bit_generator.state
        d[f"{name}_final_state"] = np.array([st["state"]["state"] >> 64, st["state"]["state"] & (2**64 - 1),
                                             st["has_uint32"], st["uinteger"]], np.uint64)
    np.savez_compressed(out, **d)
    print("replay:", out)


def gen_checkpoint(out_pt, out_npz, ref, Network, Routing, EVAL_SEEDS, NetMon, DQN, get_state_dict):
    """A checkpoint written by the reference's own get_state_dict (src/util.py:26-35) with the
    args.__dict__ of the reference's own parser (src/main.py:40-381, the parser statements executed
    here) for a small NetMon + DQN, saved with torch.save as src/main.py:812-817 does; plus the
    reference models' Q-values over 3 carried NetMon steps on 2 graphs (NetMonWrapper +
    EpsilonGreedy.q, src/env/wrapper.py:66-109, src/model.py:187-203)."""
    import torch
    import torch.nn.functional as F

    import types

    tb = types.ModuleType("torch.utils.tensorboard")
    tbw = types.ModuleType("torch.utils.tensorboard.writer")
    tbw.SummaryWriter = type("SummaryWriter", (), {})  # imported by main.py, never used by the parser
    tb.writer = tbw
    sys.modules.setdefault("torch.utils.tensorboard", tb)
    sys.modules.setdefault("torch.utils.tensorboard.writer", tbw)
    src = open(os.path.join(ref, "main.py")).read()
    ns = {"__name__": "reference_main_parser"}
    exec(compile(src[: src.index("args = parser.parse_args()")], "main.py", "exec"), ns)
    args = ns["parser"].parse_args(["--env-type=routing", "--model=dqn", "--netmon", "--netmon-dim=16",
                                    "--netmon-encoder-dim=32,16", "--netmon-iterations=2", "--hidden-dim=32,24",
                                    "--seed=3"])
    n, a, B, steps = 20, 20, 2, 3
    node_obs, node_adj, node_agent, agent_obs = collect_graph_inputs(Network, Routing, EVAL_SEEDS, n, a, B, steps, 300)
    torch.manual_seed(21)
    act = getattr(F, args.activation_function)
    netmon = NetMon(node_obs.shape[-1], args.netmon_dim, [int(x) for x in args.netmon_encoder_dim.split(",")],
                    args.netmon_iterations, activation_fn=act, rnn_type=args.netmon_rnn_type,
                    rnn_carryover=args.netmon_rnn_carryover, agg_type=args.netmon_agg_type,
                    output_neighbor_hidden=True, output_global_hidden=args.netmon_global)
    model = DQN(agent_obs.shape[-1] + netmon.get_out_features(), [int(x) for x in args.hidden_dim.split(",")], 4,
                act)
    torch.save(get_state_dict(model, netmon, args.__dict__), out_pt)
    d = {"node_obs": node_obs, "node_adj": node_adj, "node_agent": node_agent, "agent_obs": agent_obs}
    netmon.eval()
    model.eval()
    netmon.state = None
    with torch.no_grad():
        for t in range(steps):
            h = netmon(torch.tensor(node_obs[t]), torch.tensor(node_adj[t]), torch.tensor(node_agent[t]))
            joint = torch.cat([torch.tensor(agent_obs[t]), h], -1)
            d[f"q_{t}"] = model(joint, None).numpy()
    np.savez_compressed(out_npz, **d)
    print("checkpoint:", out_pt, out_npz)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference/src")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    stub_dir = tempfile.mkdtemp(prefix="gm_ref_stubs_")
    write_stubs(stub_dir)
    sys.path[:0] = [stub_dir, args.ref]

    from env.network import Network  # noqa: E402
    from env.routing import Routing  # noqa: E402
    from env.constants import EVAL_SEEDS  # noqa: E402
    from model import MLP, NetMon, DQN, DGN, DQNR, CommNet  # noqa: E402
    from util import get_state_dict, interpolate_model  # noqa: E402
    from env.simple_environment import SimpleEnvironment  # noqa: E402
    from policy import ShortestPath  # noqa: E402
    from eval import evaluate  # noqa: E402
    from replaybuffer import ReplayBuffer  # noqa: E402

    only = set(args.only.split(",")) if args.only else None
    if only is None or "seeds" in only:
        np.save(os.path.join(HERE, "eval_seeds.npy"), np.array(EVAL_SEEDS, dtype=np.int64))
    if only is None or "rng" in only:
        gen_rng(os.path.join(HERE, "rng.npz"))
    if only is None or "topology" in only:
        gen_topology(os.path.join(HERE, "topology.npz"), Network, EVAL_SEEDS)
    if only is None or "env" in only:
        gen_env(HERE, Network, Routing, EVAL_SEEDS)
    elif any(o.startswith("env:") for o in only):  # --only env:name1,env:name2
        gen_env(HERE, Network, Routing, EVAL_SEEDS, {o[4:] for o in only if o.startswith("env:")})
    if only is None or "netmon" in only:
        gen_netmon(os.path.join(HERE, "netmon.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN)
    if only is None or "netmon_global" in only:
        gen_netmon_global(os.path.join(HERE, "netmon_global.npz"), Network, Routing, EVAL_SEEDS, NetMon)
    if only is None or "netmon_nocarry" in only:
        gen_netmon_nocarry(os.path.join(HERE, "netmon_nocarry.npz"), Network, Routing, EVAL_SEEDS, NetMon)
    if only is None or "models" in only:
        gen_models(os.path.join(HERE, "models.npz"), Network, Routing, EVAL_SEEDS, DGN, DQNR, CommNet)
    if only is None or "train" in only:
        gen_train(os.path.join(HERE, "train.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN, interpolate_model)
    if only is None or "train_aux" in only:
        gen_train(os.path.join(HERE, "train_aux.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN, interpolate_model,
                  aux_coeff=0.3, MLP=MLP)
    if only is None or "train_lnlstm" in only:
        gen_train(os.path.join(HERE, "train_lnlstm.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN,
                  interpolate_model, rnn_type="lnlstm", agg="mean", K=2, B=4)
    if only is None or "train_gru" in only:
        gen_train(os.path.join(HERE, "train_gru.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN,
                  interpolate_model, rnn_type="gru", agg="sum", K=2, B=4)
    if only is None or "train_big" in only:
        # the CLI-default architecture at row counts where every training kernel runs its HIP form
        # (256 graphs x 20 nodes = 5120 rows per step, 20480 over the 4 steps)
        gen_train(os.path.join(HERE, "train_big.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN, interpolate_model,
                  H=128, enc=(512, 256), dqn_hidden=(512, 256), B=256, L=4, compact=True, det_seed=11)
    if only is None or "train_prod" in only:
        # the production forward / input-gradient tiles: 512 graphs x 4 steps = 40 960 node and agent rows
        # per batched layer (>= 32 768: the LDS-DMA k_gemm3g forms of the sequence-batched update)
        gen_train(os.path.join(HERE, "train_prod.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN, interpolate_model,
                  H=128, enc=(512, 256), dqn_hidden=(512, 256), B=512, L=4, compact=True, det_seed=23)
    # --activation-function (src/main.py:194-197, 440-441); softplus: derivative from the output, gelu / silu /
    # mish: from the pre-activation (round 4)
    for act in ("relu", "elu", "tanh", "sigmoid", "softplus", "gelu", "silu", "mish"):
        if only is None or f"train_{act}" in only:
            gen_train(os.path.join(HERE, f"train_{act}.npz"), Network, Routing, EVAL_SEEDS, NetMon, DQN,
                      interpolate_model, K=2, B=4, act=act)
    # the non-default models' updates: DGN with the attention-KL regulariser, DQNR / CommNet
    # with the replayed agent state
    for mname, coeff in (("dgn", 0.03), ("dqnr", 0.0), ("commnet", 0.0)):
        if only is None or f"train_{mname}" in only:
            gen_train_models(os.path.join(HERE, f"train_{mname}.npz"), Network, Routing, EVAL_SEEDS, DGN, DQNR, CommNet,
                             interpolate_model, mname, att_coeff=coeff)
    if only is None or "checkpoint" in only:
        gen_checkpoint(os.path.join(HERE, "ref_checkpoint.pt"), os.path.join(HERE, "ref_checkpoint.npz"), args.ref,
                       Network, Routing, EVAL_SEEDS, NetMon, DQN, get_state_dict)
    if only is None or "shortest" in only:
        gen_shortest(os.path.join(HERE, "shortest.npz"), Network, Routing, EVAL_SEEDS, ShortestPath)
    if only is None or "eval" in only:
        gen_eval(os.path.join(HERE, "eval.npz"), Network, Routing, EVAL_SEEDS, ShortestPath, evaluate)
    if only is None or "cli" in only:
        gen_cli_flags(os.path.join(HERE, "cli_flags.json"), args.ref)
    if only is None or "sl" in only:
        gen_sl(os.path.join(HERE, "sl.npz"), Network, Routing, EVAL_SEEDS, NetMon)
    if only is None or "sl100" in only:
        seeds100 = np.load(os.path.join(HERE, "topology.npz"))["rand_n100_seed"][:4]
        gen_sl(os.path.join(HERE, "sl_n100.npz"), Network, Routing, EVAL_SEEDS, NetMon, n=100, seeds=seeds100,
               H=128, enc=(512, 256))
    if only is None or "sl_prod" in only:
        gen_sl_prod(os.path.join(HERE, "sl_prod.npz"), Network, NetMon)
    if only is None or "replay" in only:
        gen_replay(os.path.join(HERE, "replay.npz"), ReplayBuffer)
    if only is None or "simple" in only:
        gen_simple(os.path.join(HERE, "simple.npz"), SimpleEnvironment)


if __name__ == "__main__":
    main()
