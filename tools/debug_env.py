"""GPU debug: first-reset state/topology of the device env vs the C oracle."""
import importlib, sys, os, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"]
import numpy as np, torch
import oracle as O
gm = importlib.import_module("graph-marl_amd")
t0 = time.time()
for mode in ["fixed", "random"]:
    N, A, B = 20, 20, 2
    if mode == "fixed":
        net = gm.Network(N, random_topology=False, topology_init_seed=476)
        cfg = O.make_config(N, A, topo_mode=O.TOPO_FIXED, topo_seed=476)
    else:
        net = gm.Network(N, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
        cfg = O.make_config(N, A, topo_mode=O.TOPO_RANDOM, excluded=gm.EVAL_SEEDS)
    env = gm.Routing(net, A, n_env=B, seeds=[0, 1])
    print(mode, "created", time.time() - t0, flush=True)
    env.reset_()
    torch.cuda.synchronize()
    print(mode, "reset done", time.time() - t0, flush=True)
    try:
        st = env.get_state()
    except Exception as ex:
        print("get_state error:", ex, flush=True)
        continue
    for b in range(B):
        o = O.OracleEnv(cfg, b)
        o.reset()
        s = o.state(); tp = o.topology()
        print(f"env {b} topo seed dev={st['topo_seed'][b]} orc={s['topo_seed']} reps dev={st['topo_reps'][b]} orc={tp['repetitions']}")
        E = tp['E']
        print(" edges dev:", np.stack([st['edge_a'][b], st['edge_b'][b], st['edge_len'][b]], -1)[:6].tolist())
        print(" edges orc:", tp['edges'][:6].tolist())
        print(" nbr_edge dev:", st['nbr_edge'][b][:4].tolist(), " orc:", tp['node_edges'][:4].tolist())
        print(" apsp row0 dev:", st['apsp'][b][0].tolist())
        print(" apsp row0 orc:", tp['apsp'][0].tolist())
        for k in ["now", "target", "spw", "size", "rng_pos"]:
            dv = st[k][b]; ov = s[k]
            print(f" {k}: eq={np.array_equal(np.asarray(dv), np.asarray(ov))} dev={np.asarray(dv).ravel()[:6]} orc={np.asarray(ov).ravel()[:6]}")
        print(" rng key eq:", np.array_equal(st['rng_key'][b], s['rng_key']), flush=True)
print("total", time.time() - t0)
