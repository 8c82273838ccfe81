"""Replays a golden environment trace (tests/golden/env_*.npz) against an env
implementation and checks every snapshot bit-exactly.

The implementation is anything with the small adapter interface used below
(reset / egreedy / step / state / observe / final_delays), so the same replay
drives the C oracle (CPU tests) and the HIP environment (GPU tests).
"""
import glob
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EVAL_SEEDS = np.load(os.path.join(GOLDEN, "eval_seeds.npy"))


def sha(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def env_golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "env_*.npz")))


def load(path):
    g = np.load(path)
    cfg = {k[4:]: g[k].item() for k in g.files if k.startswith("cfg_")}
    return g, cfg


def topo_spec(cfg, golden_topology_seedlist=None):
    """(mode, fixed seed, seed list) for a golden config, mirroring make_golden.py."""
    mode = cfg["mode"]
    if mode == "fixed":
        return "fixed", int(cfg["topo"]), None
    if mode == "random":
        return "random", int(cfg["topo"]), None
    if mode == "list":
        return "list", int(cfg["topo"]), golden_topology_seedlist
    if mode == "sequential":
        return "sequential", int(cfg["topo"]), EVAL_SEEDS[:8].astype(np.int64)
    raise ValueError(mode)


def check_snapshot(g, si, st, ob, n, A):
    E = 3 * n // 2
    for k in ["now", "target", "edge", "time", "ttl", "start", "spw"]:
        np.testing.assert_array_equal(st[k], g[k][si], err_msg=f"snapshot {si} field {k}")
    np.testing.assert_array_equal(st["size"].view(np.uint64), g["size"][si].view(np.uint64),
                                  err_msg=f"snapshot {si} size bits")
    np.testing.assert_array_equal(st["agent_steps"], g["agent_steps"][si], err_msg=f"snapshot {si} agent_steps")
    np.testing.assert_array_equal(st["loads"][:E].view(np.uint64), g["loads"][si][:E].view(np.uint64),
                                  err_msg=f"snapshot {si} loads (fp64 bits)")
    vis = g["visited"][si]
    got = st["visited"]
    got_lo = got[:, 0] if got.ndim == 2 else got
    np.testing.assert_array_equal(got_lo, vis, err_msg=f"snapshot {si} visited")
    assert st["topo_seed"] == g["topo_seed"][si], f"snapshot {si} topology seed"
    if "amask" in st:
        np.testing.assert_array_equal(st["amask"], g["action_mask"][si], err_msg=f"snapshot {si} action mask")
    assert sha(ob["obs"]) == g["obs_sha"][si], f"snapshot {si}: agent obs differs"
    assert sha(ob["node_obs"]) == g["nodeobs_sha"][si], f"snapshot {si}: node obs differs"
    if ob.get("adj") is not None:
        assert sha(ob["adj"]) == g["adj_sha"][si], f"snapshot {si}: agent adjacency differs"
    assert sha(ob["node_agent"]) == g["nodeagent_sha"][si], f"snapshot {si}: node-agent matrix differs"
    if f"full_obs_{si}" in g.files:
        np.testing.assert_array_equal(ob["obs"], g[f"full_obs_{si}"])
        np.testing.assert_array_equal(ob["node_obs"], g[f"full_nodeobs_{si}"])


def replay(path, make_env, max_steps=None):
    """make_env(cfg_dict, topo_spec) -> adapter. Returns number of checked snapshots."""
    g, cfg = load(path)
    n, A = int(cfg["n"]), int(cfg["a"])
    seedlist = None
    if cfg["mode"] == "list":
        t = np.load(os.path.join(GOLDEN, "topology.npz"))
        seedlist = t[f"seedlist_n{n}_i{int(cfg['topo'])}"][:5] if f"seedlist_n{n}_i{int(cfg['topo'])}" in t.files else None
        if seedlist is None:
            raise KeyError("list seeds")
    env = make_env(cfg, topo_spec(cfg, seedlist))
    env.reset()
    si = 0
    check_snapshot(g, si, env.state(), env.observe(), n, A)
    si += 1
    T = int(cfg["T"]) if max_steps is None else min(max_steps, int(cfg["T"]))
    ep, ep_step = int(cfg["ep"]), 0
    eps = float(cfg["eps"])
    lists = {"delays": [], "delays_arrived": [], "spr": []}
    final = []
    for t in range(1, T + 1):
        if eps >= 0:
            act = env.egreedy(g["q"][t - 1], eps)
            np.testing.assert_array_equal(act, g["actions"][t - 1], err_msg=f"step {t} egreedy actions")
        else:
            act = g["actions"][t - 1]
        rew, done, info = env.step(act)
        np.testing.assert_array_equal(rew.view(np.uint32), g["reward"][t - 1].view(np.uint32),
                                      err_msg=f"step {t} reward")
        np.testing.assert_array_equal(done.astype(np.int64), g["done"][t - 1], err_msg=f"step {t} done")
        assert info["looped"] == g["info_looped"][t - 1], t
        assert info["throughput"] == g["info_throughput"][t - 1], t
        assert info["dropped"] == g["info_dropped"][t - 1], t
        assert info["blocked"] == g["info_blocked"][t - 1], t
        if "delays" in info:
            for k in lists:
                lists[k].extend(info[k])
        assert g["kind"][si] == 0 and g["step"][si] == t
        check_snapshot(g, si, env.state(), env.observe(), n, A)
        si += 1
        ep_step += 1
        if ep_step >= ep:
            final.extend(env.final_delays() + [-1.0])
            env.reset()
            ep_step = 0
            assert g["kind"][si] == 1 and g["step"][si] == t
            check_snapshot(g, si, env.state(), env.observe(), n, A)
            si += 1
    if max_steps is None:
        for k in lists:
            if lists[k] or len(g["list_" + k]):
                np.testing.assert_array_equal(np.array(lists[k], np.float64), g["list_" + k], err_msg=k)
        np.testing.assert_array_equal(np.array(final, np.float64), g["final_delays"])
    return si
