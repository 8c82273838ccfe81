#!/usr/bin/env python3
"""Benchmark: routing env-steps/s with NetMon on MI355X (BASELINE.json metric).

One step = one vectorised rollout step over n_env graph instances on each GPU:
DQN Q-values on the joint observation -> ε-greedy draws -> Routing.step ->
NetMon step (encoder, LSTM obs cell, K x (aggregate + LSTM update), readout into
the joint observation), plus the episode resets (new random topology + NetMon
start-up) every --episode-steps steps, exactly like the reference's training
rollout (src/main.py:667-748) with NetMonWrapper (src/env/wrapper.py).

Multi-GPU: one process per GPU (torchrun), env shards with disjoint seeds, no
collective on the rollout path (weak scaling); barrier + max-over-ranks timing.
Rank 0 prints ONE JSON line. `python bench.py --gpus N` (N > 1) outside a launcher starts
`torch.distributed.run --nproc-per-node N` on this script as a child process (before any GPU
call) and exits with its return code; under a launcher WORLD_SIZE must equal --gpus.
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec (routing, --netmon, 20-node graphs) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
F32_MFMA_PEAK_TFS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA dense peak
F16_MFMA_PEAK_TFS = 16 * 157.3  # MI355X_MICROARCH.md: BF16/F16 dense = 16x the f32-input MFMA rate


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--n-env", type=int, default=4096)
    p.add_argument("--n-router", type=int, default=20)
    p.add_argument("--n-data", type=int, default=20)
    p.add_argument("--netmon-iterations", type=int, default=1)
    p.add_argument("--netmon-rnn-type", default="lstm", choices=["lstm", "lnlstm", "gru"])
    p.add_argument("--no-netmon", action="store_true",
                   help="DQN on the env observation alone (BASELINE config 2: the reference without --netmon)")
    p.add_argument("--episode-steps", type=int, default=50)
    p.add_argument("--random-topology", type=int, default=1)
    p.add_argument("--epsilon", type=float, default=0.5)
    p.add_argument("--no-kernel-timers", action="store_true")
    p.add_argument("--graph", type=int, default=10,
                   help="replay the rollout as HIP graphs of this many (even) vector steps, one graph per stream "
                        "group on its own stream (0: eager launches; DESIGN.md §9.5: host enqueue 0.36 -> 0.02 ms "
                        "per step, rollout +0.5 %%)")
    p.add_argument("--graph-single", action="store_true",
                   help="with --graph: every group in ONE graph (default: one graph per group on its own stream)")
    p.add_argument("--stagger", action="store_true",
                   help="stagger the stream groups' episodes so their resets overlap the other group's GEMMs "
                        "(measured neutral at 4096 envs: the reset is ~2%% of a 50-step episode)")
    p.add_argument("--groups", type=int, default=2,
                   help="env groups on separate HIP streams (graph-marl_amd/rollout.py StreamedRollout)")
    p.add_argument("--unfused", action="store_true", help="materialise the joint obs; separate LSTM/aggregate kernels")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-f32-compare", action="store_true",
                   help="skip the second timed pass with the exact-fp32 GEMM form (GM_GEMM=f32)")
    p.add_argument("--no-train", action="store_true", help="skip the rollout + training measurement")
    p.add_argument("--train-steps", type=int, default=5, help="timed vector steps of rollout + update")
    p.add_argument("--train-batch", type=int, default=0,
                   help="sequences per update (0: 32 * n_env / 10 = the reference replay ratio, SURVEY 8d)")
    p.add_argument("--train-seq", type=int, default=8, help="sequence length of an update")
    p.add_argument("--train-autograd", action="store_true",
                   help="training leg on the per-step autograd path (train.dqn_update) instead of train_seq")
    p.add_argument("--no-extras", action="store_true",
                   help="skip the other BASELINE configurations (K=3, configs 2/3, config 5 SL) timed after the headline")
    p.add_argument("--extra-steps", type=int, default=100, help="timed vector steps of each extra rollout configuration")
    p.add_argument("--no-config4", action="store_true",
                   help="skip the config-4 leg (4096 envs in total over the GPUs, N = 10..50, rollout + training)")
    p.add_argument("--config4-train-steps", type=int, default=2, help="timed rollout + update steps per config-4 size")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the same-run rocprofv3 PMC passes (HBM bytes of DQN layer 1 and k_env_step)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    p.add_argument("--pmc-order", default=None, help=argparse.SUPPRESS)
    p.add_argument("--cpu-envs", type=int, default=1024)
    p.add_argument("--cpu-steps", type=int, default=50, help="one full episode (includes its reset)")
    return p.parse_args()


def pmc_traffic(tag, build_src=None):
    """HBM bytes per launch of a kernel (FETCH_SIZE x2 + WRITE_SIZE) from a committed rocprofv3 PMC
    profile (profiles/*/*/pmc_traffic.json), with a provenance note. A profile whose recorded source
    hash equals this library's build.src wins; otherwise the newest one (round directory, then the
    profile's "seq", then its file time), never the largest byte count. (None, None) when no profile
    has the kernel. Used only when the same-run passes (measure_pmc) are unavailable."""
    import glob

    found = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "*", "*", "pmc_traffic.json")):
        try:
            with open(path) as f:
                d = json.load(f)
            k = d["kernels"].get(tag)
            mtime = os.path.getmtime(path)
        except (OSError, ValueError, KeyError):
            continue
        if k:
            rnd = os.path.basename(os.path.dirname(os.path.dirname(path)))
            psrc = d.get("src")
            rank = (build_src is not None and psrc == build_src, rnd, d.get("seq", 0), mtime)
            found.append((rank, k["fetch_bytes"] + k["write_bytes"], os.path.relpath(path, ROOT), psrc))
    if not found:
        return None, None
    _, tb, src, psrc = max(found, key=lambda f: f[0])
    same = ("source hash not recorded" if psrc is None else
            "same sources as this build" if psrc == build_src else f"OTHER sources ({psrc}) than this build")
    return tb, f"committed profile {src}, {same}"


PMC_S = 6  # rollout vector steps in the counted window of the --pmc-child process


def pmc_child(args):
    """The dispatch window the PMC passes count (bench.py under rocprofv3, started by measure_pmc): the
    headline's rollout as ONE group (the same kernels and launch sizes as the per-kernel timer pass),
    positioned so that the window holds no episode reset; one step records the library's launch order
    (_lib.TRACE, written to --pmc-order), then PMC_S more steps run with nothing in between."""
    torch.cuda.set_device(0)
    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    RO = importlib.import_module("graph-marl_amd.rollout")
    L = gm._lib
    N, A, B = args.n_router, args.n_data, args.n_env
    assert args.episode_steps > PMC_S + 6, "the PMC window must fit inside one episode"
    net = gm.Network(N, random_topology=bool(args.random_topology), excluded_seeds=gm.EVAL_SEEDS, device=0)
    torch.manual_seed(0)
    netmon = M.NetMon(4 * N + 8, 128, [512, 256], args.netmon_iterations).cuda()
    dqn = M.DQN(6 * N + 10 + netmon.get_out_features(), [512, 256], 4).cuda()
    M.tag_modules(netmon, "netmon.")
    M.tag_modules(dqn, "dqn.")
    ro = RO.StreamedRollout(net, A, B, netmon, dqn, groups=1, seed=0, epsilon=args.epsilon,
                            episode_steps=args.episode_steps, device=0)
    with torch.no_grad():
        ro.reset()
        ro.run(3)
        torch.cuda.synchronize()
        L.TRACE = []
        ro.step()
        order, L.TRACE = L.TRACE, None
        for _ in range(PMC_S - 1):
            ro.step()
        torch.cuda.synchronize()
    assert ro.ep == 3 + PMC_S, "an episode reset fell inside the PMC window"
    with open(args.pmc_order, "w") as f:
        json.dump(order, f)


def _pmc_window(path, counter, order):
    """Per-launch counter values of every rollout kernel from the child's CSV: the last PMC_S x len(order)
    dispatches of this library's kernels must be PMC_S repetitions of one step's launches (same kernel
    names, the env step and the aggregate where `order` has them). Returns ({tag: median value per launch},
    median over the steps of the per-step sum), or None if the window does not look like that."""
    import csv

    with open(path) as f:
        rows = [r for r in csv.DictReader(f) if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    ours = [r for r in rows if r["Kernel_Name"].lstrip("_ ").startswith(("k_", "ZN12_GLOBAL__N_1"))]
    P = len(order)
    win = ours[-(PMC_S * P):] if P else []
    if P == 0 or len(win) != PMC_S * P:
        return None
    names = [r["Kernel_Name"] for r in win]
    if any(names[i] != names[i % P] for i in range(len(win))):
        return None
    for i, tag in enumerate(order):
        for kind, kname in (("env_step", "k_env_step"), ("mp_aggregate", "k_mp_aggregate")):
            if tag.split(":")[0] == kind and kname not in names[i]:
                return None
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    vals = {}
    for i, tag in enumerate(order):
        vals.setdefault(tag, []).extend(float(win[s * P + i]["Counter_Value"]) for s in range(PMC_S))
    per_step = [sum(float(win[s * P + i]["Counter_Value"]) for i in range(P)) for s in range(PMC_S)]
    return {tag: med(v) for tag, v in vals.items()}, med(per_step)


def measure_pmc(args):
    """Same-run HBM traffic (MI355X_MICROARCH.md §HBM) of EVERY rollout kernel: two rocprofv3 passes over a
    child bench.py (--pmc-child), FETCH_SIZE and WRITE_SIZE in separate runs (they do not fit one pass),
    each under a hard time limit; KiB per launch, FETCH_SIZE doubled (gfx950 counts half of a 16-B/lane
    stream). Returns {"kernels": {tag: bytes per launch}, "step_bytes": bytes per vector step (one group of
    --n-env envs), ...} or None (no rocprofv3); {"error": ...} if a pass failed."""
    import shutil
    import tempfile

    prof = shutil.which("rocprofv3")
    if prof is None:
        return None
    out, steps = {}, {}
    with tempfile.TemporaryDirectory(dir=os.path.join(ROOT, "gpurun_out") if os.path.isdir(
            os.path.join(ROOT, "gpurun_out")) else None) as d:
        order_path = os.path.join(d, "order.json")
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", counter, "-T", "--output-format", "csv", "-d", d,
                   "-o", counter.lower(), "--", sys.executable, os.path.abspath(__file__), "--pmc-child",
                   "--pmc-order", order_path,
                   "--n-env", str(args.n_env), "--n-router", str(args.n_router), "--n-data", str(args.n_data),
                   "--netmon-iterations", str(args.netmon_iterations), "--random-topology", str(args.random_topology),
                   "--episode-steps", str(args.episode_steps), "--epsilon", str(args.epsilon)]
            try:
                r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=170)
            except subprocess.TimeoutExpired:
                return {"error": f"{counter} pass timed out"}
            if r.returncode != 0:
                return {"error": f"{counter} pass rc {r.returncode}: {r.stderr.decode(errors='replace')[-200:]}"}
            try:
                with open(order_path) as f:
                    order = json.load(f)
            except (OSError, ValueError):
                return {"error": f"{counter}: the child wrote no launch order"}
            csvs = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs
                    if f.startswith(counter.lower()) and f.endswith("counter_collection.csv")]
            got = _pmc_window(csvs[0], counter, order) if csvs else None
            if got is None:
                return {"error": f"{counter}: dispatch window not found in {csvs}"}
            f = 2.0 if counter == "FETCH_SIZE" else 1.0
            out[counter] = {tag: f * v * 1024 for tag, v in got[0].items()}
            steps[counter] = f * got[1] * 1024
    kernels = {tag: round(out["FETCH_SIZE"][tag] + out["WRITE_SIZE"].get(tag, 0.0)) for tag in out["FETCH_SIZE"]}
    return {"kernels": kernels, "step_bytes": round(steps["FETCH_SIZE"] + steps["WRITE_SIZE"]),
            "fetch_bytes": {t: round(v) for t, v in out["FETCH_SIZE"].items()},
            "write_bytes": {t: round(v) for t, v in out["WRITE_SIZE"].items()},
            "window": f"{PMC_S} rollout vector steps of one group of {args.n_env} envs, no reset inside",
            "note": f"rocprofv3 PMC in this bench run (child process, median of {PMC_S} steps; FETCH_SIZE x2, "
                    "KiB x1024)"}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def kernel_cost(tag, n_env, N, A, E, x3=False):
    """(bound, algorithmic units per launch) for a timer tag — DESIGN.md §4. GEMMs in the
    split-f16 form count the MFMA work they issue: 3 f16 products per fp32 multiply-add."""
    kind = tag.split(":")[0]
    if kind in ("linear", "lstm", "lstm_agg"):
        m, n, k = (int(v) for v in tag.split(":")[2].split("x"))
        macs = m * n * k + (m * 128 * n if "+chain" in tag else 0)  # gm_encoder_x3: + layer 3 (n -> 128)
        return ("mfma16" if x3 and n > 32 else "mfma"), (3.0 if x3 and n > 32 else 1.0) * 2.0 * macs
    if kind == "routing_enc":
        rows, n = (int(v) for v in tag.split(":")[2].split("x"))
        return "hbm", rows * n * 4 + rows * 11 * 4  # write y, read the 11 nonzero features per row
    if kind == "mp_aggregate":
        rows, H = (int(v) for v in tag.split(":")[1].split("x"))
        return "hbm", rows * H * 4 * 2 + rows * 3 * 4  # read h, write M, read nbr
    if kind == "netmon_readout":
        rows, w = (int(v) for v in tag.split(":")[1].split("x"))
        return "hbm", rows * w * 4 * 2 + rows * 4  # gather-read + write + index
    if kind == "lstm_pointwise":
        rows, H = (int(v) for v in tag.split(":")[1].split("x"))
        return "hbm", rows * H * 4 * (4 + 1 + 2)  # gates, c in; h, c out
    if kind == "env_step":
        # SURVEY §8(d) B_env: compact state (78A + 22E + 12N) + materialised fp32 obs (19 900 B
        # at N = A = 20), plus the ε-greedy prologue's Q rows, actions and RNG words per agent
        # (gm_env_policy_step). The GEMM-ready duplicate of the agent rows is NOT algorithmic
        # (env_step_overhead_bytes)
        b_state = 78 * A + 22 * E + 12 * N
        b_obs = 4 * A * (6 * N + 10) + 4 * N * (4 * N + 8)
        b_pol = A * (16 + 4 + 12) if _fused_policy_step() else 0
        return "hbm", float(n_env * (b_state + b_obs + b_pol))
    if kind == "egreedy":
        return "hbm", float(n_env * A * (16 + 4 + 12))
    return None, None


def env_step_overhead_bytes(n_env, N, A):
    """Bytes k_env_step writes beyond SURVEY §8(d)'s B_env: the GEMM-ready copy of the agent
    rows (gm_obs_buffers.obs_gemm) that DQN layer 1 reads at K = 512 + 6N + 8, when the env writes
    both copies (the rollout's lazy-obs envs write only that copy: no overhead)."""
    return float(n_env * 4 * A * (6 * N + 8)) if _gemm_obs() else 0.0


def _fused_policy_step():
    import importlib
    return importlib.import_module("graph-marl_amd.policy").FUSED_POLICY_STEP


_GEMM_OBS_ON = [False]  # set from the timed rollout's env (Routing.obs_gemm allocated)


def _gemm_obs():
    return _GEMM_OBS_ON[0]


def sl_gemm_flops(N, B, L, K, H=128, enc=(512, 256)):
    """f16 MFMA FLOPs one config-5 SL iteration issues on its split-f16 GEMMs (3 f16 products per
    fp32 multiply-add; forward, input gradient and weight gradient of each GEMM): per node row the
    encoder layers 1..2 once per iteration (enc[0]->enc[1]->H; layer 0 is the routing gather, no
    GEMM; sl.train_step encodes the unrolled steps' shared observations once), and per step the LSTM
    obs cell [x | h] (2H -> 4H) and K update cells (2H -> 4H). The three narrow output heads (exact
    f32) are left out."""
    macs = (enc[0] * enc[1] + enc[1] * H) + L * (1 + K) * 2 * H * 4 * H
    return 3.0 * 2.0 * 3.0 * macs * N * B


def measure_extras(args, gm, M, RO, timed_region, dev, N, A, x3):
    """The other BASELINE.json configurations, timed in the same process after the headline:
    NetMon with the CLI default --netmon-iterations 3 (src/main.py:153-157), config 3 (fixed
    20-node topology, seed 476), config 2 (no NetMon, fixed topology, 1024 envs) and config 5
    (src/sl.py at N = 100, batch 8192, sequence length 8, NetMon K = 1)."""
    out = {}
    steps = args.extra_steps

    def rollout(name, n_env, K, random_topology, netmon_on, desc):
        try:
            net = gm.Network(N, random_topology=random_topology, excluded_seeds=gm.EVAL_SEEDS, device=dev.index)
            torch.manual_seed(0)
            nm = M.NetMon(4 * N + 8, 128, [512, 256], K).to(dev) if netmon_on else None
            dq = M.DQN(6 * N + 10 + (nm.get_out_features() if nm is not None else 0), [512, 256], 4).to(dev)
            ro = RO.StreamedRollout(net, A, n_env, nm, dq, groups=args.groups, seed=0, epsilon=args.epsilon,
                                    episode_steps=args.episode_steps, device=dev.index)
            g = args.graph if args.graph and steps % args.graph == 0 else 0  # the headline's launch mode
            el, _ = timed_region(5, steps, False, ro=ro, graph=g)
            out[name] = {"value": round(n_env * steps / el, 1), "unit": "env-steps/s",
                         "ms_per_step": round(1e3 * el / steps, 4), "steps": steps, "n_env": n_env, "graph": g,
                         "resets_in_window": -(-steps // args.episode_steps), "workload": desc}
            del ro, nm, dq
        except Exception as ex:  # an extra configuration must never break the headline line
            if os.environ.get("GM_BENCH_RAISE") == "1":
                raise
            out[name] = {"value": None, "error": repr(ex)[:300]}
        torch.cuda.empty_cache()

    rollout("netmon_k3", args.n_env, 3, True, True,
            f"headline with the CLI default --netmon-iterations 3: random {N}-node topologies, NetMon K=3")
    rollout("config3_fixed_topology", args.n_env, 1, False, True,
            f"config 3: --random-topology 0 (fixed {N}-node graph, seed 476), NetMon K=1")
    rollout("config2_no_netmon", 1024, 1, False, False,
            f"config 2: --random-topology 0, no NetMon, DQN 512,256 on the env obs, 1024 envs")
    try:
        SL = importlib.import_module("graph-marl_amd.sl")
        n, b, sl_len, k = 100, 8192, 8, 1
        line = SL.main(["--bench", "--n-nodes", str(n), "--batch-size", str(b), "--sequence-length", str(sl_len),
                        "--netmon-iterations", str(k), "--iterations", "3", "--warmup", "2"], quiet=True)
        sec = line["ms_per_iteration"] * 1e-3
        fl = sl_gemm_flops(n, b, sl_len, k) if x3 else None
        line["roofline"] = None if fl is None else {
            "kernel": "all GEMMs of one iteration (fwd + input grad + weight grad), iteration wall time",
            "bound": "mfma", "achieved": round(fl / sec / 1e12, 2), "peak": F16_MFMA_PEAK_TFS,
            "unit": "TFLOP/s (f16 MFMA, 3 per fp32 multiply-add)", "frac": round(fl / sec / 1e12 / F16_MFMA_PEAK_TFS, 4),
            "traffic": None}
        out["config5_sl"] = line
    except Exception as ex:
        if os.environ.get("GM_BENCH_RAISE") == "1":
            raise
        out["config5_sl"] = {"value": None, "error": repr(ex)[:300]}
    torch.cuda.empty_cache()
    return out


def measure_train(args, gm, M, W, P, net, netmon, dqn, dev, world, rank, n_env=None, steps=None):
    """Rollout + DQN/NetMon training at the reference's replay ratio: every
    vector step of ALL n_env envs of the GPU (one env batch, one stream) stores its n_env
    transitions in the device replay and runs one update of B sequences x L steps
    (B = 32 n_env / 10: the paper's B=32, L=8 update every 10 env-steps, per env), with the
    gradient all-reduce across ranks (src/main.py:667-1026; graph-marl_amd/train.py).
    Value = env-steps/s of the whole loop (all ranks). n_env / steps default to --n-env / --train-steps."""
    import copy

    import importlib as il

    T = il.import_module("graph-marl_amd.train")
    TS = il.import_module("graph-marl_amd.train_seq")
    RB = il.import_module("graph-marl_amd.replaybuffer")
    B = n_env or args.n_env
    n_steps = steps or args.train_steps
    env = gm.Routing(net, args.n_data, n_env=B, seed=rank * B, obs_extra=netmon.get_out_features(),
                     agent_adjacency=False, device=dev.index)
    wenv = W.NetMonWrapper(env, netmon, 1)
    policy = P.EpsilonGreedy(wenv, dqn, epsilon=args.epsilon, epsilon_decay=1.0, epsilon_update_freq=100,
                             step_before_train=0)
    bsz = args.train_batch or max(1, (32 * B + 9) // 10)
    L_ = args.train_seq
    model_tar = copy.deepcopy(dqn)
    params = list(dqn.parameters()) + list(netmon.parameters())
    opt = torch.optim.AdamW(params, lr=1e-4)
    T.broadcast_parameters([dqn, netmon])
    slots = L_ + 8
    buff = RB.ReplayBuffer(0, slots * B, B, env.n_data, env.obs_dim, env.n_nodes, env.node_obs_dim,
                           netmon.get_state_size(), dev, nbr_width=env.nbr.shape[-1])
    ep = {"n": 0}
    seq_path = not args.train_autograd and TS.seq_ok(netmon, dqn, model_tar)

    def vstep(update):
        if ep["n"] == 0:
            wenv.reset()
        buff.add_pre(env.obs, wenv.last_netmon_state, env.node_obs, env.nbr, env.agent_node)
        with torch.no_grad():
            act = policy.act_step(wenv)
        ep["n"] += 1
        done_ep = ep["n"] >= args.episode_steps
        buff.add_post(act, env.reward, env.obs, env.done.bool(), done_ep, env.node_obs, env.agent_node)
        if done_ep:
            ep["n"] = 0
        if update:
            dqn.train()
            netmon.train()
            if seq_path:  # sequence-batched update with the hand-written backward (train_seq.py)
                TS.dqn_update_seq(netmon, dqn, model_tar, opt, params, buff.get_sequences(bsz, L_), 0.98, 0.01)
            else:
                batches = list(buff.get_batch(bsz, sequence_length=L_, lazy_next=True))
                T.dqn_update(netmon, dqn, model_tar, opt, params, batches, 0.98, 0.01, consecutive=True)
            dqn.eval()
            netmon.eval()
            netmon.state = None

    for _ in range(L_ + 2):  # fill the replay past one sequence
        vstep(False)
    vstep(True)  # warm-up update
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(n_steps):
        vstep(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    share = os.environ.get("GM_BENCH_SHARE_GPU") == "1"
    t = torch.tensor([el], dtype=torch.float64, device="cpu" if share else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    return {"value": round(B * world * n_steps / el, 1), "unit": "env-steps/s", "n_env_per_gpu": B,
            "ms_per_step": round(1e3 * el / n_steps, 3), "steps": n_steps,
            "update": {"sequences": bsz, "seq_len": L_, "graph_steps": bsz * L_,
                       "path": "train_seq (sequence-batched)" if seq_path else "train.dqn_update (autograd)",
                       "per": "vector step of n_env envs (replay ratio 25.6 = reference B=32, L=8 every 10 steps)"}}


CONFIG4_NODES = (10, 20, 30, 40, 50)
CONFIG4_TOTAL_ENVS = 4096


def measure_config4(args, gm, M, W, P, RO, timed_region, dev, world, rank):
    """BASELINE config 4 as defined: --netmon --random-topology 1 at 10-50-node random graphs, 4096 envs IN
    TOTAL sharded over the ranks (4096 / world per GPU: strong scaling), rollout alone and rollout + training
    with the gradient all-reduce (src/main.py:840-1006 wrapped by train.allreduce_gradients), one run per
    node count (scripts/start_routing_netmon_runs.sh:32-50 runs the random-topology NetMon jobs at these
    sizes). Every rank takes part in every timed region (barriers, max-over-ranks time). The rollout window
    is one 50-step episode (one topology reset + NetMon start-up, the reference's rate); the training
    window --config4-train-steps vector steps, each with one update at the reference's replay ratio."""
    out = {"workload": "config 4: --netmon --random-topology 1, NetMon K=1 H=128 enc 512,256 lstm + DQN 512,256, "
                       f"{CONFIG4_TOTAL_ENVS} envs in total over {world} GPU(s)",
           "total_envs": CONFIG4_TOTAL_ENVS, "envs_per_gpu": CONFIG4_TOTAL_ENVS // world, "n_gpus": world,
           "scaling": "strong (total envs fixed)", "unit": "env-steps/s", "per_n_nodes": {}}
    B = CONFIG4_TOTAL_ENVS // world
    for n in CONFIG4_NODES:
        rec = {}
        try:
            net = gm.Network(n, random_topology=True, excluded_seeds=gm.EVAL_SEEDS, device=dev.index)
            torch.manual_seed(0)
            nm = M.NetMon(4 * n + 8, 128, [512, 256], 1).to(dev)
            dq = M.DQN(6 * n + 10 + nm.get_out_features(), [512, 256], 4).to(dev)
            ro = RO.StreamedRollout(net, args.n_data, B, nm, dq, groups=args.groups, seed=rank * B, epsilon=args.epsilon,
                                    episode_steps=args.episode_steps, device=dev.index)
            g = args.graph if args.graph and args.episode_steps % args.graph == 0 else 0
            el, _ = timed_region(5, args.episode_steps, False, ro=ro, graph=g)
            rec["rollout"] = round(B * world * args.episode_steps / el, 1)
            rec["rollout_ms_per_step"] = round(1e3 * el / args.episode_steps, 4)
            del ro
            tr = measure_train(args, gm, M, W, P, net, nm, dq, dev, world, rank, n_env=B, steps=args.config4_train_steps)
            rec["rollout_train"] = tr["value"]
            rec["rollout_train_ms_per_step"] = tr["ms_per_step"]
            rec["update_sequences"] = tr["update"]["sequences"]
            del nm, dq, net
        except Exception as ex:  # a config-4 size must never break the headline line
            if os.environ.get("GM_BENCH_RAISE") == "1":
                raise
            rec = {"value": None, "error": repr(ex)[:300]}
        if world > 1:
            # every rank reaches this exchange whether its size passed or failed (a failure at a size is
            # normally the same on every rank: memory, an unsupported shape), so the ranks skip a failed
            # size together and go on to the next one and to the headline line
            flag = torch.tensor([0.0 if "error" not in rec else 1.0], dtype=torch.float64,
                                device="cpu" if os.environ.get("GM_BENCH_SHARE_GPU") == "1" else dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            if float(flag.item()) > 0 and "error" not in rec:
                rec = {"value": None, "error": "skipped: another rank failed at this size"}
        out["per_n_nodes"][str(n)] = rec
        torch.cuda.empty_cache()
    out["rollout_steps"] = args.episode_steps
    out["train_steps"] = args.config4_train_steps
    return out


def launch_ranks(args, argv=None):
    """--gpus N > 1 without a launcher: run N ranks of this script under torch.distributed.run as a
    CHILD process (nothing here has touched the GPU; no exec from this process) and return its exit
    code. Returns None when this process is already a rank (WORLD_SIZE set) or N == 1."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)]
    cmd += list(sys.argv[1:] if argv is None else argv)
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def check_world(args, world):
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} ranks were launched")


def main():
    args = parse()
    if args.pmc_child:
        return pmc_child(args)
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    check_world(args, world)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GM_BENCH_SHARE_GPU=1 rehearses the N-rank path on one GPU (all ranks on cuda:0, gloo)
    share = os.environ.get("GM_BENCH_SHARE_GPU") == "1"
    if world > 1:
        import datetime

        gpu = 0 if share else local
        torch.cuda.set_device(gpu)
        timeout = datetime.timedelta(seconds=float(os.environ.get("GM_DIST_TIMEOUT", "900")))
        if share:
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu), timeout=timeout)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    gm = importlib.import_module("graph-marl_amd")
    M = importlib.import_module("graph-marl_amd.model")
    W = importlib.import_module("graph-marl_amd.wrapper")
    P = importlib.import_module("graph-marl_amd.policy")
    L = gm._lib

    N, A, B, K = args.n_router, args.n_data, args.n_env, args.netmon_iterations
    E = 3 * N // 2
    net = gm.Network(N, random_topology=bool(args.random_topology), excluded_seeds=gm.EVAL_SEEDS,
                     device=dev.index)
    torch.manual_seed(0)
    netmon = None if args.no_netmon else M.NetMon(4 * N + 8, 128, [512, 256], K, rnn_type=args.netmon_rnn_type).to(dev)
    dqn = M.DQN(6 * N + 10 + (0 if netmon is None else netmon.get_out_features()), [512, 256], 4).to(dev)
    if netmon is not None:
        M.tag_modules(netmon, "netmon.")
    M.tag_modules(dqn, "dqn.")
    RO = importlib.import_module("graph-marl_amd.rollout")
    ro = RO.StreamedRollout(net, A, B, netmon, dqn, groups=args.groups, seed=rank * B, epsilon=args.epsilon,
                            episode_steps=args.episode_steps, device=dev.index,
                            stagger=args.stagger, stagger_quantum=args.graph or 1)
    _GEMM_OBS_ON[0] = ro.envs[0].obs_gemm is not None and not ro.envs[0]._lazy_obs  # both copies written
    if args.unfused:
        for w in ro.wenvs:
            w.fused = False

    state = {}

    def timed_region(warmup, steps, timers, ro=ro, graph=0):
        """W warmup steps, then untimed steps up to the episode phase where the FIRST timed step
        (graph: replay) ends an episode, so the K timed steps always contain ceil(K / episode)
        topology resets + NetMon start-ups (at the reference's rate or above, whatever K is)."""
        EP = args.episode_steps
        g = graph or 1
        with torch.no_grad():
            ro.reset()
            # graph replays start at multiples of the captured length: warm up to one
            for _ in range(-(-warmup // graph) * graph if graph else warmup):
                ro.step()
            if graph:
                # capture after the eager warmup (packed weights, scratch buffers exist), then
                # one untimed replay; the timed loop replays steps/graph graphs
                assert steps % graph == 0, "--steps must be a multiple of --graph"
                ro.capture(graph, per_group=not args.graph_single)
                ro.run(graph)
            while ro.ep != EP - g:  # position: the first timed step (replay) triggers a reset
                ro.run(g) if graph else ro.step()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            if timers:
                L.PROF = {}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if graph:
                ro.run(steps)
            else:
                for _ in range(steps):
                    ro.step()
            t_issue = time.perf_counter() - t0  # host time to enqueue the steps
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            elapsed = time.perf_counter() - t0
            prof, L.PROF = L.PROF, None
            state["host_ms_per_step"] = 1e3 * t_issue / steps
            state["resets"] = -(-steps // EP)
        el = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if share else dev)
        if world > 1:
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item()), prof

    x3 = L.GEMM_MODE == "x3"
    G = args.groups
    # headline: the groups run concurrently, no per-kernel events in the timed region
    timers = not args.no_kernel_timers
    elapsed, prof = timed_region(args.warmup, args.steps, timers and G == 1 and not args.graph, graph=args.graph)
    host_ms = state["host_ms_per_step"]
    resets = state["resets"]
    if timers and (G > 1 or args.graph):
        # per-kernel durations from the same rollout as ONE group (kernels not overlapped), for
        # the roofline fields and the rocprofv3 cross-check (tools/gpu_check.sh prof: --groups 1)
        ro1 = RO.StreamedRollout(net, A, B, netmon, dqn, groups=1, seed=rank * B, epsilon=args.epsilon,
                                 episode_steps=args.episode_steps, device=dev.index)
        _, prof = timed_region(5, min(args.steps, 100), True, ro=ro1)
        del ro1
    total = B * world * args.steps
    value = total / elapsed
    f32cmp = None
    if x3 and world == 1 and not args.no_f32_compare:
        # the same rollout with every GEMM in the exact-fp32 form, for reference
        L.GEMM_MODE = "f32"
        el32, _ = timed_region(5, args.steps, False)
        L.GEMM_MODE = "x3"
        f32cmp = {"value": round(B * args.steps / el32, 1), "ms_per_step": round(1e3 * el32 / args.steps, 4)}

    kernels = {}
    if prof:
        for tag, evs in prof.items():
            ts = [s.elapsed_time(e) for s, e in evs]
            kernels[tag] = {"launches": len(ts), "avg_us": 1e3 * sum(ts) / len(ts), "total_ms": sum(ts)}
    roof = None
    roof_hbm = {}
    if kernels:
        dom = max(kernels, key=lambda k: kernels[k]["total_ms"])
        bound, units = kernel_cost(dom, B, N, A, E, x3)
        sec = kernels[dom]["avg_us"] * 1e-6
        if bound in ("mfma", "mfma16"):
            ach = units / sec / 1e12
            peak = F16_MFMA_PEAK_TFS if bound == "mfma16" else F32_MFMA_PEAK_TFS
            tb, src = pmc_traffic(dom, L.build_info().get("src"))
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": peak,
                    "unit": "TFLOP/s" + (" (f16 MFMA, 3 per fp32 multiply-add)" if bound == "mfma16" else " (f32 MFMA)"),
                    "frac": round(ach / peak, 4), "traffic": tb,
                    "traffic_note": None if tb is None else f"HBM bytes per launch (rocprofv3 PMC, {src})"}
        else:
            ach = units / sec / 1e9
            roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
        for tag, kv in kernels.items():
            bound, units = kernel_cost(tag, B, N, A, E, x3)
            if bound:
                s = kv["avg_us"] * 1e-6
                kv["achieved"] = round(units / s / (1e9 if bound == "hbm" else 1e12), 2)
                kv["unit"] = {"hbm": "GB/s", "mfma": "TFLOP/s f32", "mfma16": "TFLOP/s f16"}[bound]
        # the two HBM-bound kernels the north star names: env step (+ obs emission) and the
        # message-passing aggregate; algorithmic bytes per launch / HIP-event time
        for tag, kv in kernels.items():
            if tag.split(":")[0] not in ("env_step", "mp_aggregate"):
                continue
            bound, units = kernel_cost(tag, B, N, A, E, x3)
            ach = units / (kv["avg_us"] * 1e-6) / 1e9
            tb, src = pmc_traffic(tag, L.build_info().get("src"))
            roof_hbm[tag] = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": units, "traffic": tb,
                             "traffic_note": None if tb is None else f"HBM bytes per launch (rocprofv3 PMC, {src})",
                             "avg_us": round(kv["avg_us"], 2)}
            if tag == "env_step":
                ov = env_step_overhead_bytes(B, N, A)
                roof_hbm[tag]["overhead_bytes"] = ov
                roof_hbm[tag]["overhead_note"] = ("GEMM-ready duplicate of the agent rows (obs_gemm), written by the "
                                                  "same launch, excluded from achieved/frac")

    extras = None
    if world == 1 and not args.no_extras and netmon is not None:
        extras = measure_extras(args, gm, M, RO, timed_region, dev, N, A, x3)

    train = None
    if not args.no_train and netmon is not None:
        try:
            train = measure_train(args, gm, M, W, P, net, netmon, dqn, dev, world, rank)
        except Exception as ex:  # the training figure must never break the rollout line
            if os.environ.get("GM_BENCH_RAISE") == "1":
                raise
            import traceback

            where = " <- ".join(f"{fs.name}:{fs.lineno}" for fs in traceback.extract_tb(ex.__traceback__)[::-1][:4])
            train = {"value": None, "error": repr(ex)[:300], "where": where}

    config4 = None
    if not args.no_config4 and netmon is not None and not args.no_extras:
        config4 = measure_config4(args, gm, M, W, P, RO, timed_region, dev, world, rank)
        if extras is None:
            extras = {}
        extras["config4"] = config4

    pmc = None
    if rank == 0 and world == 1 and not args.no_pmc and netmon is not None and args.netmon_rnn_type == "lstm":
        try:
            pmc = measure_pmc(args)
        except Exception as ex:  # the traffic probe must never break the GPU line
            pmc = {"error": repr(ex)[:200]}
    pk = (pmc or {}).get("kernels") or {}
    if roof and roof.get("kernel") in pk:
        roof["traffic"] = pk[roof["kernel"]]
        roof["traffic_note"] = "HBM bytes per launch, " + pmc["note"]
    for tag, kv in roof_hbm.items():
        if tag in pk:
            kv["traffic"] = pk[tag]
            kv["traffic_note"] = "HBM bytes per launch, " + pmc["note"]
    for tag, kv in kernels.items():
        if tag in pk:
            kv["traffic"] = pk[tag]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import cpu_baseline

            # the GPU box's CPU share of one GPU (its harness exports OMP_NUM_THREADS=16; nproc shows the
            # whole machine); in a plain environment every core
            threads = int(os.environ.get("OMP_NUM_THREADS") or (os.cpu_count() or 1))
            v, dt = cpu_baseline.measure(args.cpu_envs, args.cpu_steps, threads, K=K,
                                         episode_steps=args.episode_steps)
            cpu = {"value": round(v, 1), "unit": "env-steps/s", "cores": threads, "kind": "port",
                   "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
                   "sample": f"{args.cpu_envs} envs x {args.cpu_steps} steps ({dt:.1f} s): C oracle env (OpenMP) "
                             f"+ NumPy fp32 NetMon(K={K}) + DQN eps-greedy, same shapes"}
        except Exception as ex:  # the baseline must never break the GPU line
            cpu = {"value": None, "error": repr(ex)[:200]}

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": (f"f32 (GEMMs: 3xf16-split MFMA, A low piece scaled 2^{L.build_info().get('x3', '?')[2:]}, "
                      "f32 accumulate)") if x3 else "f32",
            "data": "synthetic: random-init NetMon+DQN weights, on-device random topologies and packets",
            "config": {"workload": ("routing rollout (no NetMon) + " if netmon is None else
                                    f"routing rollout --netmon (NetMon K={K}, H=128, enc 512,256, {args.netmon_rnn_type}, sum) + ") +
                                   f"DQN 512,256 eps-greedy, {'random' if args.random_topology else 'fixed'} "
                                   f"{N}-node topologies, episode {args.episode_steps} steps",
                       "n_env_per_gpu": B, "n_nodes": N, "n_data": A, "netmon_iterations": K,
                       "gemm_form": L.GEMM_MODE,
                       "parallelism": f"dp{world} (env shards, no rollout collective)",
                       "stream_groups": G, "graph_steps": args.graph,
                       "resets_in_window": resets},
            "host_enqueue_ms_per_step": round(host_ms, 4),
            "roofline": roof, "roofline_hbm": roof_hbm or None, "cpu_baseline": cpu, "f32_exact_gemms": f32cmp, "rollout_train": train,
            "other_configs": extras,
            "pmc": pmc,
            "kernels": kernels,
            "build": L.build_info(),
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
