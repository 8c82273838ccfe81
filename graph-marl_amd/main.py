#!/usr/bin/env python3
"""Train and evaluate agents in graph environments on MI355X — the CLI of the reference
(src/main.py) with the same flags, on the device path of this package.

    python graph-marl_amd/main.py --env-type=routing --model=dqn --netmon ...

Flow (src/main.py:409-1090): seed everything (set_seed), build Network + env (the routing
env or the simple env, n_env parallel instances, --n-env), optionally NetMon + the
NetMonWrapper, the DQN and its target copy, ε-greedy policy, AdamW, device replay; then
per step: reset on episode end, act, step, store the transition, log every 1000 steps,
update (TD loss over sampled sequences, clip 0.5 / norm 1.0, AdamW, soft target update)
and checkpoint; finally evaluate on EVAL_SEEDS (random topologies) and print the metrics
JSON. --eval only evaluates a loaded model.

Differences from the reference, by design:
  * everything runs on the GPU (--device=cpu is accepted for CLI compatibility and
    runs on the GPU as well; there is no CPU path);
  * --n-env N steps N independent envs per step (env b seeded with --seed + b, so N=1
    consumes exactly the reference's numpy stream); one update per vector step;
  * no tensorboard: the log lines go to stdout and checkpoints / eval metrics to
    --log-dir (default runs/<date>_<host><comment>, like SummaryWriter's logdir);
  * models: dqn, dgn, dqnr, commnet (comm_rounds 2); activation: any elementwise torch.nn.functional name
    (model.ACTIVATIONS: leaky_relu, relu, elu, tanh, sigmoid, relu6, hardtanh, hardsigmoid, selu, celu,
    softsign, logsigmoid, softplus, gelu, silu, mish, hardswish, tanhshrink);
    NetMon: sum/mean aggregation, lstm/lnlstm/gru cells, carry-over on, --netmon-global;
  * data parallel over the GPUs of a node: launched by torch.distributed.run (WORLD_SIZE > 1), each
    rank steps its own --n-env envs (disjoint seeds: --seed + rank * n_env + b), keeps its own replay
    (seeded --seed + rank), starts from rank 0's parameters and averages every update's gradients
    with one all-reduce (train.allreduce_gradients), so the replicas stay identical; rank 0 logs,
    writes the checkpoints and evaluates. The reference runs one independent job per GPU instead
    (scripts/start_routing_netmon_runs.sh:50). A rank whose training step raises posts the gradient
    exchange with a failure flag (train.abort_peers): every other rank raises train.PeerFailure at its
    next exchange or at the end-of-loop sync, so all ranks leave the loop together and exit non-zero
    (GM_FAULT=rank:step injects such a failure, for the tests).
"""
import argparse
import copy
import datetime
import importlib
import json
import os
import random
import socket
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
W = importlib.import_module("graph-marl_amd.wrapper")
P = importlib.import_module("graph-marl_amd.policy")
T = importlib.import_module("graph-marl_amd.train")
TS = importlib.import_module("graph-marl_amd.train_seq")
RB = importlib.import_module("graph-marl_amd.replaybuffer")
S = importlib.import_module("graph-marl_amd.simple")
HEU = importlib.import_module("graph-marl_amd.heuristics")
EV = importlib.import_module("graph-marl_amd.evaluate")
L = gm._lib


def build_parser():
    """The reference's flags (src/main.py:39-381) plus --n-env and --log-dir."""
    p = argparse.ArgumentParser(description="Train and test reinforcement learning agents in graph environments.")
    a = p.add_argument
    # environment settings
    a("--env-type", type=str, choices=["routing", "simple"], default="routing", help="The environment type")
    a("--n-router", type=int, default=20, help="Number of routers in the routing environment")
    a("--n-data", type=int, default=20, help="Number of packets in the routing environment")
    a("--env-var", type=int, choices=[1, 2, 3], default=1,
      help="Set the environment variant (1: local, 2: k neighbors, 3: global)")
    a("--episode-steps", type=int, default=300, help="Maximum number of steps for an episode")
    a("--ttl", type=int, default=0, help="Time to live for packets, set to 0 to disable")
    a("--random-topology", type=int, choices=[False, True], default=True,
      help="Use a random topology (1) or default topology (0)")
    a("--topology-init-seed", type=int, default=476, help="Init seed for fixed and random topology generation")
    a("--train-topology-allow-eval-seed", dest="train_topology_allow_eval_seed", action="store_true",
      help="Allow the use of evaluation seeds during training (e.g. for debugging)")
    a("--num-topologies-train", type=int, default=0,
      help="Number of random topologies for training (0 for unlimited)")
    a("--no-congestion", dest="no_congestion", action="store_true",
      help="Disables congestion in the routing environment")
    a("--action-mask", dest="enable_action_mask", action="store_true",
      help="Enables action masking in the routing environment")
    # approach settings
    a("--netmon", dest="netmon", action="store_true", help="Enables graph observations")
    a("--no-netmon", dest="netmon", action="store_false", help="Disables graph observations (default)")
    p.set_defaults(netmon=False)
    a("--netmon-global", dest="netmon_global", action="store_true",
      help="Enables global pooling of graph observations (only allowed in centralized case)")
    a("--netmon-dim", type=int, default=128, help="Size of NetMon state and observations")
    a("--netmon-encoder-dim", type=str, default="512,256", help="NetMon encoder dimensions. Examples: '128', '512,128'..")
    a("--netmon-iterations", type=int, default=3, help="Number of NetMon iterations between environment steps")
    a("--netmon-startup-iterations", type=int, default=1,
      help="Number of message passing iterations after environment reset (before first step)")
    a("--netmon-rnn-type", type=str, default="lstm", help="NetMon RNN type")
    a("--netmon-rnn-carryover", type=int, choices=[False, True], default=True,
      help="Carry over RNN state between RNN modules")
    a("--netmon-agg-type", type=str, default="sum", help="NetMon aggregation function")
    # model settings
    a("--model", type=str, choices=["dgn", "dqn", "dqnr", "commnet"], default="dgn", help="Base algorithm/model")
    a("--activation-function", type=str, default="leaky_relu", help="Activation function used in the model")
    a("--hidden-dim", type=str, default="512,256",
      help="Set the encoder dimension(s) that determine the hidden dim. Examples: '128', '512, 128'.. ")
    a("--num-heads", type=int, default=8, help="Number of agent attention heads (DGN only)")
    a("--num-attention-layers", type=int, default=2, help="Number of agent attention layers (DGN only)")
    # training settings
    a("--total-steps", type=int, default=1e6, help="Total number of training steps")
    a("--step-between-train", type=int, default=1,
      help="Number of steps that are performed between training iterations.")
    a("--lr", type=float, default=1e-4, help="Learning rate")
    a("--step-before-train", type=int, default=2000, help="Number of steps that are collected before training")
    a("--capacity", type=int, default=2e5, help="Replay memory capacity")
    a("--replay-half-precision", dest="replay_half_precision", action="store_true",
      help="Limit replay memory to half precision")
    a("--gamma", type=float, default=0.98, help="Discount factor")
    a("--mini-batch-size", type=int, default=10, help="Training mini batch size")
    a("--epsilon", type=float, default=0.6, help="Initial exploration probability")
    a("--epsilon-decay", type=float, default=0.996, help="Epsilon decay rate (multiplicative)")
    a("--epsilon-update-freq", type=int, default=100,
      help="Number of steps between applications of the epsilon decay factor")
    a("--sequence-length", type=int, default=1, help="Length of sampled sequences during training")
    a("--att-regularization-coeff", type=float, default=0.03, help="Attention regularization coefficient (DGN only)")
    a("--aux-loss-coeff", type=float, default=0.0,
      help="Auxiliary loss coefficient to enable supervised learning during RL")
    a("--target-update-steps", type=int, default=0,
      help="Number of steps between target model updates (smooth updates for 0)")
    a("--tau", type=float, default=0.01, help="Interpolation factor for smooth target model updates")
    a("--model-checkpoint-steps", type=int, default=1e5, help="Number of steps between saved model checkpoints")
    a("--comment", type=str, default="", help="Select a comment that allows to identify the run")
    a("--model-load-path", type=str, default=None, help="Loads a model from the given path")
    a("--model-load-no-args", dest="model_load_no_args", action="store_true",
      help="When loading a model, do not automatically overwrite the model's arguments.")
    a("--eval", dest="eval", action="store_true", help="Only run the evaluation")
    a("--eval-output-dir", type=str, default=None,
      help="Output eval directory (set to save results, only used with --eval)")
    a("--eval-output-detailed", dest="eval_output_detailed", action="store_true",
      help="Output more detailed evaluation output for all episodes.")
    a("--eval-output-node-state-aux", dest="output_node_state_aux", action="store_true",
      help="Output node state and aux information after eval (WARNING: potentially huge filesize).")
    a("--disable-progressbar", dest="disable_progressbar", action="store_true", help="Disables the progress bar")
    a("--eval-episodes", type=int, default=1000, help="Number of eval episodes")
    a("--eval-episode-steps", type=int, default=300, help="Maximum steps per eval episode")
    a("--debug-plots", dest="debug_plots", action="store_true", help="Create debug plots")
    a("--debug", type=int, default=0, help="Debug input to toggle experimental features")
    a("--device", type=str, choices=["cpu", "cuda"], default="cpu", help="Device to use")
    a("--seed", type=int, default=42, help="Seed for the experiment")
    a("--policy", type=str, choices=["heuristic", "random", "trained"], default="trained",
      help="The policy that should be used, 'heuristic' depends on the given --env-type")
    # graph-marl_amd
    a("--n-env", type=int, default=1, help="Parallel environment instances per step (graph-marl_amd)")
    a("--log-dir", type=str, default=None, help="Checkpoint / metrics directory (default runs/<date>_<host><comment>)")
    return p


MODEL_ARG_KEYS = ["model", "hidden_dim", "netmon", "netmon_dim", "netmon_encoder_dim", "netmon_iterations",
                  "netmon_rnn_type", "netmon_agg_type", "netmon_global", "activation_function", "num_heads",
                  "num_attention_layers"]


def dim_str_to_list(dims):
    """src/util.py:108-111"""
    return [] if len(dims) == 0 else [int(x) for x in dims.split(",")]


def set_seed(seed):
    """src/util.py:81-105"""
    torch.manual_seed(seed)
    random.seed(seed)
    np.random.seed(seed)


def get_state_dict(model, netmon, args):
    """src/util.py:26-35: the reference's checkpoint dict (loadable by either side)."""
    d = {"type": type(model).__name__, "state_dict": model.state_dict(), "args": args}
    if netmon is not None:
        d["netmon_state_dict"] = netmon.state_dict()
    return d


def load_state_dict(state_dict, model, netmon):
    """src/util.py:38-52"""
    if state_dict["type"] != type(model).__name__:
        print(f"Warning: Loader expected {type(model).__name__} but found {state_dict['type']}")
    if "netmon_state_dict" in state_dict:
        if netmon is None:
            raise ValueError("Model uses NetMon which has not been initialized.")
        netmon.load_state_dict(state_dict["netmon_state_dict"])
    elif netmon is not None:
        raise ValueError("NetMon state could not be found.")
    model.load_state_dict(state_dict["state_dict"])


def load_checkpoint(path):
    # weights_only: the args entry is a plain dict, nothing is unpickled beyond tensors/primitives
    return torch.load(path, map_location="cpu", weights_only=True)


class Logger:
    """Per-log-interval means of the reward and the env statistics, kept on the device
    (the reference's Buffer objects, src/main.py:615-625,749-793)."""

    LIST_KEYS = {"delays": ("sum_delays", "n_delays"), "delays_arrived": ("sum_delays_arrived", "n_arrived"),
                 "spr": ("sum_spr", "n_arrived")}
    SCALAR_KEYS = ["looped", "throughput", "dropped", "blocked"]

    def __init__(self):
        self.clear()

    def clear(self):
        self.acc = {}
        self.host = {}
        self.steps = 0

    def add(self, k, v):
        self.acc[k] = self.acc[k] + v if k in self.acc else v.detach().clone()

    def add_host(self, k, v):
        self.host.setdefault(k, []).append(v)

    def step(self, reward, info_sum=None):
        """reward [n_env, A]; info_sum: per-step env statistics summed over envs [GM_INFO_FIELDS]."""
        self.steps += 1
        self.add("reward", reward.to(torch.float64).mean())
        self.add("envs", torch.tensor(float(reward.shape[0]), dtype=torch.float64, device=reward.device))
        if info_sum is not None:
            self.add("info", info_sum)

    def means(self):
        h = {k: v.detach().cpu().numpy() for k, v in self.acc.items()}
        out = {}
        if "info" in h:
            inf = dict(zip(L.INFO_KEYS, h["info"].tolist()))
            for k, (s_, c) in self.LIST_KEYS.items():
                if inf[c] > 0:
                    out[k] = inf[s_] / inf[c]
            for k in self.SCALAR_KEYS:
                out[k] = inf[k] / float(h["envs"])
        for k, v in self.host.items():
            out[k] = float(np.mean(v))
        return float(h.get("reward", 0.0)) / max(self.steps, 1), out


def build_model(args, agent_obs_size, n_actions):
    """src/main.py:486-523"""
    hidden = dim_str_to_list(args.hidden_dim)
    if args.model == "dgn":
        return M.DGN(agent_obs_size, hidden, n_actions, args.num_heads, args.num_attention_layers,
                     activation=args.activation_function)
    if args.model == "dqnr":
        return M.DQNR(agent_obs_size, hidden, n_actions, activation=args.activation_function)
    if args.model == "commnet":
        return M.CommNet(agent_obs_size, hidden, n_actions, comm_rounds=2, activation=args.activation_function)
    if args.model == "dqn":
        return M.DQN(agent_obs_size, hidden, n_actions, activation=args.activation_function)
    raise ValueError(f"Unknown model type {args.model}")


def make_env(args, dev, obs_extra, rank=0, world=1):
    seeds = T.shard_seeds(rank, world, args.n_env, args.seed)  # rank 0 of 1: --seed + b
    if args.env_type == "routing":
        network = gm.Network(n_nodes=args.n_router, random_topology=bool(args.random_topology),
                             n_random_seeds=args.num_topologies_train, topology_init_seed=args.topology_init_seed,
                             excluded_seeds=None if args.train_topology_allow_eval_seed else gm.EVAL_SEEDS,
                             device=dev.index)
        return gm.Routing(network, args.n_data, args.env_var, enable_congestion=not args.no_congestion,
                          enable_action_mask=args.enable_action_mask, ttl=args.ttl, n_env=args.n_env,
                          seeds=seeds, obs_extra=obs_extra,
                          agent_adjacency=args.model in ("dgn", "commnet"), device=dev.index)
    if args.env_type == "simple":
        return S.SimpleEnvironment(args.env_var, bool(args.random_topology), n_env=args.n_env, seeds=seeds,
                                   obs_extra=obs_extra, device=dev.index)
    raise ValueError(f"Unknown environment {args.env_type}")


def main(argv=None):
    args = build_parser().parse_args(argv)
    rank, world, _ = T.init_distributed()
    try:
        return _main(args, rank, world)
    finally:
        if world > 1 and T.dist.is_initialized():
            T.dist.destroy_process_group()


def _main(args, rank, world):
    lead = rank == 0
    log_print = print if lead else (lambda *a, **k: None)
    # src/main.py: no more capacity than transitions; with --n-env envs a step stores n_env of them
    args.capacity = min(args.total_steps * args.n_env, args.capacity)
    if args.model_load_path and not args.model_load_no_args:
        assert os.path.exists(args.model_load_path)
        loaded = load_checkpoint(args.model_load_path)
        vals = {k: v for k, v in loaded["args"].items() if k in MODEL_ARG_KEYS}
        vals["policy"] = "trained"
        for k, v in vals.items():
            setattr(args, k, v)
    if args.device == "cpu":
        log_print("Note: graph-marl_amd runs on the GPU; --device=cpu runs on cuda:0")
    L.require_gpu()
    dev = torch.device("cuda", torch.cuda.current_device())
    set_seed(args.seed)
    if args.sequence_length <= 0:
        raise ValueError(f"Invalid sequence length {args.sequence_length}. Must be greater 0.")
    act = args.activation_function
    M.act_code(act)  # src/main.py:440-441 getattr(F, name): names outside model.ACTIVATIONS raise here

    H = args.netmon_dim
    env = make_env(args, dev, obs_extra=(5 if args.netmon_global else 4) * H if args.netmon else 0, rank=rank,
                   world=world)
    env.reset()  # reset_and_get_sizes (src/main.py:443): the reference's first reset
    n_agents, n_nodes, node_obs_size = env.n_data, env.n_nodes, env.node_obs_dim
    netmon = None
    if args.netmon:
        netmon = M.NetMon(node_obs_size, H, dim_str_to_list(args.netmon_encoder_dim), args.netmon_iterations,
                          rnn_type=args.netmon_rnn_type, rnn_carryover=bool(args.netmon_rnn_carryover),
                          agg_type=args.netmon_agg_type, output_neighbor_hidden=True,
                          output_global_hidden=args.netmon_global, activation=act).to(dev)
        node_state_size = netmon.get_state_size()
        env = W.NetMonWrapper(env, netmon, args.netmon_startup_iterations)
        env.reset()  # second reset_and_get_sizes (src/main.py:478)
        agent_obs_size = env.obs_dim
    else:
        node_state_size = 0
        agent_obs_size = env.obs_dim
    base = env.get()
    model = model_tar = None
    if args.policy == "trained" or args.model_load_path:
        model = build_model(args, agent_obs_size, base.action_space.n).to(dev)
        if args.model_load_path:
            load_state_dict(load_checkpoint(args.model_load_path), model, netmon)
        T.broadcast_parameters([m for m in (model, netmon) if m is not None])  # replicas start as rank 0's
        model_tar = copy.deepcopy(model)

    if args.policy == "trained":
        policy = P.EpsilonGreedy(env, model, base.action_space.n, args)
    elif args.policy == "heuristic":
        policy = HEU.ShortestPath(env) if args.env_type == "routing" else HEU.SimplePolicy(env)
    else:
        policy = HEU.RandomPolicy(env, action_space=base.action_space.n, seed=args.seed)

    def switch_to_eval_seeds():
        if isinstance(base, gm.Routing) and args.random_topology:
            if args.eval_episodes > len(gm.EVAL_SEEDS):
                print("WARNING: Duplicate eval seeds as number of eval episodes is higher than "
                      f"the number of available seeds ({len(gm.EVAL_SEEDS)})!")
            base.set_topology_seeds(gm.EVAL_SEEDS, sequential=True, interleave=base.n_env > 1)

    if args.eval:
        if not lead:  # evaluation runs on rank 0
            return None
        print(f"Policy: {type(policy).__name__}")
        switch_to_eval_seeds()
        print("Performing Evaluation")
        metrics = EV.evaluate(env, policy, args.eval_episodes, args.eval_episode_steps, args.disable_progressbar,
                              args.eval_output_dir)
        print(json.dumps(metrics, indent=4, sort_keys=True, default=str))
        return metrics

    assert args.policy == "trained", f"Given policy {args.policy} cannot be used for training."
    params = list(model.parameters()) + ([] if netmon is None else list(netmon.parameters()))
    aux_model = None
    node_aux_size = n_nodes if (netmon is not None and isinstance(base, gm.Routing)) else 0
    if netmon is not None and node_aux_size > 0 and args.aux_loss_coeff > 0:
        # NetMon aux head (src/main.py:586-594): MLP(state, (state, aux), activation_on_output=False)
        aux_model = M.MLP(node_state_size, [node_state_size, node_aux_size], activation_on_output=False,
                          activation=act).to(dev)
        T.broadcast_parameters([aux_model])
        params = params + list(aux_model.parameters())
    optimizer = torch.optim.AdamW(params, lr=args.lr)
    has_state = hasattr(model, "state")
    needs_adj = args.model in ("dgn", "commnet")
    buff = RB.ReplayBuffer(args.seed + rank, int(args.capacity), base.n_env, n_agents, base.obs_dim, n_nodes,
                           node_obs_size, node_state_size, dev, half_precision=args.replay_half_precision,
                           nbr_width=base.nbr.shape[-1] if hasattr(base, "nbr") else 3,
                           agent_state_size=model.get_state_len() if has_state else 0, store_adj=needs_adj,
                           node_aux_size=node_aux_size if aux_model is not None else 0)
    last_state = None
    comment = "_" + (f"R{args.env_var}" if args.env_type == "routing" else "Simple") + "_" + \
        {"dqn": "DQN", "dgn": "DGN", "dqnr": "DQNR", "commnet": "CommNet"}[args.model]
    if netmon is not None:
        comment += "_netmon"
    if args.comment:
        comment += f"_{args.comment}"
    log_dir = args.log_dir or os.path.join(
        "runs", datetime.datetime.now().strftime("%b%d_%H-%M-%S") + "_" + socket.gethostname() + comment)
    if lead:
        os.makedirs(log_dir, exist_ok=True)

    log_print("Start training with arguments")
    log_print(json.dumps(args.__dict__, indent=4, sort_keys=True, default=str))
    log_print("Model type: DQN")
    log_print(env)
    if world > 1:
        log_print(f"Data parallel: {world} ranks x {base.n_env} envs, one gradient all-reduce per update")
    log = Logger()
    best = -float("inf")
    episode_step = None
    episode_done = False
    current_episode = 0
    iteration = 0
    t0 = time.time()
    exception_training = None
    fault = os.environ.get("GM_FAULT")  # "rank:step": that rank raises at that step (failure-path tests)
    fault = tuple(int(v) for v in fault.split(":")) if fault else None
    try:
        for step in range(1, int(args.total_steps) + 1):
            if fault == (rank, step):
                raise RuntimeError(f"GM_FAULT: injected failure on rank {rank} at step {step}")
            if episode_step is None or episode_done:
                if episode_step is not None:
                    L.check_range()  # split-f16 range guard (graph_marl_amd.h gm_gemm_range_status)
                episode_step = 0
                env.reset()
                current_episode += 1
                last_state = None  # src/main.py:683-686
            if has_state:
                model.state = last_state
            adj = base.agent_adj if needs_adj else None
            if netmon is not None:
                buff.add_pre(base.obs, env.last_netmon_state, base.node_obs, base.nbr, base.agent_node, adj=adj,
                             agent_state=last_state,
                             node_aux=base.get_node_aux() if aux_model is not None else None)
            else:
                buff.add_pre(base.obs, adj=adj, agent_state=last_state)
            with torch.no_grad():
                if hasattr(policy, "act_step"):  # ε-greedy draws fused into the env step kernel
                    actions = policy.act_step(env)
                else:
                    actions = policy.act(env)
                    env.step_(actions)
            if has_state:  # done agents restart from a zero state (src/main.py:710-716)
                last_state = model.state * ~base.done.bool().unsqueeze(-1)
            episode_step += 1
            episode_done = episode_step >= args.episode_steps
            buff.add_post(actions, base.reward, base.obs, base.done.bool(), episode_done,
                          base.node_obs if netmon is not None else None,
                          base.agent_node if netmon is not None else None,
                          next_adj=base.agent_adj if needs_adj else None)
            info_sum = None
            if isinstance(base, gm.Routing):
                info_sum = base.info.sum(0)
                if episode_done:  # get_final_info: packets still running count into the delays
                    fin = base.final_info().sum(0)
                    info_sum[L.INFO_KEYS.index("sum_delays")] += fin[0]
                    info_sum[L.INFO_KEYS.index("n_delays")] += fin[1]
            log.step(base.reward, info_sum)

            if step % 1000 == 0 and lead:
                mean_reward, means = log.means()
                log.clear()
                eps = f"  eps: {policy._epsilon:.2f}" if hasattr(policy, "_epsilon") else ""
                print(f"Episode: {current_episode}  step: {step / 1000:.0f}k  reward: {mean_reward:.2f}"
                      f"{''.join(f'  {k}: {v:.2f}' for k, v in means.items())}{eps}"
                      f"{' | BEST' if mean_reward > best else ''}"
                      f"  ({world * base.n_env * step / (time.time() - t0):.0f} env-steps/s)", flush=True)
                if mean_reward > best:
                    torch.save(get_state_dict(model, netmon, args.__dict__), os.path.join(log_dir, "model_best.pt"))
                    best = mean_reward

            if step < args.step_before_train or buff.count * base.n_env < args.mini_batch_size \
                    or step % args.step_between_train != 0:
                continue
            iteration += 1
            model.train()
            if netmon is not None:
                netmon.train()
            parts = {}
            att = args.att_regularization_coeff if args.model == "dgn" else 0.0
            if args.sequence_length > 1 and TS.seq_ok(netmon, model, model_tar, att, aux_model):
                # sequence-batched update with the hand-written backward (train_seq.py)
                loss, q_all, qt_all = TS.dqn_update_seq(netmon, model, model_tar, optimizer, params,
                                                        buff.get_sequences(args.mini_batch_size,
                                                                           args.sequence_length),
                                                        args.gamma, args.tau, args.target_update_steps, iteration)
                qs, qts = list(q_all), list(qt_all)
            else:
                batches = list(buff.get_batch(args.mini_batch_size, sequence_length=args.sequence_length,
                                              lazy_next=True))
                loss, qs, qts = T.dqn_update(netmon, model, model_tar, optimizer, params, batches, args.gamma,
                                             args.tau, args.target_update_steps, iteration, att_coeff=att,
                                             aux_model=aux_model, aux_coeff=args.aux_loss_coeff, parts=parts,
                                             consecutive=True)  # replay sequences: the target reuses online steps
            model.eval()
            if netmon is not None:
                netmon.eval()
                netmon.state = None
            if step % 100 == 0:  # host reads are sampled to keep the step loop asynchronous
                log.add_host("q_values", float(torch.stack([q.detach().mean() for q in qs]).mean().item()))
                log.add_host("q_target", float(torch.stack([q.mean() for q in qts]).mean().item()))
                log.add_host("loss", float(loss.item()))
                if aux_model is not None:
                    log.add_host("loss_aux", float(parts["loss_aux"].item()))
            if args.target_update_steps > 0 and iteration % args.target_update_steps == 0:
                log_print(f"Update network, train iteration {iteration}")
            if step % int(args.model_checkpoint_steps) == 0 and lead:
                torch.save(get_state_dict(model, netmon, args.__dict__),
                           os.path.join(log_dir, f"model_{int(step):_d}.pt"))
    except Exception as e:  # like the reference: evaluate and save, then fail
        import traceback

        traceback.print_exc()
        exception_training = e
        dist_err = getattr(T.dist, "DistError", ())
        if world > 1 and not isinstance(e, (T.PeerFailure, dist_err)):
            T.abort_peers(params)  # the peers' next gradient exchange raises PeerFailure: every rank stops
    if world > 1 and exception_training is None:
        try:  # meets a peer that failed after this rank's last update
            T.finish_sync(params)
        except T.PeerFailure as e:
            print(f"rank {rank}: {e}", flush=True)
            exception_training = e
    log_print("Performing clean exit")
    del buff
    metrics = None
    exception_evaluation = None
    if not lead:  # rank 0 evaluates and saves the (identical) replica
        if exception_training is not None:
            raise SystemExit(f"rank {rank}: an exception was raised during training (see above).")
        return None
    try:
        if netmon is not None:
            netmon.state = None
        switch_to_eval_seeds()
        print("Performing Evaluation")
        metrics = EV.evaluate(env, policy, args.eval_episodes, args.eval_episode_steps, args.disable_progressbar,
                              os.path.join(log_dir, "eval"))
        print(json.dumps(metrics, indent=4, sort_keys=True, default=str))
    except Exception as e:
        import traceback

        traceback.print_exc()
        exception_evaluation = e
    finally:
        torch.save(get_state_dict(model, netmon, args.__dict__), os.path.join(log_dir, "model_last.pt"))
    if exception_training is not None or exception_evaluation is not None:
        what = " and ".join(w for w, e in (("training", exception_training), ("evaluation", exception_evaluation))
                            if e is not None)
        raise SystemExit(f"An exception was raised during {what} (see above).")
    return metrics


if __name__ == "__main__":
    main()
