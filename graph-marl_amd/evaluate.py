"""Evaluation reducer (reference src/eval.py:33-168 evaluate / get_eval_metrics).

Runs `episodes` episodes of `steps_per_episode` steps with the policy in eval mode
(ε = 0) and reduces the per-step env statistics to the reference's metrics:
  reward_mean              mean over every agent reward of every step
  delays/delays_arrived/spr_mean
                           mean over the per-packet lists (delays include the packets still
                           running at the last step, get_final_info)
  looped/throughput/dropped/blocked_mean
                           mean over the per-step counts
  + eval-only statistics (routing.py:414-441) when the env supports set_eval_info.
The n_env envs run ceil(episodes / n_env) rounds of parallel episodes; sums are kept in
fp64 on the device and read back once at the end.
"""
import math

import torch

from . import _lib as L


@torch.no_grad()
def evaluate(env, policy, episodes, steps_per_episode, disable_progressbar=True, output_dir=None):
    base = env.get() if hasattr(env, "get") else env
    n_env = base.n_env
    dev = base.device
    if hasattr(policy, "eval"):
        policy.eval()
    if hasattr(env, "set_eval_info"):
        env.set_eval_info(True)
    routing = hasattr(base, "info")
    acc = {}

    def add(key, val):
        acc[key] = acc[key] + val if key in acc else val.clone()

    rounds = math.ceil(episodes / n_env)
    for r in range(rounds):
        active = torch.arange(n_env, device=dev) < (episodes - r * n_env)
        w = active.to(torch.float64)
        env.reset()
        if hasattr(policy, "reset"):  # recurrent agent models start every episode from zeros
            policy.reset(True)
        if hasattr(policy, "reset_episode"):
            policy.reset_episode()
        for step in range(steps_per_episode):
            actions = policy.act(env) if hasattr(policy, "act") else policy(env.obs)
            _, _, reward, done, info = env.step(actions)
            if step + 1 == steps_per_episode:
                info = env.get_final_info(info)
            add("reward_sum", (reward.to(torch.float64).sum(-1) * w).sum())
            add("reward_cnt", w.sum() * reward.shape[-1])
            if routing:
                for k in L.INFO_KEYS:
                    add(k, (info[k] * w).sum())
                if "total_edge_load" in info:
                    for k in L.EVAL_KEYS:
                        add(k, (info[k] * w).sum())
            add("steps", w.sum())
            if hasattr(policy, "reset"):  # reset done agents (src/eval.py:111-113)
                policy.reset(done)
    if hasattr(env, "set_eval_info"):
        env.set_eval_info(False)
    h = {k: float(v.item()) for k, v in acc.items()}

    def mean(s, c):
        return s / c if c > 0 else float("inf")

    metrics = {"reward_mean": mean(h["reward_sum"], h["reward_cnt"])}
    if routing:
        A = base.n_data
        metrics.update({
            "delays_mean": mean(h["sum_delays"], h["n_delays"]),
            "delays_arrived_mean": mean(h["sum_delays_arrived"], h["n_arrived"]),
            "spr_mean": mean(h["sum_spr"], h["n_arrived"]),
            "looped_mean": mean(h["looped"], h["steps"]),
            "throughput_mean": mean(h["throughput"], h["steps"]),
            "dropped_mean": mean(h["dropped"], h["steps"]),
            "blocked_mean": mean(h["blocked"], h["steps"]),
        })
        if "total_edge_load" in h:
            metrics.update({
                "total_edge_load_mean": mean(h["total_edge_load"], h["steps"]),
                "occupied_edges_mean": mean(h["occupied_edges"], h["steps"]),
                "packets_on_edges_mean": mean(h["packets_on_edges"], h["steps"]),
                "total_packet_size_mean": mean(h["total_packet_size"], h["steps"]),
                "packet_sizes_mean": mean(h["total_packet_size"], h["steps"] * A),
                "packet_distances_mean": mean(h["sum_packet_distances"], h["steps"] * A),
            })
    if output_dir is not None:
        import json
        import os

        os.makedirs(output_dir, exist_ok=True)
        with open(os.path.join(output_dir, "metrics.json"), "w") as f:
            json.dump(metrics, f, indent=4, sort_keys=True)
    return metrics
