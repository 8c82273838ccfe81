#!/usr/bin/env python3
"""Supervised shortest-path task with NetMon (reference src/sl.py) on MI355X — the
BASELINE config-5 driver: pure NetMon message-passing forward + backward throughput.

    python graph-marl_amd/sl.py --iterations 4000 --sequence-length 4
    python graph-marl_amd/sl.py --bench --n-nodes 100 --batch-size 8192 --sequence-length 8 \\
        --netmon-iterations 1           # config 5: node-steps/s of fwd + bwd + AdamW

Task (src/sl.py:174-218): for every node of a random topology (with --n-packets random
packets), regress the shortest-path distances to all nodes (the APSP row, the loss uses
the first --num-targets columns). Model (src/sl.py:132-168): NetMon without agent
mapping (every node reads out [h, h_prev of its neighbours]) + three linear heads
(classes, distance to node 0, distances to all nodes). Training (src/sl.py:322-445):
per iteration a batch of graphs is drawn with replacement, NetMon is unrolled
--sequence-length times on the same graphs from a zero state, the per-step losses are
averaged, AdamW (torch defaults) steps.

Datasets are generated on the device by the batched routing env (one env per graph,
env b seeded with --seed + b; train topologies are random with EVAL_SEEDS excluded,
validation topologies walk a build_seed_list of 1000 seeds, test topologies walk
EVAL_SEEDS — as in src/sl.py:565-590). The reference's pickle cache and HDF5 result
files are not built; --filename writes the results as JSON.
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

gm = importlib.import_module("graph-marl_amd")
M = importlib.import_module("graph-marl_amd.model")
SQ = importlib.import_module("graph-marl_amd.sl_seq")
L = gm._lib

NUM_CLASSES = 4
WITH_CLASSIFICATION, WITH_REGRESSION, WITH_REGRESSION_ALL = False, False, True  # src/sl.py:546-548


def build_parser():
    """src/sl.py:19-126 plus the sizes the reference hard-codes (543-563) and --bench."""
    p = argparse.ArgumentParser(description="Train and test graph observation models on a supervised routing task.")
    a = p.add_argument
    a("--num-targets", type=int, default=None,
      help="Number of targets included in the loss for regression with all destinations")
    a("--num-samples-train", type=int, default=10_000,
      help="Number of generated training graphs (ignored when loading a dataset)")
    a("--seed", type=int, default=42, help="Seed for the experiment")
    a("--iterations", type=int, default=4_000, help="Number of training iterations")
    a("--validate-after", type=int, default=1_000, help="Validate model after the given number of training steps")
    a("--sequence-length", type=int, default=4, help="Unroll depth of the model for each sample")
    a("--filename", type=str, default=None, help="Where to save the results (JSON)")
    a("--test-sequence-lengths", type=str, default="1,2,4,8,16,32,64,128,256",
      help="Sequence lengths used during testing")
    a("--netmon-dim", type=int, default=128, help="Size of NetMon state and observations")
    a("--netmon-encoder-dim", type=str, default="512,256", help="NetMon encoder dimensions. Examples: '128', '512,128'..")
    a("--netmon-iterations", type=int, default=3, help="Number of NetMon iterations between environment steps")
    a("--netmon-rnn-type", type=str, default="lstm", help="NetMon RNN type")
    a("--netmon-rnn-carryover", type=int, choices=[False, True], default=True,
      help="Carry over RNN state between RNN modules")
    a("--netmon-agg-type", type=str, default="sum", help="NetMon aggregation function")
    a("--netmon-global", dest="netmon_global", action="store_true",
      help="Enables global pooling of graph observations (only allowed in centralized case)")
    a("--netmon-last-neighbors", type=int, choices=[False, True], default=True,
      help="Append last node state received by neighbors to graph observation")
    a("--disable-progressbar", dest="disable_progressbar", action="store_true",
      help="Disables the progress bar and iteration-wise status prints")
    a("--clear-cache", dest="clear_cache", action="store_true",
      help="Forces generation of new datasets (datasets are generated on the device, never cached)")
    # sizes the reference hard-codes
    a("--n-nodes", type=int, default=20, help="Nodes per graph (src/sl.py:562)")
    a("--n-packets", type=int, default=20, help="Packets per graph (src/sl.py:563)")
    a("--batch-size", type=int, default=32, help="Graphs per iteration (src/sl.py:543)")
    a("--num-samples-test", type=int, default=1_000, help="Validation / test graphs (src/sl.py:550)")
    a("--bench", action="store_true",
      help="Throughput mode: no validation / test; print one JSON line with node-steps/s")
    a("--warmup", type=int, default=3, help="Untimed iterations before the timed region (--bench)")
    a("--sl-autograd", dest="sl_autograd", action="store_true",
      help="Per-step autograd NetMon instead of the sequence-batched unroll (sl_seq.py; A/B and diagnostics)")
    return p


def dim_str_to_list(dims):
    return [] if len(dims) == 0 else [int(x) for x in dims.split(",")]


class NetMonSL(torch.nn.Module):
    """src/sl.py:132-168: NetMon over all nodes + classification / distance heads."""

    def __init__(self, args, node_obs_dim, nb_classes, nb_nodes):
        super().__init__()
        self.netmon = M.NetMon(node_obs_dim, args.netmon_dim, dim_str_to_list(args.netmon_encoder_dim),
                               args.netmon_iterations, rnn_type=args.netmon_rnn_type,
                               rnn_carryover=bool(args.netmon_rnn_carryover), agg_type=args.netmon_agg_type,
                               output_neighbor_hidden=bool(args.netmon_last_neighbors),
                               output_global_hidden=args.netmon_global)
        F = self.netmon.get_out_features()
        self.linear = M.Linear(F, nb_classes)
        self.linear_reg = M.Linear(F, 1)
        self.linear_reg_all = M.Linear(F, nb_nodes)
        self.class_logits = None

    def forward(self, node_obs, nbr, enc=None):
        node_features = self.netmon.forward_graph(node_obs, nbr, None, enc=enc)
        class_logits = self.linear(node_features)
        pred = self.linear_reg(node_features)
        pred_all = self.linear_reg_all(node_features)
        self.class_logits = class_logits.detach()
        return class_logits, pred, pred_all

    def forward_seq(self, node_obs, nbr, steps):
        """`steps` unrolled NetMon steps from a zero state (src/sl.py:363-368) as one sequence-batched
        autograd node (sl_seq.readout_seq), then the all-destinations head once over every step's
        rows: pred_all [steps, B, N, nb_nodes]. The class / distance-to-0 heads are not evaluated
        (they do not enter the training loss of the reference's default task, src/sl.py:546-548)."""
        B, N = node_obs.shape[:2]
        R = SQ.readout_seq(self.netmon, node_obs, nbr, steps)
        return self.linear_reg_all(R).view(steps, B, N, -1)

    def get_class_probabilities(self):
        return torch.softmax(self.class_logits, dim=-1)

    def get_prediction(self):
        return torch.argmax(self.get_class_probabilities(), axis=-1)


class Dataset:
    """node_obs f32 [S, N, 4N+8], nbr int32 [S, N, 3], targets_all f32 [S, N, N] (APSP),
    targets f32 [S, N] (distance to node 0), labels int64 [S, N] (first hop to node 0 as
    1 + edge index by neighbour id, 0 at node 0)."""

    def __init__(self, node_obs, nbr, targets_all, labels):
        self.node_obs, self.nbr, self.targets_all, self.labels = node_obs, nbr, targets_all, labels
        self.targets = targets_all[:, :, 0].contiguous()

    def __len__(self):
        return self.node_obs.shape[0]


def build_dataset(n_nodes, n_packets, count, seed, seeds=None, chunk=8192):
    """get_sl_sample (src/sl.py:174-218) for `count` graphs on the device: random topologies
    (EVAL_SEEDS excluded) or, with `seeds`, graph i from seeds[i] (sequential networks)."""
    obs, nbrs, aux, labels = [], [], [], []
    for c0 in range(0, count, chunk):
        B = min(chunk, count - c0)
        net = gm.Network(n_nodes, random_topology=True, excluded_seeds=gm.EVAL_SEEDS)
        env = gm.Routing(net, n_packets, n_env=B, seeds=[(seed + c0 + b) & 0xFFFFFFFF for b in range(B)],
                         agent_adjacency=False)
        if seeds is not None:
            env.set_topology_seeds(seeds[c0:c0 + B], sequential=True, interleave=True)
        env.reset_()
        obs.append(env.node_obs.clone())
        nbrs.append(env.nbr.clone())
        aux.append(env.get_node_aux())
        act = torch.zeros(B, n_nodes, dtype=torch.int32, device=env.device)
        labels.append(_labels_to_zero(env, act))
        env.close()
    return Dataset(torch.cat(obs), torch.cat(nbrs), torch.cat(aux), torch.cat(labels))


def _labels_to_zero(env, scratch):
    """Classification labels (src/sl.py:189-210): ShortestPath first hop towards node 0."""
    B, N = env.n_env, env.n_nodes
    first = torch.empty(B, N, N, dtype=torch.int32, device=env.device)
    L.check(L.lib().gm_env_first_hops(env._h, L.ptr(first), L.stream_ptr(env.device)))
    nxt = first[:, :, 0]  # [B, N]: first hop of node n towards node 0
    idx = (env.nbr == nxt.unsqueeze(-1)).int().argmax(-1) + 1
    return torch.where(torch.arange(N, device=env.device) == 0, torch.zeros_like(idx), idx).long()


def _loss_terms(args, out, tgt_all, tgt, labels, reduction="mean"):
    log_probs, pred, pred_all = out
    loss = 0
    terms = {}
    if WITH_CLASSIFICATION:
        terms["class"] = torch.nn.functional.cross_entropy(log_probs.reshape(-1, NUM_CLASSES), labels.reshape(-1),
                                                           reduction=reduction)
        loss = loss + terms["class"]
    if WITH_REGRESSION:
        terms["reg"] = torch.nn.functional.mse_loss(pred.reshape(-1, 1), tgt.reshape(-1, 1), reduction=reduction)
        loss = loss + terms["reg"]
    if WITH_REGRESSION_ALL:
        k = args.num_targets
        terms["reg_all"] = torch.nn.functional.mse_loss(pred_all[..., :k], tgt_all[..., :k], reduction=reduction)
        loss = loss + terms["reg_all"]
    return loss, terms


class _StepMSE(torch.autograd.Function):
    """Per-step mse_loss of pred [L, ...] against one target [...] (src/sl.py:396-400 at every unroll
    step): [L] losses. The squares are summed in two stages (a single torch reduction of a few
    outputs over hundreds of millions of elements ran at ~0.15 TB/s); backward = one elementwise pass
    over the saved difference."""

    @staticmethod
    def forward(ctx, pred, tgt):
        steps, n = pred.shape[0], pred[0].numel()
        ctx.n = n
        ctx.fused = _step_mse_fits(pred, tgt)
        if ctx.fused:
            # one pass over pred with the target held in registers across the steps (gm_step_mse); the
            # difference is not stored: backward recomputes it from pred and tgt (gm_step_mse_bwd)
            part = torch.empty(steps, L.lib().gm_step_mse_blocks(n), device=pred.device)
            L.check(L.lib().gm_step_mse(pred.data_ptr(), tgt.data_ptr(), n, steps, part.data_ptr(), L.stream_ptr()))
            ctx.save_for_backward(pred, tgt)
            return part.sum(1) / n
        d = pred - tgt
        c = next(c for c in (4096, 1024, 256, 64, 16, 4, 1) if n % c == 0)
        per = d.reshape(steps, c, n // c).pow(2).sum(2).sum(1) / n
        ctx.save_for_backward(d)
        return per

    @staticmethod
    def backward(ctx, g):
        if ctx.fused:
            pred, tgt = ctx.saved_tensors
            g = g.contiguous()
            grad = torch.empty_like(pred)
            L.check(L.lib().gm_step_mse_bwd(pred.data_ptr(), tgt.data_ptr(), ctx.n, pred.shape[0], g.data_ptr(),
                                            2.0 / ctx.n, grad.data_ptr(), L.stream_ptr()))
            return grad, None
        (d,) = ctx.saved_tensors
        return d * (g.view((-1,) + (1,) * (d.dim() - 1)) * (2.0 / ctx.n)), None


def _step_mse_fits(pred, tgt):
    """gm_step_mse covers fp32 device tensors with contiguous rows of a multiple of 4 elements per step and
    16-byte bases (the config-5 loss: pred_all [L, B, N, N] against targets_all [B, N, N]); other shapes
    (a --num-targets slice, fp64 host tensors in the CPU tests) take the torch expression."""
    return (pred.is_cuda and pred.dtype == torch.float32 and tgt.dtype == torch.float32 and pred.is_contiguous()
            and tgt.is_contiguous() and tgt.shape == pred.shape[1:] and pred[0].numel() % 4 == 0
            and pred.data_ptr() % 16 == 0 and tgt.data_ptr() % 16 == 0)


def train_step(args, model, optim, data, batch_idx):
    """One iteration of src/sl.py:360-424."""
    model.netmon.state = None
    obs, nbr = data.node_obs[batch_idx], data.nbr[batch_idx]
    tgt_all, tgt, labels = data.targets_all[batch_idx], data.targets[batch_idx], data.labels[batch_idx]
    steps = max(args.sequence_length, 1)
    if (WITH_REGRESSION_ALL and not WITH_CLASSIFICATION and not WITH_REGRESSION
            and SQ.seq_ok(model.netmon, rows=obs.shape[0] * obs.shape[1], steps=steps)
            and not getattr(args, "sl_autograd", False)):
        # sequence-batched NetMon (sl_seq.py): the mean of the per-step MSEs over all steps' rows at once
        k = args.num_targets
        pred_all = model.forward_seq(obs, nbr, steps)
        per = _StepMSE.apply(pred_all[..., :k], tgt_all[..., :k])
        total = per.mean()
        optim.zero_grad()
        total.backward()
        optim.step()
        return total.detach(), {"reg_all": per[-1].detach()}
    seq = []
    terms = {}
    # the reference re-encodes the same observations at every unroll step (src/sl.py:360-424); the
    # encoder output is identical each time, so it is computed once and its gradient (the sum of
    # the steps' contributions) runs back through the encoder once
    enc = model.netmon.encode_nodes(obs, nbr)
    for _ in range(max(args.sequence_length, 1)):
        loss, terms = _loss_terms(args, model(obs, nbr, enc), tgt_all, tgt, labels)
        seq.append(loss)
    total = torch.mean(torch.stack(seq))
    optim.zero_grad()
    total.backward()
    optim.step()
    return total.detach(), {k: v.detach() for k, v in terms.items()}


@torch.no_grad()
def test(args, model, data, batch_size, sequence_length):
    """src/sl.py:448-536 -> (accuracy, class loss, reg loss, reg_all loss) per node."""
    model.eval()
    tot = {"correct": 0.0, "class": 0.0, "reg": 0.0, "reg_all": 0.0}
    S = len(data)
    for i0 in range(0, S, batch_size):
        idx = torch.arange(i0, min(S, i0 + batch_size), device=data.node_obs.device)
        model.netmon.state = None
        enc = model.netmon.encode_nodes(data.node_obs[idx], data.nbr[idx])
        for _ in range(max(sequence_length, 1)):
            out = model(data.node_obs[idx], data.nbr[idx], enc)
        _, terms = _loss_terms(args, out, data.targets_all[idx], data.targets[idx], data.labels[idx], "sum")
        for k, v in terms.items():
            tot[k] += float(v)
        if WITH_CLASSIFICATION:
            tot["correct"] += float((model.get_prediction() == data.labels[idx]).sum())
    model.train()
    count = S * data.node_obs.shape[1]
    res = (tot["correct"] / count, tot["class"] / count, tot["reg"] / count, tot["reg_all"] / (count * args.num_targets))
    if WITH_CLASSIFICATION:
        print(f"{res[0]:.2f} acc, {res[1]} loss")
    if WITH_REGRESSION:
        print(f"Pred loss {res[2]}")
    if WITH_REGRESSION_ALL:
        print(f"Pred_all loss {res[3]}")
    return res


def main(argv=None, quiet=False):
    args = build_parser().parse_args(argv)
    args.test_sequence_lengths = dim_str_to_list(args.test_sequence_lengths)
    L.require_gpu()
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    N = args.n_nodes
    if args.num_targets is None:
        args.num_targets = N
    assert 1 <= args.num_targets <= N
    node_obs_dim = 4 * N + 8
    model = NetMonSL(args, node_obs_dim, NUM_CLASSES, N).cuda()
    M.tag_modules(model, "sl.")
    optim = torch.optim.AdamW(model.parameters())
    model.train()

    n_train = args.batch_size if args.bench else args.num_samples_train
    t0 = time.time()
    train = build_dataset(N, args.n_packets, n_train, args.seed)
    torch.cuda.synchronize()
    if not quiet:
        print(f"train dataset: {len(train)} graphs of {N} nodes in {time.time() - t0:.2f} s", flush=True)

    if args.bench:
        # config 5: every graph of the batch once per iteration (fixed batch = the dataset)
        idx = torch.arange(args.batch_size, device="cuda")
        for _ in range(args.warmup):
            train_step(args, model, optim, train, idx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iterations):
            loss, _ = train_step(args, model, optim, train, idx)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        node_steps = args.iterations * args.batch_size * N * max(args.sequence_length, 1)
        line = {"metric": "node-steps/s (NetMon SL fwd+bwd+AdamW, src/sl.py config 5)",
                "value": round(node_steps / dt, 1), "unit": "node-steps/s", "iterations": args.iterations,
                "ms_per_iteration": round(1e3 * dt / args.iterations, 3), "loss": float(loss),
                "config": {"n_nodes": N, "batch": args.batch_size, "seq_len": args.sequence_length,
                           "netmon_iterations": args.netmon_iterations, "netmon_dim": args.netmon_dim,
                           "encoder": args.netmon_encoder_dim, "rnn": args.netmon_rnn_type}}
        if not quiet:
            print(json.dumps(line))
        return line

    seeds_val = gm.build_seed_list(N, 476, args.num_samples_test, gm.EVAL_SEEDS)
    seeds_test = list(gm.EVAL_SEEDS[:args.num_samples_test]) if N == 20 else \
        gm.build_seed_list(N, 923430603, args.num_samples_test, np.concatenate([gm.EVAL_SEEDS, seeds_val]))
    val = build_dataset(N, args.n_packets, args.num_samples_test, args.seed + 1_000_000, seeds_val)
    test_data = build_dataset(N, args.n_packets, args.num_samples_test, args.seed + 2_000_000, seeds_test)

    losses, validation = [], []
    print("Validation..")
    validation.append((0, *test(args, model, val, args.batch_size, args.sequence_length)))
    for it in range(args.iterations):
        bidx = torch.as_tensor(np.random.choice(len(train), args.batch_size, replace=True), device="cuda")
        total, terms = train_step(args, model, optim, train, bidx)
        losses.append(total)
        if not args.disable_progressbar and (it + 1) % 100 == 0:
            print(f"Iteration {it + 1} | reg_all loss = {float(terms.get('reg_all', 0.0)):.2f} "
                  f"| total = {float(total):.2f}" + (f" (seq_len={args.sequence_length})"
                                                     if args.sequence_length > 1 else ""), flush=True)
        if (it + 1) % args.validate_after == 0:
            print(f"Iteration {it + 1}: validation")
            validation.append((it + 1, *test(args, model, val, args.batch_size, args.sequence_length)))
    print("Train data eval: ")
    train_res = test(args, model, train, args.batch_size, args.sequence_length)
    print(f"Test data eval: (seq_len={args.sequence_length})")
    test_res = test(args, model, test_data, args.batch_size, args.sequence_length)
    seq_results = []
    for sl in args.test_sequence_lengths:
        print(f"Extended test data eval (seq_len={sl})")
        seq_results.append((sl, *test(args, model, test_data, args.batch_size, sl)))
    results = {"total_loss": [float(x) for x in losses], "validation": validation, "train": train_res,
               "test": test_res, "test_sequence": seq_results}
    if args.filename:
        with open(args.filename, "w") as f:
            json.dump(results, f)
    return results


if __name__ == "__main__":
    main()
