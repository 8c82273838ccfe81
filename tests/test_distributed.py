"""world_size-2 gloo tests (CPU) of the data-parallel pieces: the bucketed gradient
all-reduce used before clipping, parameter broadcast, and env-seed sharding."""
import importlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        T = importlib.import_module("graph-marl_amd.train")
        torch.manual_seed(100 + rank)  # deliberately different replicas
        model = torch.nn.Sequential(torch.nn.Linear(7, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
        T.broadcast_parameters([model])
        params = list(model.parameters())
        opt = torch.optim.AdamW(params, lr=1e-2)
        x = torch.randn(11, 7) * (rank + 1)
        for _ in range(3):
            loss = model(x).pow(2).mean()
            opt.zero_grad()
            loss.backward()
            local = [p.grad.clone() for p in params]
            T.allreduce_gradients(params)
            gathered = [torch.zeros_like(g) for g in local for _ in range(world)]
            for i, g in enumerate(local):
                out = [torch.zeros_like(g) for _ in range(world)]
                dist.all_gather(out, g)
                avg = sum(out) / world
                assert torch.allclose(params[i].grad, avg, atol=1e-6)
            torch.nn.utils.clip_grad_value_(params, 0.5)
            torch.nn.utils.clip_grad_norm_(params, 1.0)
            opt.step()
        flat = torch.cat([p.detach().reshape(-1) for p in params])
        out = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(out, flat)
        q.put((rank, all(torch.equal(out[0], o) for o in out)))
    finally:
        dist.destroy_process_group()


def test_dp_gradient_allreduce_keeps_replicas_identical():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(2))
    assert res == {0: True, 1: True}


def test_env_seed_shards_are_disjoint():
    T = importlib.import_module("graph-marl_amd.train")
    B, world = 4096, 8
    seeds = [set(T.shard_seeds(r, world, B, base=0)) for r in range(world)]
    assert all(len(s) == B for s in seeds)
    assert len(set().union(*seeds)) == B * world
