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


def _init_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    T = importlib.import_module("graph-marl_amd.train")
    try:
        r, w, loc = T.init_distributed(use_gpu=False)
        t = torch.tensor([float(r + 1)])
        dist.all_reduce(t)
        q.put((rank, (r, w, loc, float(t), dist.get_backend())))
    finally:
        dist.destroy_process_group()


def test_init_distributed_from_launcher_env():
    """train.init_distributed reads the launcher's RANK / WORLD_SIZE / LOCAL_RANK (the entry of
    main.py and the bench's ranks); world 1 initialises nothing."""
    T = importlib.import_module("graph-marl_amd.train")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    assert T.init_distributed(use_gpu=False) == (0, 1, 0) and not dist.is_initialized()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_init_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = dict(q.get() for _ in range(2))
    assert res == {0: (0, 2, 0, 3.0, "gloo"), 1: (1, 2, 1, 3.0, "gloo")}


def test_bench_gpus_flag_launches_ranks(monkeypatch):
    """bench.py --gpus N (N > 1) outside a launcher runs torch.distributed.run with N ranks on itself
    as a child process; under a launcher WORLD_SIZE must equal --gpus."""
    import subprocess
    import sys

    import bench

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 0)
    args = type("A", (), {"gpus": 4})()
    assert bench.launch_ranks(args, ["--gpus", "4", "--steps", "10"]) == 0
    cmd, env = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[-3:] == ["--gpus", "4", "--steps", "10"][-3:]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    args.gpus = 1
    assert bench.launch_ranks(args, []) is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    args.gpus = 4
    assert bench.launch_ranks(args, []) is None
    bench.check_world(args, 4)
    with pytest.raises(SystemExit):
        bench.check_world(args, 2)


def test_bench_pmc_window_parser(tmp_path):
    """bench.py's same-run PMC probe (measure_pmc) reads the child's counter CSV: the last PMC_S x P
    dispatches of the library's kernels must repeat one step's P launches (the order the child recorded);
    medians per launch per tag, the per-step sum; a window of another shape is rejected."""
    import bench

    S = bench.PMC_S
    order = ["linear:dqn.l0", "linear:dqn.l1+head", "env_step", "linear:netmon.chain", "lstm:obs",
             "mp_aggregate:81920x128", "lstm_agg:upd"]
    kern = ["k_gemm3g_a", "k_gemm3g_b", "k_env_step", "k_gemm3g_c", "k_gemm3g_d", "k_mp_aggregate3", "k_gemm3g_d"]
    rows = [("at::native::fill", 64, 1.0)] * 3 + [("k_env_reset", 4096, 7.0), ("k_gemm3g_a", 655360, 5.0)]
    for s in range(S):
        rows += [(k, 1000, 10.0 * (i + 1) + s) for i, k in enumerate(kern)]
        rows += [("__amd_rocclr_fillBufferAligned", 256, 3.0)]  # not ours: skipped
    p = tmp_path / "c.csv"

    def write(rs):
        with open(p, "w") as f:
            f.write("Dispatch_Id,Kernel_Name,Grid_Size,Counter_Name,Counter_Value\n")
            for i, (n, g, v) in enumerate(rs):
                f.write(f"{i},{n},{g},FETCH_SIZE,{v}\n")

    write(rows)
    per, step = bench._pmc_window(str(p), "FETCH_SIZE", order)
    assert per["env_step"] == 30.0 + S // 2 and per["linear:dqn.l0"] == 10.0 + S // 2
    assert step == sum(10.0 * (i + 1) for i in range(len(kern))) + len(kern) * (S // 2)
    write(rows + [("k_gemm3g_b", 1000, 1.0)])  # one more dispatch after the window: not a whole step
    assert bench._pmc_window(str(p), "FETCH_SIZE", order) is None
    swapped = list(order)
    swapped[2], swapped[3] = swapped[3], swapped[2]  # the env step where the order has a GEMM
    write(rows)
    assert bench._pmc_window(str(p), "FETCH_SIZE", swapped) is None
    assert bench._pmc_window(str(p), "FETCH_SIZE", []) is None


def test_bench_committed_traffic_prefers_same_sources(tmp_path, monkeypatch):
    """The committed-profile fallback (bench.pmc_traffic) takes a profile whose source hash is the build's,
    else the newest (round, seq, file time), never the largest byte count."""
    import json

    import bench

    def prof(rnd, name, src, seq, fetch):
        d = tmp_path / "profiles" / rnd / name
        d.mkdir(parents=True)
        (d / "pmc_traffic.json").write_text(json.dumps(
            {"src": src, "seq": seq, "kernels": {"k": {"fetch_bytes": fetch, "write_bytes": 0}}}))

    prof("r05", "a", "aaaa", 0, 900)
    prof("r05", "b", "bbbb", 0, 100)
    prof("r04", "c", "cccc", 3, 50)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    tb, note = bench.pmc_traffic("k", "bbbb")
    assert tb == 100 and "same sources" in note
    os.utime(tmp_path / "profiles" / "r05" / "a" / "pmc_traffic.json", (1, 1))
    tb, note = bench.pmc_traffic("k", "zzzz")  # no same-source profile: the newest file of the newest round
    assert tb == 100 and "OTHER sources (bbbb)" in note
    assert bench.pmc_traffic("missing", "bbbb") == (None, None)


def _fail_worker(rank, world, port, q, fail_at, steps, update_every):
    """main.py's loop protocol on gloo: every rank steps; every `update_every` steps it exchanges
    gradients; rank 1 raises at step fail_at (in its 'rollout', before the exchange) and posts the
    abort; at the end every rank that did not fail runs finish_sync."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank), GM_DIST_TIMEOUT="120")
    T = importlib.import_module("graph-marl_amd.train")
    T.DIST_TIMEOUT_S = 120.0
    T.init_distributed(use_gpu=False)
    t0 = time.time()
    model = torch.nn.Linear(4, 3)
    params = list(model.parameters())
    err = None
    last = 0
    try:
        try:
            for step in range(1, steps + 1):
                if rank == 1 and step == fail_at:
                    raise ValueError("injected")
                if step % update_every == 0:
                    model.zero_grad()
                    model(torch.randn(5, 4)).sum().backward()
                    T.allreduce_gradients(params)
                    last = step
        except Exception as e:  # noqa: BLE001 (the protocol under test)
            err = e
            if not isinstance(e, T.PeerFailure):
                T.abort_peers(params)
        if err is None:
            try:
                T.finish_sync(params)
            except T.PeerFailure as e:
                err = e
        q.put((rank, type(err).__name__ if err else None, last, time.time() - t0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fail_at,steps,expect_last0", [(5, 10, 4), (11, 11, 10), (None, 10, 10)])
def test_rank_failure_stops_every_rank(fail_at, steps, expect_last0):
    """A rank that raises mid-training (VERDICT / ADVICE r04: round 4 left its peers blocked in the next
    all_reduce until the collective timeout) makes every rank leave the loop together: rank 1 fails at
    step 5, rank 0 raises PeerFailure in the exchange of step 6 (its last completed update: step 4);
    rank 1 fails at step 11 after both ranks' last update (step 10), rank 0 raises in the end-of-loop
    sync. Both well inside the 120 s collective timeout; without a failure both finish normally."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, 2, port, q, fail_at or 0, steps, 2)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
        assert p.exitcode == 0
    res = {r: rest for r, *rest in (q.get() for _ in range(2))}
    if fail_at is None:
        assert res[0][:2] == [None, expect_last0] and res[1][:2] == [None, expect_last0], res
        return
    assert res[1][0] == "ValueError", res
    assert res[0][:2] == ["PeerFailure", expect_last0], res
    assert max(r[2] for r in res.values()) < 60, res  # far below the 120 s collective timeout


def test_init_distributed_refuses_fewer_gpus_than_ranks(monkeypatch):
    """Round 4 silently ran every rank on cuda:0 over gloo when the node showed fewer GPUs than local
    ranks; now that is an error unless GM_DIST_SHARE_GPU=1 asks for the one-GPU rehearsal."""
    T = importlib.import_module("graph-marl_amd.train")
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("LOCAL_RANK", "0")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.delenv("GM_DIST_SHARE_GPU", raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 1)
    with pytest.raises(RuntimeError, match="visible GPUs"):
        T.init_distributed(use_gpu=True)
    assert not dist.is_initialized()
