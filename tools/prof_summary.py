#!/usr/bin/env python3
"""Summarise rocprofv3 CSVs (kernel trace + PMC FETCH_SIZE/WRITE_SIZE passes) per
kernel and launch shape. Usage:
  python tools/prof_summary.py --trace gpurun_out/prof/bench_kernel_trace.csv \
      [--fetch gpurun_out/pmc/fetch_counter_collection.csv --write gpurun_out/pmc/write_counter_collection.csv]
HBM bytes follow MI355X_MICROARCH.md §HBM: counters are KiB; FETCH_SIZE reads 1/2 of
a wide (16 B/lane) coalesced stream on gfx950, so the corrected read figure is 2x.
"""
import argparse
import csv
from collections import defaultdict


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def key(r):
    g = r.get("Grid_Size") or r.get("Grid_Size_X")
    w = r.get("Workgroup_Size") or r.get("Workgroup_Size_X")
    return r["Kernel_Name"], int(g), int(w)


NETMON = ["netmon.enc0(K=88)", "netmon.enc1(K=512)", "netmon.enc2(K=256)", "netmon.rnn_obs(K=256)",
          "netmon.rnn_update(K=256)"]
DQN = ["dqn.enc0(K=642)", "dqn.enc1(K=512)", "dqn.q(K=256)"]


# k_gemm (gm_gemm_f32, fused path): encoder layer 0 runs in k_routing_enc, the LSTM
# cells carry their gate epilogue, the DQN's first layer gathers the NetMon readout
# (round 5: encoder layers 1-3 are one launch, gm_encoder_x3; --netmon-layers for older profiles)
NETMON_G_LAYERS = ["netmon.enc1(K=512)", "netmon.enc2(K=256)", "netmon.rnn_obs(K=128+128)",
                   "netmon.rnn_update(K=sum128+128)"]
NETMON_G = ["netmon.enc(layers 1-3 chained)", "netmon.rnn_obs(K=128+128)", "netmon.rnn_update(K=sum128+128)"]
def dqn_g(env_k=128, fused_head=True):
    """DQN layer labels of the fused rollout; env_k = env-obs columns of layer 1 (128 with the
    GEMM-ready obs copy, 130 without); before gm_gemm_x3_head the head was a third GEMM."""
    l1 = f"dqn.enc0(K=512 readout+{env_k})"
    return [l1, "dqn.enc1+q(K=512, Q head fused)"] if fused_head else [l1, "dqn.enc1(K=512)", "dqn.q(K=256)"]


DQN_G = dqn_g()


def linear_labels(n_dispatch, episode_steps, netmon_iters=1, netmon=NETMON, dqn=DQN):
    """Call-site names of the GEMM dispatches of one bench.py process, in launch
    order: reset (NetMon start-up step), then per step the DQN layers + 1 NetMon step,
    and a reset after every `episode_steps` steps."""
    nm = netmon[:-1] + [netmon[-1]] * netmon_iters
    out = list(nm)
    step = 0
    while len(out) < n_dispatch:
        out += dqn + nm
        step += 1
        if step % episode_steps == 0:
            out += nm
    return out[:n_dispatch]


def relabel(rows, episode_steps, dqn_g=DQN_G, netmon_g=None):
    for r in rows:  # k_gemm3<...> (split-f16 form) and k_gemm<...> (f32) are one call-site sequence
        if "k_gemm3" in r["Kernel_Name"] or r["Kernel_Name"].startswith("k_gemm") or "k_gemmI" in r["Kernel_Name"]:
            r["Kernel_Name"] = "k_gemm"
    for name, nm, dq in (("k_linear_f32", NETMON, DQN), ("k_gemm", netmon_g or NETMON_G, dqn_g)):
        lin = [r for r in rows if r["Kernel_Name"].startswith(name)]
        for r, lab in zip(lin, linear_labels(len(lin), episode_steps, netmon=nm, dqn=dq)):
            r["Kernel_Name"] = f"{name}[{lab}]"
    return rows


def bench_tag(name, grid, rows, env_k=128):
    """bench.py timer tag of a relabelled kernel (default rollout: N=20, H=128, M = rows; env_k:
    the env-obs columns of DQN layer 1, 128 with the GEMM-ready obs copy, 130 without)."""
    M = rows
    gemm = {
        f"dqn.enc0(K=512 readout+{env_k})": f"linear:dqn.encoder.linear_layers.0:{M}x512x{512 + env_k}",
        "dqn.enc1+q(K=512, Q head fused)": f"linear:dqn.encoder.linear_layers.1+head:{M}x256x512",
        "netmon.enc(layers 1-3 chained)": f"linear:netmon.encode.linear_layers.1+chain:{M}x256x512",
        "netmon.enc1(K=512)": f"linear:netmon.encode.linear_layers.1:{M}x256x512",
        "netmon.enc2(K=256)": f"linear:netmon.encode.linear_layers.2:{M}x128x256",
        "netmon.rnn_obs(K=128+128)": f"lstm:netmon.rnn_obs:{M}x512x256",
        "netmon.rnn_update(K=sum128+128)": f"lstm_agg:netmon.rnn_update:{M}x512x256",
    }
    if name.startswith("k_gemm[") and name.endswith("]"):
        return gemm.get(name[7:-1])
    if name.startswith("k_env_step"):
        return "env_step"
    if name.startswith("k_mp_aggregate"):
        return f"mp_aggregate:{M}x128"
    if name.startswith("k_routing_enc"):
        return f"routing_enc:netmon.encode.linear_layers.0:{M}x512"
    if name.startswith("k_policy_egreedy"):
        return "egreedy"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--top", type=int, default=20)
    ap.add_argument("--episode-steps", type=int, default=50)
    ap.add_argument("--unfused-head", action="store_true", help="profiles taken before gm_gemm_x3_head")
    ap.add_argument("--json", help="write per-launch HBM bytes keyed by bench.py timer tags (pmc_traffic.json)")
    ap.add_argument("--src", help="build.src of the profiled library (recorded; bench.py compares it)")
    ap.add_argument("--rows", type=int, default=81920, help="GEMM rows of the profiled rollout (n_env * N)")
    ap.add_argument("--env-k", type=int, default=128,
                    help="env-obs columns of DQN layer 1 (128: GEMM-ready obs copy, 130: the round-1/2 profiles)")
    ap.add_argument("--netmon-layers", action="store_true", help="profiles taken before gm_encoder_x3 (round 5)")
    a = ap.parse_args()
    nmg = NETMON_G_LAYERS if a.netmon_layers else NETMON_G
    dqn_g_ = dqn_g(a.env_k, not a.unfused_head)
    dur = defaultdict(list)
    trace = load(a.trace)
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    for r in relabel(trace, a.episode_steps, dqn_g_, nmg):
        dur[key(r)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = defaultdict(dict)
    for name, path in (("FETCH_SIZE", a.fetch), ("WRITE_SIZE", a.write)):
        if not path:
            continue
        acc = defaultdict(list)
        rows = [r for r in load(path) if r["Counter_Name"] == name]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        for r in relabel(rows, a.episode_steps, dqn_g_, nmg):
            if r["Counter_Name"] == name:
                acc[key(r)].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            pmc[k][name] = sum(v) / len(v)
    total = sum(sum(v) for v in dur.values())
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    print("| kernel | grid (threads) | wg | calls | avg us | share % | FETCH KiB/launch (x2 corr.) | WRITE KiB/launch |")
    print("|---|---|---|---|---|---|---|---|")
    for (n, g, w), v in rows:
        p = pmc.get((n, g, w), {})
        fe = p.get("FETCH_SIZE")
        wr = p.get("WRITE_SIZE")
        fes = "" if fe is None else f"{fe:.0f} ({2 * fe:.0f})"
        wrs = "" if wr is None else f"{wr:.0f}"
        print(f"| {n} | {g} | {w} | {len(v)} | {sum(v) / len(v) / 1e3:.1f} | {100 * sum(v) / total:.1f} | {fes} | {wrs} |")
    if a.json:
        import json

        out = {}
        for (n, g, w), p in pmc.items():
            tag = bench_tag(n, g, a.rows, a.env_k)
            if tag and "FETCH_SIZE" in p and "WRITE_SIZE" in p and tag not in out:
                # KiB per launch; FETCH_SIZE doubled (gfx950 counts half of a 16-B/lane stream)
                out[tag] = {"fetch_bytes": int(2 * p["FETCH_SIZE"] * 1024), "write_bytes": int(p["WRITE_SIZE"] * 1024),
                            "kernel": n, "grid": g}
        with open(a.json, "w") as f:
            json.dump({"source": {"trace": a.trace, "fetch": a.fetch, "write": a.write}, "src": a.src, "kernels": out}, f,
                      indent=1)


if __name__ == "__main__":
    main()
