"""Supervised shortest-path driver (src/sl.py, BASELINE config 5) against the reference:
samples (APSP targets, first-hop labels) and one NetMonSL iteration (seq_len 2)."""
import argparse
import importlib
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# sl.npz: N = 20, small NetMon (H 32); sl_n100.npz: BASELINE config 5's N = 100 graphs with the
# CLI-default NetMon (H 128, encoder 512,256)
GOLDENS = ["sl.npz", "sl_n100.npz"]


def _golden(name):
    g = np.load(os.path.join(HERE, name))
    n, H, e0, e1 = (int(v) for v in g["config"]) if "config" in g.files else (20, 32, 64, 48)
    return g, n, H, f"{e0},{e1}"


@pytest.mark.parametrize("name", GOLDENS)
def test_sl_samples_match_reference(name):
    SL = importlib.import_module("graph-marl_amd.sl")
    M = importlib.import_module("graph-marl_amd.model")
    g, n, _, _ = _golden(name)
    seeds = [int(s) for s in g["seeds"]]
    data = SL.build_dataset(n, 20, len(seeds), 0, seeds=seeds)
    np.testing.assert_array_equal(data.targets_all.cpu().numpy(), g["targets_all"])
    np.testing.assert_array_equal(data.labels.cpu().numpy(), g["labels"])
    nbr_ref = M.dense_to_nbr(torch.as_tensor(g["node_adj"], device="cuda"))
    np.testing.assert_array_equal(data.nbr.cpu().numpy(), nbr_ref.cpu().numpy())


@pytest.mark.parametrize("shared_enc", [False, True])
@pytest.mark.parametrize("name", GOLDENS)
def test_sl_iteration_matches_reference(name, shared_enc):
    """shared_enc: the encoder output computed once and reused by both unroll steps (sl.train_step)
    instead of re-encoding at every step like the reference: same predictions and gradients."""
    SL = importlib.import_module("graph-marl_amd.sl")
    M = importlib.import_module("graph-marl_amd.model")
    g, n, H, enc = _golden(name)
    args = argparse.Namespace(netmon_dim=H, netmon_encoder_dim=enc, netmon_iterations=1, netmon_rnn_type="lstm",
                              netmon_rnn_carryover=1, netmon_agg_type="sum", netmon_last_neighbors=1,
                              netmon_global=False, num_targets=n)
    model = SL.NetMonSL(args, 4 * n + 8, 4, n).cuda()
    names = [str(n) for n in g["param_names"]]
    sd = {n: torch.as_tensor(g["w_" + n]) for n in names}
    model.load_state_dict(sd)
    x = torch.as_tensor(g["node_obs"], device="cuda")
    nbr = M.dense_to_nbr(torch.as_tensor(g["node_adj"], device="cuda"))
    tgt = torch.as_tensor(g["targets_all"], device="cuda")
    model.netmon.state = None
    seq = []
    enc = model.netmon.encode_nodes(x, nbr) if shared_enc else None
    for t in range(2):
        _, _, pred_all = model(x, nbr, enc)
        np.testing.assert_allclose(pred_all.detach().cpu().numpy(), g[f"pred_all_{t}"], atol=1e-5, rtol=0,
                                   err_msg=f"pred_all step {t}")
        seq.append(torch.nn.functional.mse_loss(pred_all, tgt))
    total = torch.mean(torch.stack(seq))
    total.backward()
    np.testing.assert_allclose(total.item(), float(g["loss"]), rtol=1e-5)
    params = dict(model.named_parameters())
    for n in names:
        gr = params[n].grad
        got = np.zeros(params[n].shape, np.float32) if gr is None else gr.cpu().numpy()
        np.testing.assert_allclose(got, g["g_" + n], atol=1e-5, rtol=1e-4, err_msg=n)


def test_sl_bench_config5_shape():
    SL = importlib.import_module("graph-marl_amd.sl")
    line = SL.main(["--bench", "--n-nodes=100", "--batch-size=64", "--sequence-length=2", "--netmon-iterations=1",
                    "--iterations=2", "--warmup=1"])
    assert line["value"] > 0 and np.isfinite(line["loss"])


def test_sl_train_short():
    SL = importlib.import_module("graph-marl_amd.sl")
    res = SL.main(["--iterations=20", "--num-samples-train=256", "--num-samples-test=64", "--validate-after=10",
                   "--test-sequence-lengths=1,2", "--disable-progressbar", "--netmon-iterations=1"])
    assert all(np.isfinite(v) for v in res["total_loss"])
    assert len(res["validation"]) == 3 and len(res["test_sequence"]) == 2
