"""End-to-end CLI training runs (src/main.py flow) on the device."""
import importlib
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CI_FLAGS = ("--model=dqn --hidden-dim=8 --random-topology=1 --mini-batch-size=32 --device=cpu --episode-steps=1 "
            "--eval-episode-steps=1 --lr=0.001 --tau=0.01 --netmon --netmon-encoder-dim=4 --hidden-dim=4 "
            "--netmon-dim=2 --netmon-iterations=1 --sequence-length=1 --step-before-train=1_000 --capacity=10_000 "
            "--eval-episodes=100 --total-steps=5_000 --env-type=simple --epsilon=0.1 --epsilon-decay=1.0 --seed=0 "
            "--disable-progress")


def test_reference_ci_train_example(tmp_path):
    """The reference's CI check (.github/workflows/train-example.yml): train DQN + NetMon on
    the simple env, then evaluation must report reward_mean 1.0."""
    main = importlib.import_module("graph-marl_amd.main")
    m = main.main(CI_FLAGS.split() + [f"--log-dir={tmp_path}"])
    assert m["reward_mean"] == 1.0
    assert os.path.exists(tmp_path / "model_last.pt")


def test_routing_netmon_train_checkpoint_and_reload(tmp_path):
    main = importlib.import_module("graph-marl_amd.main")
    common = ["--env-type=routing", "--model=dqn", "--netmon", "--netmon-iterations=1", "--n-env=64",
              "--episode-steps=50", "--eval-episodes=64", "--eval-episode-steps=20", "--disable-progressbar"]
    m = main.main(common + ["--total-steps=300", "--step-before-train=100", "--mini-batch-size=32",
                            "--sequence-length=4", "--capacity=20000", f"--log-dir={tmp_path}"])
    for k in ("reward_mean", "delays_mean", "throughput_mean", "spr_mean"):
        assert np.isfinite(m[k]), k
    ck = tmp_path / "model_last.pt"
    assert ck.exists()
    m2 = main.main(common + ["--eval", f"--model-load-path={ck}", "--policy=trained"])
    assert np.isfinite(m2["reward_mean"])


def test_routing_netmon_aux_loss_train(tmp_path, capsys):
    """--aux-loss-coeff > 0: the NetMon aux head trains with the update (src/main.py:586-594,
    868-875, 996-1009) and its loss is logged."""
    main = importlib.import_module("graph-marl_amd.main")
    m = main.main(["--env-type=routing", "--model=dqn", "--netmon", "--netmon-iterations=1", "--n-env=32",
                   "--episode-steps=50", "--total-steps=1000", "--step-before-train=100", "--mini-batch-size=32",
                   "--sequence-length=4", "--capacity=40000", "--aux-loss-coeff=0.5", "--eval-episodes=32",
                   "--eval-episode-steps=20", "--disable-progressbar", f"--log-dir={tmp_path}"])
    assert np.isfinite(m["reward_mean"])
    assert "loss_aux" in capsys.readouterr().out


def test_routing_no_netmon_train(tmp_path):
    main = importlib.import_module("graph-marl_amd.main")
    m = main.main(["--env-type=routing", "--model=dqn", "--random-topology=0", "--n-env=32", "--total-steps=200",
                   "--step-before-train=50", "--mini-batch-size=16", "--episode-steps=100", "--eval-episodes=8",
                   "--eval-episode-steps=20", "--disable-progressbar", f"--log-dir={tmp_path}"])
    assert np.isfinite(m["reward_mean"])


@pytest.mark.parametrize("model", ["dgn", "dqnr", "commnet"])
@pytest.mark.parametrize("netmon", [False, True])
def test_routing_agent_models_train_and_eval(tmp_path, model, netmon):
    """--model dgn / dqnr / commnet through the CLI: rollout with the recurrent state and the
    agent adjacency, replay, updates (DGN with attention regularisation), checkpoint,
    evaluation with per-episode / done-agent state resets, and --eval from the checkpoint."""
    main = importlib.import_module("graph-marl_amd.main")
    common = ["--env-type=routing", f"--model={model}", "--hidden-dim=64,32", "--num-heads=4", "--n-env=16",
              "--episode-steps=30", "--eval-episodes=16", "--eval-episode-steps=10", "--disable-progressbar"]
    if netmon:
        common += ["--netmon", "--netmon-iterations=1", "--netmon-dim=32", "--netmon-encoder-dim=64"]
    m = main.main(common + ["--total-steps=120", "--step-before-train=40", "--mini-batch-size=16",
                            "--sequence-length=3", "--capacity=5000", f"--log-dir={tmp_path}"])
    for k in ("reward_mean", "delays_mean", "throughput_mean"):
        assert np.isfinite(m[k]), k
    ck = tmp_path / "model_last.pt"
    assert ck.exists()
    m2 = main.main(common + ["--eval", f"--model-load-path={ck}", "--policy=trained"])
    assert np.isfinite(m2["reward_mean"])


def test_routing_netmon_global_train(tmp_path):
    main = importlib.import_module("graph-marl_amd.main")
    m = main.main(["--env-type=routing", "--model=dqn", "--netmon", "--netmon-global", "--netmon-iterations=1",
                   "--netmon-dim=32", "--netmon-encoder-dim=64", "--n-env=16", "--total-steps=80",
                   "--step-before-train=30", "--mini-batch-size=16", "--sequence-length=2", "--episode-steps=30",
                   "--eval-episodes=16", "--eval-episode-steps=10", "--disable-progressbar", f"--log-dir={tmp_path}"])
    assert np.isfinite(m["reward_mean"])


@pytest.mark.parametrize("rnn", ["lstm", "gru"])
def test_routing_netmon_no_carryover_train(tmp_path, rnn):
    """--netmon-rnn-carryover 0: the doubled NetMon state goes through rollout, replay and the
    sequence update (unfused NetMon path)."""
    main = importlib.import_module("graph-marl_amd.main")
    m = main.main(["--env-type=routing", "--model=dqn", "--netmon", "--netmon-rnn-carryover=0",
                   f"--netmon-rnn-type={rnn}", "--netmon-iterations=1", "--netmon-dim=32",
                   "--netmon-encoder-dim=64", "--n-env=16", "--total-steps=80", "--step-before-train=30",
                   "--mini-batch-size=16", "--sequence-length=2", "--episode-steps=30", "--eval-episodes=16",
                   "--eval-episode-steps=10", "--disable-progressbar", f"--log-dir={tmp_path}"])
    assert np.isfinite(m["reward_mean"])
