"""TensorBoard summaries (reference C15 ``variable_summaries`` + C30 ``FileWriter``): event-file framing and the
reference's per-variable tags, for the parity trainer and the vectorised trainer."""
import glob
import os

import numpy as np
import pytest
import torch

from actor_critic_algs_on_tensorflow_amd.ops.stats import seg_stats
from actor_critic_algs_on_tensorflow_amd.utils import tensorboard as TB


def test_event_file_roundtrip_and_crc(tmp_path):
    w = TB.SummaryWriter(str(tmp_path))
    w.add_scalars({"a/b": 1.5, "c": -2.25}, step=3)
    w.add_scalar("a/b", 0.1, step=300)
    w.close()
    ev = TB.read_events(w.path)
    assert ev[0]["file_version"] == "brain.Event:2"
    assert ev[1]["step"] == 3 and ev[1]["scalars"] == {"a/b": 1.5, "c": -2.25}
    assert ev[2]["step"] == 300 and abs(ev[2]["scalars"]["a/b"] - 0.1) < 1e-7
    raw = bytearray(open(w.path, "rb").read())
    raw[-6] ^= 1
    open(w.path, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        TB.read_events(w.path)


def test_summaries_dir_is_reference_layout():
    assert TB.summaries_dir("log.txt") == os.path.join("summaries", "log.data")
    assert TB.summaries_dir("runs/exp1.txt", "tb") == os.path.join("tb", "runs/exp1.data")


def test_seg_stats_cpu_matches_float64():
    x = torch.randn(1000)
    segs = torch.tensor([[0, 1], [5, 100], [200, 800]])
    st = seg_stats(x, segs)
    for i, (o, n) in enumerate(segs.tolist()):
        v = x[o:o + n].double()
        want = [v.mean().item(), v.std(unbiased=False).item(), v.max().item(), v.min().item()]
        assert np.allclose(st[i].tolist(), want, rtol=1e-6, atol=1e-7)


def test_basic_ac_writes_reference_tags(tmp_path):
    from actor_critic_algs_on_tensorflow_amd.api import train
    out = str(tmp_path / "log.txt")
    r = train("basic_ac", env="CartPole-v0", total_updates=2, outdir=out, quiet=True, save_every=0,
              checkpoint_dir=None, ep_length_stop=200, tboard=True, tb_root=str(tmp_path))
    files = glob.glob(os.path.join(TB.summaries_dir(out, str(tmp_path)), "events.out.tfevents.*"))
    assert len(files) == 1
    ev = TB.read_events(files[0])
    assert [e["step"] for e in ev[1:]] == [0, 1]
    last = ev[-1]["scalars"]
    # Critic: its own 8 variables; Actor: the Critic's 8, then its own 8 (discrete head: no log-std)
    assert "Critic/var_7summaries/mean" in last and "Critic/var_8summaries/mean" not in last
    assert "Actor/var_15summaries/mean" in last and "Actor/stddev_15/min" in last
    assert "Actor/var_16summaries/mean" not in last
    assert last["Actor/var_0summaries/mean"] == last["Critic/var_0summaries/mean"]
    k = r.trainer.critic.net.first_layer.kernel.detach().double()
    assert abs(last["Critic/var_0summaries/mean"] - k.mean().item()) < 1e-6
    assert abs(last["Critic/stddev/stddev"] - k.std(unbiased=False).item()) < 1e-6
    wk = r.trainer.actor.net.first_layer.kernel.detach().double()
    assert abs(last["Actor/stddev_8/max"] - wk.max().item()) < 1e-6


def test_vectorised_trainer_tboard_and_phase_timers(tmp_path):
    from actor_critic_algs_on_tensorflow_amd import preset
    from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
    out = str(tmp_path / "run.txt")
    metrics = str(tmp_path / "m.jsonl")
    tr = ActorCriticTrainer(preset("mujoco_ppo_dp8", num_envs=4, n_steps=8, ppo_minibatches=2, ppo_epochs=1,
                                   device="cpu", cuda_graph=False, outdir=out, quiet=True, stdout_freq=1,
                                   save_every=0, tboard=True, tb_root=str(tmp_path), trace=True,
                                   metrics_path=metrics))
    tr.train(3)
    tr.close()
    files = glob.glob(os.path.join(TB.summaries_dir(out, str(tmp_path)), "events.*"))
    ev = TB.read_events(files[0])
    assert [e["step"] for e in ev[1:]] == [0, 1, 2]
    s = ev[-1]["scalars"]
    # continuous head: the Actor scope has 8 critic + 8 actor + log-std = 17 variables
    assert "Actor/var_16summaries/mean" in s and "Actor/var_17summaries/mean" not in s
    assert "train/act_loss" in s
    k = tr.model.critic.first_layer.kernel.detach().double()
    assert abs(s["Critic/var_0summaries/mean"] - k.mean().item()) < 1e-6
    ls = tr.model.actor.log_std.detach().double()
    assert abs(s["Actor/var_16summaries/mean"] - ls.mean().item()) < 1e-6
    import json
    rows = [json.loads(x) for x in open(metrics)]
    assert set(rows[-1]["phase_ms"]) == {"rollout", "returns", "learn"}
