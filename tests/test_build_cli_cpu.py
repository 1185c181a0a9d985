"""Native build artefacts load on CPU; reference-compatible CLIs run."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

OPS = ["env_step_cartpole", "env_step_pendulum", "env_step_linear", "env_step_pong", "categorical_sample",
       "categorical_sample_env", "gaussian_sample", "gae", "nstep_returns", "normalize", "moments", "ev", "sumsq",
       "adam_step", "rmsprop_step", "cast_bf16", "gemm", "im2col_u8", "im2col_nhwc", "col2im_nhwc", "colsum_bf16",
       "ac_loss"]


def test_native_library_registers_every_op():
    import torch
    from actor_critic_algs_on_tensorflow_amd import _native
    assert _native.load(raise_on_error=True)
    ops = torch.ops.acamd
    assert ops.ping() == 355
    for name in OPS:
        assert hasattr(ops, name), name
    # gfx950 code object is embedded in the library
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_gpu_ops_refuse_cpu_tensors():
    import torch
    from actor_critic_algs_on_tensorflow_amd import _native
    ops = _native.require()
    with pytest.raises(Exception):
        ops.normalize(torch.zeros(4), torch.zeros(4), 1e-8)


def _run(args, cwd):
    return subprocess.run([sys.executable, "-m"] + args, cwd=cwd, capture_output=True, text=True, timeout=600,
                          env=dict(os.environ, PYTHONPATH=ROOT))


def test_cli_run_ac_and_test_model(tmp_path):
    r = _run(["actor_critic_algs_on_tensorflow_amd.cli.run_ac", "--env", "CartPole-v0", "--iters", "2",
              "--outdir", str(tmp_path / "log.txt"), "--checkpoint_dir", str(tmp_path / "tmp" / "checkpoints"),
              "--save_every", "1", "--quiet"], str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "done: 2 iterations" in r.stdout
    lines = open(tmp_path / "log.txt").read().splitlines()
    assert lines[0].startswith("step avg_rew") and len(lines) == 3
    ck = [f for f in os.listdir(tmp_path / "tmp") if f.endswith(".index")]
    assert ck
    r = _run(["actor_critic_algs_on_tensorflow_amd.cli.test_model", "CartPole-v0",
              str(tmp_path / "tmp" / ck[0][:-len(".index")]), "--no_animation", "--num_episodes", "2"], str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "Average reward over 2 was" in r.stdout


def test_cli_vectorised_a2c(tmp_path):
    r = _run(["actor_critic_algs_on_tensorflow_amd.cli.run_ac", "--algo", "a2c", "--env", "CartPole-v1", "--iters",
              "30", "--num_envs", "4", "--outdir", str(tmp_path / "log.txt"), "--save_every", "0", "--quiet",
              "--metrics", str(tmp_path / "m.jsonl")], str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "env-steps/s" in r.stdout
    assert os.path.getsize(tmp_path / "m.jsonl") > 0
