"""In-kernel phase stamps of the headline rollout step (cnn_fused.hip pong_fused_step_kernel) on the headline config
(32 envs): slots 0 entry, 1 head + sample + env + render staged (after the staging barrier), 2 conv1, 3 conv2,
4 conv3 + owned-row stores issued, 5 drained (s_memrealtime, 100 MHz; per-workgroup medians over the 224 row
workgroups). Also the first-observation trunk (cnn_trunk_rows_kernel, same slots from 1 on) in both weight-load
modes.

Usage (GPU box): python scripts/microbench_fused_step.py [--out gpurun_out/mb_step.json]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import KEY_ENV_BITS, ActorCriticTrainer  # noqa: E402


def phases(st, names):
    s = st.cpu().double() * 10e-3
    t0 = s[:, 0].min()
    ph = {"start_spread_us": float(s[:, 0].max() - t0)}
    prev = 0
    for slot, name in names:
        ph[name] = float((s[:, slot] - s[:, prev]).median())
        prev = slot
    ph["end_from_first_start_us"] = float(s[:, names[-1][0]].max() - t0)
    return ph


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops = _native.require()
    cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=3)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    eng, st, env = tr.engine, tr.storage, tr.env
    N = env.num_envs
    b = eng.bufs(N)
    nxt = eng.bufs(N)
    out = {}
    scratch = st.obs[1].clone()
    for mode in (1, 2):
        for rep in range(3):
            stamps = torch.zeros(N * 7, 16, dtype=torch.int64, device="cuda:0")
            ops.cnn_trunk_fwd(st.obs[0], eng.sW1, eng.b1, eng.sW2, eng.b2, eng.sW3, eng.b3, b.y1, b.y2, b.y3,
                              1.0 / 255.0, scratch, stamps, mode, None)
            torch.cuda.synchronize()
        out[f"trunk_rows_mode{mode}"] = phases(stamps, [(1, "staged"), (2, "conv1"), (3, "conv2"), (4, "conv3_issue"),
                                                        (5, "drained")])
    eng.forward(st.obs[0], b, head=False, fc_parts=True)
    hp, S = eng.last_fc
    obs_a, obs_b, obs_c = st.obs[0].clone(), st.obs[1].clone(), st.obs[2].clone()
    res = []
    for rep in range(3):
        stamps = torch.zeros(N * 7, 16, dtype=torch.int64, device="cuda:0")
        sn, tn, tgn, ern = env.next_state()
        outs = [torch.empty_like(st.actions[0]), torch.empty_like(st.logp[0]), torch.empty_like(st.entropy[0]),
                torch.empty_like(st.values[0]), torch.empty_like(st.rewards[0]), torch.empty_like(st.dones[0]),
                torch.empty_like(st.truncated[0])]
        ops.pong_fused_step(b.h, eng.sWh, eng.bh, b.z, outs[0], outs[1], outs[2], outs[3], KEY_ENV_BITS,
                            tr.policy_seed, env.state, env.t, env.tg, env.ep_ret, sn, tn, tgn, ern, env.ep_stats,
                            env.env_ids, obs_a, obs_b, outs[4], outs[5], outs[6], env.seed, env.max_episode_steps, hp,
                            S, eng.bfc, eng.sW1, eng.b1, eng.sW2, eng.b2, eng.sW3, eng.b3, nxt.y1, nxt.y2, nxt.y3,
                            1.0 / 255.0, obs_c, stamps)
        torch.cuda.synchronize()
        res.append(stamps)
    out["pong_fused_step"] = phases(res[-1], [(1, "head_env_render_staged"), (2, "conv1"), (3, "conv2"),
                                              (4, "conv3_issue"), (5, "drained")])
    st = res[-1].cpu().double() * 10e-3
    if bool((st[:, 6:10] != 0).any()):   # probe builds: wave 0's conv1 sub-phases (slots 6..9) from slot 1
        out["pong_fused_step_conv1_wave0"] = {f"slot{k}": float((st[:, k] - st[:, 1]).median()) for k in range(6, 10)
                                               if bool((st[:, k] != 0).all())}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
