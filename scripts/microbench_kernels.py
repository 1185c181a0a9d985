"""Micro-benchmark + in-kernel phase timing of the rollout's fused kernels (trunk, policy/env step) and the
learner's optimiser pair, on the bench configuration (A2C Pong, 32 envs, native engine).

* chained: per-launch time of N back-to-back launches of one kernel captured in a hipGraph (what the kernel costs
  inside the update graph when it is warm);
* phases: per-workgroup s_memrealtime stamps (100 MHz) written by the kernels' diagnostic hooks, reported as the
  median over workgroups of each phase's duration, plus the spread of workgroup start times.
Usage (GPU box): python scripts/microbench_kernels.py [--out gpurun_out/mb.json]
"""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer, KEY_ENV_BITS  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def graph_time(fn, reps=100):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / 5 / reps * 1e6


def phases(st, names):
    st = st.cpu().double() * 10e-3   # ticks of 10 ns -> us
    t0 = st[:, 0].min()
    out = {"start_spread_us": float(st[:, 0].max() - t0)}
    for i in range(1, len(names)):
        d = (st[:, i] - st[:, i - 1])
        out[names[i]] = float(d.median())
    out["total_median_us"] = float((st[:, len(names) - 1] - st[:, 0]).median())
    out["end_from_first_start_us"] = float(st[:, len(names) - 1].max() - t0)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ops = _native.require()
    cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=3)
    for _ in range(10):
        tr.step()
    torch.cuda.synchronize()
    eng, env, st = tr.engine, tr.env, tr.storage
    N = env.num_envs
    lb = eng.bufs(N * st.T, with_grad=True)
    bt = lb.rows(0, N)
    res = {}
    shift_scratch = st.obs[1].clone()
    trunk = lambda stamps=None: ops.cnn_trunk_fwd(st.obs[0], eng.sW1, eng.b1, eng.sW2, eng.b2, eng.sW3, eng.b3,  # noqa
                                                  bt.y1, bt.y2, bt.y3, 1.0 / 255.0, shift_scratch, stamps)
    res["trunk_chained_us"] = graph_time(trunk)
    fc = lambda: G.gemm(bt.y3, 3136, True, eng.sWfc, 512, False, bt.h, 512, 1, N, 512, 3136, bias=eng.bfc,  # noqa
                        relu=True, workspace=eng.ws)
    res["fc_chained_us"] = graph_time(fc)
    # the env step mutates state: run it on scratch copies of the env tensors
    scratch = {k: getattr(env, k).clone() for k in ("state", "t", "tg", "ep_ret", "ep_stats")}
    prev, out = st.obs[0].clone(), st.obs[1].clone()
    rew, done, trunc = st.rewards[0].clone(), st.dones[0].clone(), st.truncated[0].clone()
    act, logp, ent, val = (st.actions[0].clone(), st.logp[0].clone(), st.entropy[0].clone(), st.values[0].clone())

    def pstep(stamps=None):
        ops.env_policy_step_pong(bt.h, eng.sWh, eng.bh, bt.z, act, logp, ent, val, KEY_ENV_BITS, tr.policy_seed,
                                 scratch["state"], scratch["t"], scratch["tg"], scratch["ep_ret"], scratch["ep_stats"],
                                 env.env_ids, prev, out, rew, done, trunc, env.seed, env.max_episode_steps,
                                 env.frame_stack, True, stamps=stamps)
    res["policy_step_chained_us"] = graph_time(pstep)
    opt = tr.actor_opt
    parts = torch.zeros(256, device=eng.dev)
    res["sumsq_chained_us"] = graph_time(lambda: ops.sumsq(opt.g, parts))
    g_copy = opt.g.clone()
    p_copy, v_copy = opt.p.clone(), opt.v.clone()
    lr = opt.lr.clone()
    sh = torch.empty(opt.p.numel(), dtype=torch.bfloat16, device=eng.dev)
    res["rmsprop_chained_us"] = graph_time(lambda: ops.rmsprop_step(p_copy, g_copy, v_copy, lr, parts, None, sh,
                                                                    0.99, 1e-5, -1.0, 0.5, False))
    # in-kernel phases (eager, after a full update so the caches look like the real loop)
    stamps = torch.zeros(max(N, 64), 16, dtype=torch.int64, device=eng.dev)
    tr.step()
    trunk(stamps)
    torch.cuda.synchronize()
    res["trunk_phases"] = phases(stamps[:N], ["start", "stage", "conv1", "conv2", "conv3_issue", "drain"])
    stamps.zero_()
    fc()
    pstep(stamps)
    torch.cuda.synchronize()
    s = stamps[:N].cpu().double() * 10e-3
    t0 = s[:, 0]
    res["policy_phases"] = {
        "start_spread_us": float(t0.max() - t0.min()),
        "head_staged_us": float((s[:, 8] - t0).median()),
        "head_dots_us": float((s[:, 9] - t0).median()),
        "head_sums_us": float((s[:, 10] - t0).median()),
        "head_done_us": float((s[:, 1] - t0).median()),
        "advance_done_us": float((s[:, 2] - t0).median()),
        "shift_issued_us": float((s[:, 3] - t0).median()),
        "barrier_us": float((s[:, 4] - t0).median()),
        "render_issued_us": float((s[:, 5] - t0).median()),
        "drained_us": float((s[:, 6] - t0).median()),
        "end_from_first_start_us": float(s[:, 6].max() - t0.min()),
    }
    res["tuned_gemms"] = {str(k): v for k, v in G.tuned_plans().items()}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
