"""Per-kernel A/B micro-benchmark of the headline config's rollout / learner kernels (graph-chained launches, warm,
interleaved rounds in one process -- cdna_hip_programming.md §5.4 rule 24).

Usage (GPU box): python scripts/microbench_r2.py [--out gpurun_out/mb_r2.json] [--rounds 5]
"""
import argparse
import json
import statistics
import sys
import time

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def make_graph(fn, reps):
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
    return g


def time_graph(g, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / 5 / reps * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    ops = _native.require()
    cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=3)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    eng, st = tr.engine, tr.storage
    N = tr.env.num_envs
    lb = eng.bufs(N * st.T, with_grad=True)
    bt = lb.rows(0, N)
    scratch = st.obs[1].clone()
    cands = {}
    for mode in (3, 1, 2):
        cands[f"trunk_mode{mode}"] = (lambda m=mode: ops.cnn_trunk_fwd(
            st.obs[0], eng.sW1, eng.b1, eng.sW2, eng.b2, eng.sW3, eng.b3, bt.y1, bt.y2, bt.y3, 1.0 / 255.0, scratch,
            None, m, None))
    hp = eng.hpart(N)
    cands["fc_parts"] = lambda: G.gemm(bt.y3, 3136, True, eng.sWfc, 512, False, hp, 512, 3, N, 512, 3136,
                                       workspace=eng.ws, max_planes=32)
    # learner data-gradient chain at the bench batch (B = T * N = 160): fused per-sample kernel vs the two GEMMs
    B = lb.B
    biasp = torch.zeros(B, 160, device="cuda:0")
    cands["bwd_fused_dy2_dy1"] = lambda: ops.cnn_trunk_bwd(lb.dy3, eng.sW3, lb.y2, eng.sW2, lb.y1, lb.dy2, lb.dy1,
                                                           biasp)
    cs2 = torch.zeros(64, device="cuda:0")
    cs1 = torch.zeros(32, device="cuda:0")

    def gemms():
        G.gemm(lb.dy3, 0, True, eng.sW3, 0, False, lb.dy2, 64, 1, B * 81, 64, 576, mask=lb.y2, ldm=64, colsum=cs2,
               workspace=eng.ws, ga=[3, B, 64, 9, 9, 3, 3, 1], gb=[4, 1, 64, 1, 64, 3, 3, 1])
        G.gemm(lb.dy2, 0, True, eng.sW2, 0, False, lb.dy1, 32, 1, B * 400, 32, 256, mask=lb.y1, ldm=32, colsum=cs1,
               workspace=eng.ws, ga=[5, B, 64, 20, 20, 4, 4, 2], gb=[6, 1, 64, 1, 32, 4, 4, 2])
    cands["bwd_gemms_dy2_dy1"] = gemms
    eng.defer_finalize = False   # time the finaliser itself (the trainer folds it into the optimiser launch)
    cands["finalize_engine"] = lambda: eng.finalize(lb)
    fw = list(eng._fin_words.values())[-1][0]
    bias_w = fw[(fw[:, 1] != 0) & (fw[:, 2] <= 64)].clone()
    plane_w = fw[(fw[:, 1] != 0) & (fw[:, 2] > 64)].clone()
    ro_w = fw[fw[:, 1] == 0].clone()
    cands["finalize_planes_only"] = lambda: ops.grad_finalize(plane_w, eng.fin_parts)
    cands["finalize_bias_only"] = lambda: ops.grad_finalize(bias_w, eng.fin_parts)
    cands["finalize_readonly_only"] = lambda: ops.grad_finalize(ro_w, eng.fin_parts)
    cands["sumsq_slab"] = lambda: ops.sumsq(eng.flat.grad, eng.fin_parts)
    # fused A2C head (loss + head backward) on the rollout's buffers
    cfg_ = tr.cfg
    rets = dict(mode=1, rew=st.rewards, val=st.values, dones=st.dones, L=st.T, gamma=cfg_.gamma, lam=cfg_.gae_lambda,
                norm_adv=cfg_.norm_adv, ret_w=tr._ret_w, adv_w=tr._adv_w)
    acts, lpo = st.flat("actions"), st.flat("logp")
    sbuf = torch.zeros(16, device="cuda:0")
    cands["head_bwd"] = lambda: eng.head_backward(lb, acts, lpo, tr.ent_coef, tr.kl_coef, cfg_.vf_coef, sbuf, rets)
    graphs = {k: make_graph(f, a.reps) for k, f in cands.items()}
    res = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            res[k].append(time_graph(g, a.reps))
    out = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in res.items()}
    # in-kernel phase stamps of the row-split trunk (slots: 0 entry, 1 staged, 2 conv1, 3 conv2, 4 conv3, 5 drained)
    stamps = torch.zeros(N * 7, 16, dtype=torch.int64, device="cuda:0")
    ops.cnn_trunk_fwd(st.obs[0], eng.sW1, eng.b1, eng.sW2, eng.b2, eng.sW3, eng.b3, bt.y1, bt.y2, bt.y3,
                      1.0 / 255.0, scratch, stamps, 1, None)
    torch.cuda.synchronize()
    s = stamps.cpu().double() * 10e-3
    t0 = s[:, 0].min()
    names = ["entry", "staged", "conv1", "conv2", "conv3", "drained"]
    ph = {"start_spread_us": float(s[:, 0].max() - t0)}
    for i in range(1, 6):
        ph[names[i]] = float((s[:, i] - s[:, i - 1]).median())
    ph["end_from_first_start_us"] = float(s[:, 5].max() - t0)
    out["trunk_rows_phases"] = ph
    # fused backward phases (0 entry, 1 staged, 2 dy2, 3 W2 in + dy2 out + db3/db2, 4 dy1, 5 dy1 out, 6 drained)
    st2 = torch.zeros(B, 16, dtype=torch.int64, device="cuda:0")
    ops.cnn_trunk_bwd(lb.dy3, eng.sW3, lb.y2, eng.sW2, lb.y1, lb.dy2, lb.dy1, biasp, st2)
    torch.cuda.synchronize()
    s2 = st2.cpu().double() * 10e-3
    t0 = s2[:, 0].min()
    names = ["entry", "staged", "dy2", "w2_dy2out_db", "dy1", "dy1_out", "drained"]
    ph = {"start_spread_us": float(s2[:, 0].max() - t0)}
    for i in range(1, 7):
        ph[names[i]] = float((s2[:, i] - s2[:, i - 1]).median())
    ph["end_from_first_start_us"] = float(s2[:, 6].max() - t0)
    out["trunk_bwd_phases"] = ph
    # policy/env step phases (slots: 0 entry, 8 fc planes reduced + Wh loaded, 9 head partials, 10 logits,
    # 1 sampled, 4 barrier, 5 committed + rendered (issued), 6 drained)
    env = tr.env
    eng.forward(st.obs[0], bt, head=False, shift_out=scratch, fc_parts=True)
    hp_, S_ = eng.last_fc
    st4 = torch.zeros(N, 16, dtype=torch.int64, device="cuda:0")
    outs = [torch.empty_like(st.actions[0]), torch.empty_like(st.logp[0]), torch.empty_like(st.entropy[0]),
            torch.empty_like(st.values[0]), torch.empty_like(st.rewards[0]), torch.empty_like(st.dones[0]),
            torch.empty_like(st.truncated[0])]
    scratch2 = scratch.clone()
    ops.env_policy_step_pong(bt.h, eng.sWh, eng.bh, bt.z, outs[0], outs[1], outs[2], outs[3], 20, tr.policy_seed,
                             env.state, env.t, env.tg, env.ep_ret, env.ep_stats, env.env_ids, st.obs[0], scratch2,
                             outs[4], outs[5], outs[6], env.seed, env.max_episode_steps, env.frame_stack, True, hp_,
                             S_, eng.bfc, st4)
    torch.cuda.synchronize()
    s4 = st4.cpu().double() * 10e-3
    t0 = s4[:, 0].min()
    seq = [(8, "fc_reduce_wh"), (9, "head_partials"), (10, "logits"), (1, "sample"), (4, "barrier"),
           (5, "commit_render_issue"), (6, "drained")]
    ph = {"start_spread_us": float(s4[:, 0].max() - t0)}
    prev = 0
    for slot, name in seq:
        ph[name] = float((s4[:, slot] - s4[:, prev]).median())
        prev = slot
    ph["end_from_first_start_us"] = float(s4[:, 6].max() - t0)
    out["policy_phases"] = ph
    st3 = torch.zeros(8, 16, dtype=torch.int64, device="cuda:0")
    r = rets
    ops.head_bwd(lb.z, acts, lpo, tr.ent_coef, tr.kl_coef, float(cfg_.vf_coef), r["rew"], r["val"], r["dones"],
                 int(r["L"]), 1, bool(r["norm_adv"]), float(r["gamma"]), float(r["lam"]), r["ret_w"], r["adv_w"],
                 lb.h, eng.sWh, lb.dh, eng.gWh, eng.gbh, eng.gbfc, sbuf, st3)
    torch.cuda.synchronize()
    s3 = st3.cpu().double() * 10e-3
    t0 = s3[:, 0].min()
    names = ["entry", "loads", "returns_reduce", "loss_reduce", "head_compute", "head_reduce_store", "drained"]
    ph = {"start_spread_us": float(s3[:, 0].max() - t0)}
    for i in range(1, 7):
        ph[names[i]] = float((s3[:, i] - s3[:, i - 1]).median())
    ph["end_from_first_start_us"] = float(s3[:, 6].max() - t0)
    out["head_bwd_phases"] = ph
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
