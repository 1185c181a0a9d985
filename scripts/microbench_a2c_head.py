"""In-kernel phase stamps + graph-chained time of the A2C head launch (loss.hip a2c_head_kernel) on the headline
config's buffers (32 envs x 5 steps). Stamp slots per workgroup (s_memrealtime, 100 MHz): 0 entry, 1 bootstrap
values + operand loads + grid barrier, 2 returns + moments, 3 loss + dz, 4 head backward + lane reduction, 5 wave
reduction + stores issued, 6 drained.

Usage (GPU box): python scripts/microbench_a2c_head.py [--out gpurun_out/mb_head.json]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "scripts")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


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
    N, T = tr.env.num_envs, st.T
    lb = eng.bufs(N * T, with_grad=True)
    bt = eng.bufs(N)
    eng.forward(st.obs[T], bt, head=False, fc_parts=True)
    hp, S = eng.last_fc
    acts, lpo = st.flat("actions"), st.flat("logp")
    sbuf = torch.zeros(16, device="cuda:0")
    bar = torch.zeros(4, dtype=torch.int32, device="cuda:0")
    val = st.values.clone()
    c = cfg

    def launch(stamps=None, boot=True):
        ops.a2c_head(lb.z, acts, lpo, tr.ent_coef, tr.kl_coef, float(c.vf_coef), st.rewards, val, st.dones, T, 1,
                     bool(c.norm_adv), float(c.gamma), float(c.gae_lambda), tr._ret_w, tr._adv_w, lb.h, eng.sWh, lb.dh,
                     eng.gWh, eng.gbh, eng.gbfc, sbuf, hp if boot else None, S, eng.bfc if boot else None,
                     eng.bh if boot else None, bar if boot else None, stamps)

    graphs = {"a2c_head_boot": make_graph(lambda: launch(), a.reps),
              "a2c_head_noboot": make_graph(lambda: launch(boot=False), a.reps)}
    res = {k: [] for k in graphs}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            res[k].append(time_graph(g, a.reps))
    out = {k: {"median_us": statistics.median(v), "min_us": min(v)} for k, v in res.items()}
    names = ["entry", "boot_loads_barrier", "returns_moments", "loss_dz", "head_bwd_lanes", "waves_store_issue",
             "drained"]
    for boot in (True, False):
        stamps = torch.zeros(32, 16, dtype=torch.int64, device="cuda:0")
        launch(stamps, boot)
        torch.cuda.synchronize()
        s = stamps.cpu().double() * 10e-3
        t0 = s[:, 0].min()
        ph = {"start_spread_us": float(s[:, 0].max() - t0)}
        for i in range(1, 7):
            ph[names[i]] = float((s[:, i] - s[:, i - 1]).median())
        ph["end_from_first_start_us"] = float(s[:, 6].max() - t0)
        ph["lead_end_us"] = float(s[0, 6] - t0)
        out["phases_boot" if boot else "phases_noboot"] = ph
    assert bar.tolist()[:3] == [0, 0, 0], bar
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
