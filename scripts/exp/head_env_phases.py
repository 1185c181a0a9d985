"""Phase stamps of the per-env A2C head (loss.hip a2c_head_env_kernel) on the headline's buffers, launched right after
the bootstrap observation's fc product (as in the captured update): slots 0 entry, 1 planes + V(s_T) + barrier,
2 returns / loss / dz + barrier, 3 head backward loop, 4 stores drained. Also the graph-chained time of
[fc_rollout ; a2c_head_env] against [fc_rollout] alone. GPU only. python scripts/exp/head_env_phases.py"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def main():
    ops = _native.require()
    cfg = preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=2)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    eng, st = tr.engine, tr.storage
    N, T = tr.env.num_envs, st.T
    lb = eng.bufs(N * T, with_grad=True)
    bt = eng.bufs(N)
    eng.forward(st.obs[T], bt, head=False, fc_parts=True)
    hp, S = eng.last_fc
    ae = eng._ae[N]
    acts, lpo = st.flat("actions"), st.flat("logp")
    val = st.values.clone()

    def head(stamps=None):
        ops.a2c_head_env(lb.z, acts, lpo, tr.ent_coef, tr.kl_coef, float(cfg.vf_coef), st.rewards, val, st.dones,
                         T, 1, float(cfg.gamma), float(cfg.gae_lambda), tr._ret_w, tr._adv_w, lb.h, eng.sWh, lb.dh,
                         hp, S, eng.bfc, eng.bh, ae["Wh"], ae["bfc"], ae["bh"], ae["st"], stamps)

    fc = lambda: eng.fc_planes(bt)   # noqa: E731
    out = {}
    for name, fn in (("fc_then_head", lambda: (fc(), head())), ("fc_only", fc), ("head_only", head)):
        g = make_graph(fn, 100)
        out[name + "_us"] = round(min(time_graph(g, 100) for _ in range(5)), 2)
        del g
    names = ["entry", "planes_V_barrier", "returns_loss_dz_barrier", "backward_loop", "stores_drained"]
    ph = []
    for _ in range(20):
        stamps = torch.zeros(N, 16, dtype=torch.int64, device="cuda:0")
        fc()
        head(stamps)
        torch.cuda.synchronize()
        s = stamps.cpu().double() / 100.0
        t0 = float(s[:, 0].min())
        d = {"start_spread_us": float(s[:, 0].max()) - t0}
        for i in range(1, 5):
            d[names[i]] = float((s[:, i] - s[:, i - 1]).median())
        d["end_from_first_start_us"] = float(s[:, 4].max()) - t0
        ph.append(d)
    out["phases_median"] = {k: round(statistics.median(x[k] for x in ph), 3) for k in ph[0]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
