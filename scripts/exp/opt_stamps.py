"""Per-workgroup phase stamps (s_memrealtime, 10 ns ticks) of the MuJoCo-shape multi-group Adam launch, right after a
train + weight-gradient pair (the in-graph data state): start, element loads issued, global norm reduced, element
loop done, block items done, stores landed. Prints the median / max of each phase over the workgroups and the last
finishers."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def main():
    cfg = preset("mujoco_ppo_dp8", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                 cuda_graph=False)
    tr = ActorCriticTrainer(cfg)
    tr.step()
    torch.cuda.synchronize()
    eng, st = tr.mlp, tr.storage
    obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
    v_old = st.flat("values")
    B = obs.shape[0]
    mb = B // cfg.ppo_minibatches
    adv = torch.randn(B, device="cuda:0")
    ret = torch.randn(B, device="cuda:0")
    perm = (tr.update_counter.view(1), 0, 0, B, tr.policy_seed)
    kw = dict(v_old=v_old, vf_coef=1.0, ppo=True, ppo_clip=cfg.ppo_clip, v_clip=0.0, stats=tr.stats_buf,
              clips=(cfg.clip_value, cfg.critic_clip_value))
    gs = tr._group_step
    for t, g in enumerate(("actor", "critic")):
        tr.opts[g].ext_parts = eng.parts[t]
    buf = torch.zeros(512, 8, dtype=torch.int64, device="cuda:0")
    out = {}
    for mode in (0, 4, 8):
        _native.require().opt_set_unroll(100 + mode)
        rows = []
        for rep in range(12):
            eng.train(obs, actions, logp_old, adv, ret, tr.ent_coef, tr.kl_coef, mb, perm=perm, **kw)
            buf.zero_()
            _native.require().opt_set_stamps(buf)
            gs.step(t_off=0)
            _native.require().opt_set_stamps(None)
            torch.cuda.synchronize()
            b = buf.cpu()
            b = b[b[:, 0] > 0]
            t0 = int(b[:, 0].min())
            rows.append((b - t0).tolist())
        # median over reps of per-phase max / median across workgroups
        ph = {}
        for k, name in enumerate(("start", "issued", "norm", "elem", "blocks", "landed")):
            mx = sorted(max(r[k] for r in rep) for rep in rows[2:])
            md = sorted(sorted(r[k] for r in rep)[len(rep) // 2] for rep in rows[2:])
            ph[name] = {"max_us": mx[len(mx) // 2] / 100, "med_us": md[len(md) // 2] / 100}
        last = rows[-1]
        order = sorted(range(len(last)), key=lambda i: -last[i][5])[:5]
        ph["last_wgs"] = [(i, [x / 100 for x in last[i][:6]]) for i in order]
        ph["n_wg"] = len(last)
        out[f"mode{mode}"] = ph
    _native.require().opt_set_unroll(100)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
