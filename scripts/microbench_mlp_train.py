"""Phase timings of the fused MLP train kernel (mlp_fwd_kernel mode 2) from its s_memrealtime stamps (100 MHz),
MuJoCo-shape PPO minibatch (512 rows, both towers): per tower, the end of the row gather, of the input tile, of each
forward layer, of the loss head, of each data-gradient layer; plus CUDA-event times of a whole PPO minibatch step
(train + weight gradient + optimiser) and of each launch alone."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def ev_time(fn, n=50):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / n, 2)


def main():
    cfg = preset("mujoco_ppo_dp8", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                 cuda_graph=False)
    tr = ActorCriticTrainer(cfg)
    tr.step()
    eng, st = tr.mlp, tr.storage
    obs, actions, logp_old = st.flat("obs"), st.flat("actions"), st.flat("logp")
    v_old = st.flat("values")
    B = obs.shape[0]
    mb = B // cfg.ppo_minibatches
    adv = torch.randn(B, device="cuda:0")
    ret = torch.randn(B, device="cuda:0")
    uc = tr.update_counter.view(1)
    stamps = torch.zeros(2, 16, dtype=torch.int64, device="cuda:0")
    kw = dict(v_old=v_old, vf_coef=1.0, ppo=True, ppo_clip=cfg.ppo_clip, v_clip=0.0, stats=tr.stats_buf,
              clips=(cfg.clip_value, cfg.critic_clip_value))
    out = {"B_minibatch": mb}
    names = {1: "gather", 2: "x0", 3: "fwd0", 4: "fwd1", 5: "fwd2", 6: "fwd3", 8: "head", 14: "headC",
             9: "dg_top", 10: "dg_2", 11: "dg_3", 7: "end", 15: "headA"}
    res = {0: [], 1: []}
    for rep in range(20):
        stamps.zero_()
        # contiguous minibatch rows (the trainer's epoch-gathered layout)
        eng.train(obs[:mb], actions[:mb], logp_old[:mb], adv[:mb], ret[:mb], tr.ent_coef, tr.kl_coef, mb,
                  stamps=stamps, **dict(kw, v_old=v_old[:mb]))
        torch.cuda.synchronize()
        s = stamps.cpu().tolist()
        for t in (0, 1):
            res[t].append(s[t])
    for t in (0, 1):
        ph = {}
        for slot, name in names.items():
            vals = [(r[slot] - r[0]) * 0.01 for r in res[t][2:] if r[slot] > 0]
            if vals:
                ph[name] = round(sorted(vals)[len(vals) // 2], 2)
        out[f"tower{t}_us_from_start"] = dict(sorted(ph.items(), key=lambda kv: kv[1]))
        last = max(k for k in (9, 10, 11) if res[t][-1][k] > 0)
        ghz = [(r[13] - r[12]) / ((r[last] - r[2]) * 10.0) for r in res[t][2:] if r[last] > r[2]]
        out[f"tower{t}_shader_clock_ghz"] = round(sorted(ghz)[len(ghz) // 2], 3) if ghz else None
    out["train_launch_us"] = ev_time(lambda: eng._fwd(2, obs, mb, 0, 2, desc_B=mb, perm=(uc, 0, 0, B, tr.policy_seed),
                                                      act_in=actions, logp_old=logp_old, adv=adv, ret=ret,
                                                      v_old=v_old, ent_coef=tr.ent_coef, kl_coef=tr.kl_coef,
                                                      ppo=True, ppo_clip=cfg.ppo_clip))
    out["train_plus_wgrad_us"] = ev_time(lambda: eng.train(obs, actions, logp_old, adv, ret, tr.ent_coef, tr.kl_coef, mb,
                                                           perm=(uc, 0, 0, B, tr.policy_seed), **kw))
    out["minibatch_step_us"] = ev_time(lambda: tr._mlp_step(eng, mb, None, obs, actions, logp_old, adv, ret, v_old,
                                                            perm=(uc, 0, 0, B, tr.policy_seed)))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
