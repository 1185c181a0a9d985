"""MuJoCo-shape PPO minibatch step, per launch: each of the three learner launches (fused train, weight gradient,
multi-group Adam) replayed alone and in sequence from captured graphs of 50 minibatch steps, plus optimiser
variants (no fragment copies, no global-norm partials). Prints one JSON object (us per launch)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def graph_us(fn, n=50, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return round(best, 2)


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
    uc = tr.update_counter.view(1)
    perm = (uc, 0, 0, B, tr.policy_seed)
    kw = dict(v_old=v_old, vf_coef=1.0, ppo=True, ppo_clip=cfg.ppo_clip, v_clip=0.0, stats=tr.stats_buf,
              clips=(cfg.clip_value, cfg.critic_clip_value))

    def train():
        eng._fwd(2, obs, mb, 0, 2, desc_B=mb, perm=perm, act_in=actions, logp_old=logp_old, adv=adv, ret=ret,
                 v_old=v_old, ent_coef=tr.ent_coef, kl_coef=tr.kl_coef, ppo=True, ppo_clip=cfg.ppo_clip)

    def train_wgrad():
        eng.train(obs, actions, logp_old, adv, ret, tr.ent_coef, tr.kl_coef, mb, perm=perm, **kw)

    gs = tr._group_step
    for t, g in enumerate(("actor", "critic")):
        tr.opts[g].ext_parts = eng.parts[t]

    def opt():
        gs.step(t_off=0)

    def step():
        tr._mlp_step(eng, mb, None, obs, actions, logp_old, adv, ret, v_old, perm=perm)

    out = {"B_minibatch": mb}
    out["train"] = graph_us(train)
    out["train+wgrad"] = graph_us(train_wgrad)
    out["opt"] = graph_us(opt)
    tr._t_off = 0
    out["step"] = graph_us(step)
    items = gs._items
    gs._items = [None, None]
    gs._key = None
    out["opt_no_frag_copies"] = graph_us(opt)
    gs._items = items
    gs._key = None
    parts = [tr.opts[g].ext_parts for g in ("actor", "critic")]
    for g in ("actor", "critic"):
        tr.opts[g].ext_parts = None
        tr.opts[g].max_grad_norm_saved = tr.opts[g].max_grad_norm
        tr.opts[g].max_grad_norm = None
    gs._key = None
    out["opt_no_norm"] = graph_us(opt)
    for t, g in enumerate(("actor", "critic")):
        tr.opts[g].max_grad_norm = tr.opts[g].max_grad_norm_saved
        tr.opts[g].ext_parts = parts[t]
    gs._key = None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
