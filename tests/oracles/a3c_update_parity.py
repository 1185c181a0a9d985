#!/usr/bin/env python3
"""One reference A3C update, this framework vs the independent oracle (tests/oracles/a3c_oracle.py), from the SAME
parameters on the SAME batch: targets, normalised advantages, post-update actor / critic parameters, KL proxy and
the adaptive lr. Prints the largest differences. CPU.

    python tests/oracles/a3c_update_parity.py [--updates 3]
"""
import argparse
import math
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

import a3c_oracle as O  # noqa: E402
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def load_oracle(m):
    a, c = O.Actor(3), O.Critic(3)
    with torch.no_grad():
        for dst, src in ((a.l1, m.actor.first_layer), (a.l2, m.actor.second_layer), (a.l3, m.actor.third_layer),
                         (a.mu, m.actor.mu_layer)):
            dst.weight.copy_(src.kernel.t())
            dst.bias.copy_(src.bias)
        a.log_std.copy_(m.actor.log_std)
        for k, src in zip((0, 2, 4, 6), (m.critic.first_layer, m.critic.second_layer, m.critic.third_layer,
                                          m.critic.value)):
            c.net[k].weight.copy_(src.kernel.t())
            c.net[k].bias.copy_(src.bias)
    return a, c


def flat_actor(a):
    return torch.cat([a.l1.weight.t().reshape(-1), a.l1.bias, a.l2.weight.t().reshape(-1), a.l2.bias,
                      a.l3.weight.t().reshape(-1), a.l3.bias, a.mu.weight.t().reshape(-1), a.mu.bias,
                      a.log_std]).detach()


def flat_ours(m):
    x = m.actor
    return torch.cat([x.first_layer.kernel.reshape(-1), x.first_layer.bias, x.second_layer.kernel.reshape(-1),
                      x.second_layer.bias, x.third_layer.kernel.reshape(-1), x.third_layer.bias,
                      x.mu_layer.kernel.reshape(-1), x.mu_layer.bias, x.log_std]).detach()


def flat_ours_grad(m):
    x = m.actor
    ps = [x.first_layer.kernel, x.first_layer.bias, x.second_layer.kernel, x.second_layer.bias, x.third_layer.kernel,
          x.third_layer.bias, x.mu_layer.kernel, x.mu_layer.bias, x.log_std]
    return torch.cat([p.grad.reshape(-1) if p.grad is not None else torch.full((p.numel(),), float("nan"))
                      for p in ps]).detach().clone()


def flat_oracle_grad(oa, grads):
    g = {n: x for (n, _), x in zip(oa.named_parameters(), grads)}
    return torch.cat([g["l1.weight"].t().reshape(-1), g["l1.bias"], g["l2.weight"].t().reshape(-1), g["l2.bias"],
                      g["l3.weight"].t().reshape(-1), g["l3.bias"], g["mu.weight"].t().reshape(-1), g["mu.bias"],
                      g["log_std"]]).detach()


def run(updates=3, num_envs=6, verbose=True, seed=5, schedule=True):
    """-> one dict per update: gradient relative error, max parameter difference, KL and lr (ours, oracle)."""
    rows = []
    log = print if verbose else (lambda *x, **k: None)
    cfg = preset("a3c", algo="a2c", num_envs=num_envs, n_steps=200, seed=seed, device="cpu", cuda_graph=False,
                 outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    # the oracle keeps its own Adam moments across updates, started in step with ours
    oa, oc = load_oracle(tr.model)
    aopt, copt = O.TFAdam(oa.parameters(), float(tr.actor_opt.get_lr())), O.TFAdam(oc.parameters(), cfg.critic_lr)
    g_ent, beta = float(tr.ent_coef), float(tr.kl_coef)
    for u in range(updates):
        with torch.no_grad():   # both start from OUR parameters each update (isolates one update's maths)
            oa2, oc2 = load_oracle(tr.model)
            oa.load_state_dict(oa2.state_dict())
            oc.load_state_dict(oc2.state_dict())
        tr.collect()
        st = tr.storage
        T, N = st.T, st.N
        obs = st.obs[:T + 1].reshape(T + 1, N, -1).float().clone()   # copies: roll_over rewrites obs[0]
        acs, lp_old = st.actions[:T].reshape(T, N, -1).clone(), st.logp[:T].reshape(T, N).clone()
        rews, dones = st.rewards[:T].reshape(T, N).clone(), st.dones[:T].reshape(T, N).clone()
        ret, adv = tr.compute_returns()
        # oracle targets on the same batch (episodes end exactly at the rollout end: terminal there)
        with torch.no_grad():
            vals = oc(obs.reshape(-1, 3)).reshape(T + 1, N)
        tgt, oadv = O.path_adv(rews, vals, cfg.gamma, cfg.look_ahead)
        log(f"update {u + 1}: dones at last step {int(dones[-1].sum())}/{N}, elsewhere {int(dones[:-1].sum())}; "
              f"max |ret - oracle target| {float((ret.reshape(T, N) - tgt).abs().max()):.3e}")
        g_before = g_ent, beta
        tr.learn(ret, adv)
        tr.storage.roll_over()
        # oracle update
        X, A, LP = obs[:T].reshape(-1, 3), acs.reshape(-1, 1), lp_old.reshape(-1)
        t_, ad = tgt.reshape(-1), oadv.reshape(-1)
        ad = (ad - ad.mean()) / (1e-8 + ad.std(unbiased=False))
        closs = ((oc(X) - t_) ** 2).mean()
        copt.step(torch.autograd.grad(closs, list(oc.parameters())))
        mu, ls, _ = oa(X)
        lp = (-0.5 * ((A - mu) / torch.exp(ls)) ** 2 - ls - 0.5 * math.log(2 * math.pi)).sum(1)
        ent = (0.5 + 0.5 * math.log(2 * math.pi) + ls).sum() * torch.ones_like(lp)
        loss = -(ad * lp).mean() + g_before[1] * ((LP - lp) ** 2).mean() - g_before[0] * ent.mean()
        log(f"  stored logp_old vs logp of the stored actions at the rollout parameters: max diff "
              f"{float((lp.detach() - LP).abs().max()):.3e}; |a| max {float(A.abs().max()):.3f}")
        raw = torch.autograd.grad(loss, list(oa.parameters()))
        grads = [torch.clamp(g, -0.1, 0.1) for g in raw]
        aopt.step(grads)
        with torch.no_grad():
            mu2, ls2, _ = oa(X)
            lp2 = (-0.5 * ((A - mu2) / torch.exp(ls2)) ** 2 - ls2 - 0.5 * math.log(2 * math.pi)).sum(1)
            kl = float(((LP - lp2) ** 2).mean())
        if kl < cfg.desired_kl / 4:
            aopt.lr = min(cfg.max_lr, aopt.lr * 1.5)
        elif kl > cfg.desired_kl * 4:
            aopt.lr = max(cfg.min_lr, aopt.lr / 1.5)
        go, gr = flat_ours_grad(tr.model), flat_oracle_grad(oa, raw)
        rel = float((go - gr).norm() / gr.norm())
        cos = float(torch.nn.functional.cosine_similarity(go, gr, dim=0))
        log(f"  actor gradient: rel err {rel:.3e}, cosine {cos:.6f}, |g| ours {float(go.norm()):.4e} oracle "
              f"{float(gr.norm()):.4e}; log_std grad ours {float(go[-1]):.5e} oracle {float(gr[-1]):.5e}; "
              f"mu bias grad ours {float(go[-2]):.5e} oracle {float(gr[-2]):.5e}")
        d = (flat_ours(tr.model) - flat_actor(oa)).abs()
        log(f"  actor params max |ours - oracle| {float(d.max()):.3e} (step size ~{aopt.lr:.1e}); "
              f"log_std ours {float(tr.model.actor.log_std.detach()):.5f} oracle {float(oa.log_std.detach()):.5f}; "
              f"kl ours {float(tr.stats['kl']):.6f} oracle {kl:.6f}; lr ours {float(tr.actor_opt.get_lr()):.6f} "
              f"oracle {aopt.lr:.6f}; clipped grad elems {sum(int((g.abs() > 0.1).sum()) for g in raw)}")
        rows.append(dict(grad_rel=rel, param_max=float(d.max()), kl=(float(tr.stats["kl"]), kl),
                         lr=(float(tr.actor_opt.get_lr()), aopt.lr), logp_consistency=float((lp.detach() - LP).abs().max()),
                         target_max=float((ret.reshape(T, N) - tgt).abs().max())))
        if schedule and tr.reg_sched is not None:   # what step() does after the update (Basic_AC/run_AC.py:268-275)
            e, k = tr.reg_sched.entropy_coef(tr.iteration), tr.reg_sched.kl_coef(tr.iteration)
            if e is not None:
                tr.ent_coef.fill_(e)
            if k is not None:
                tr.kl_coef.fill_(k)
        tr.iteration += 1
        g_ent, beta = float(tr.ent_coef), float(tr.kl_coef)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=3)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--no-schedule", action="store_true")
    a = ap.parse_args()
    torch.set_num_threads(4)
    run(a.updates, seed=a.seed, schedule=not a.no_schedule)


if __name__ == "__main__":
    main()
