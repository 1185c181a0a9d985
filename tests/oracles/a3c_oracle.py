#!/usr/bin/env python3
"""Independent plain-PyTorch oracle of ONE reference A3C worker (``A3C/process.py:156-285``, ``A3C/policies.py``):
no code from this package, so its trajectory tells whether a divergence is in the reference's update itself or in
this framework's implementation of it.

Per iteration: 6 whole 200-step Pendulum-v0 episodes (EP_LENGTH_STOP = 1200) with a ``--frames``-deep Framer
(``process.py:14-43``; CLI default 1, ``train.py:22``), PathAdv targets (gamma 0.98, L 40, no bootstrap at the time-limit terminal), global
advantage normalisation, ONE critic Adam step (MSE, lr 1e-3) and ONE actor Adam step (lr 5e-3 initial, gradients
clipped by value to +-0.1; loss = -mean(adv logp) + beta mean((logp_old - logp)^2) - gamma mean(entropy)), then the
KL-adaptive lr in [1e-6, 0.1] and the log10 gamma / beta schedules (``process.py:173-174,265-278``). TF1 Adam
(eps 1e-8 outside the bias correction). ``--separate-local-init``: the first rollout uses a second random init as
the reference's unsynced local actor does (``process.py:205-207``).

    python tests/oracles/a3c_oracle.py --updates 300 --desired-kl 2e-3 [--seed 0]
"""
import argparse
import json
import math

import torch
import torch.nn as nn


def glorot(lin):
    nn.init.xavier_uniform_(lin.weight)
    nn.init.zeros_(lin.bias)
    return lin


class Actor(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.l1, self.l2, self.l3 = glorot(nn.Linear(d, 128)), glorot(nn.Linear(128, 128)), glorot(nn.Linear(128, 64))
        self.mu = glorot(nn.Linear(64, 1))
        self.log_std = nn.Parameter(torch.zeros(1))

    def forward(self, x):
        a = lambda t: 0.8 * torch.relu(t) + 0.2 * t   # lrelu(0.2) as policies.py:9
        h = a(self.l3(a(self.l2(a(self.l1(x))))))
        pre = self.mu(h)
        return torch.tanh(pre) * 2.0, torch.clamp(self.log_std, -2.5, 2.5), pre


class Critic(nn.Module):
    def __init__(self, d):
        super().__init__()
        self.net = nn.Sequential(glorot(nn.Linear(d, 256)), nn.ReLU(), glorot(nn.Linear(256, 128)), nn.ReLU(),
                                 glorot(nn.Linear(128, 128)), nn.ReLU(), glorot(nn.Linear(128, 1)))

    def forward(self, x):
        return self.net(x).reshape(-1)


class TFAdam:
    def __init__(self, params, lr):
        self.p = list(params)
        self.lr = lr
        self.m = [torch.zeros_like(q) for q in self.p]
        self.v = [torch.zeros_like(q) for q in self.p]
        self.t = 0

    @torch.no_grad()
    def step(self, grads):
        self.t += 1
        lr_t = self.lr * math.sqrt(1 - 0.999 ** self.t) / (1 - 0.9 ** self.t)
        for q, g, m, v in zip(self.p, grads, self.m, self.v):
            m.mul_(0.9).add_(g, alpha=0.1)
            v.mul_(0.999).addcmul_(g, g, value=0.001)
            q.sub_(lr_t * m / (v.sqrt() + 1e-8))


def pendulum_rollout(actor, n, T, gen, F=1):
    th = (torch.rand(n, generator=gen) * 2 - 1) * math.pi
    thd = (torch.rand(n, generator=gen) * 2 - 1)
    ob = lambda: torch.stack([torch.cos(th), torch.sin(th), thd], 1)
    frames = [ob()] * F
    obs, acs, logps, rews = [], [], [], []
    with torch.no_grad():
        for _ in range(T):
            x = torch.cat(frames[-F:], 1)
            mu, ls, _ = actor(x)
            a = mu + torch.exp(ls) * torch.randn(n, 1, generator=gen)
            lp = (-0.5 * ((a - mu) / torch.exp(ls)) ** 2 - ls - 0.5 * math.log(2 * math.pi)).sum(1)
            u = torch.clamp(a[:, 0], -2.0, 2.0)
            an = ((th + math.pi) % (2 * math.pi)) - math.pi
            rews.append(-(an ** 2 + 0.1 * thd ** 2 + 0.001 * u ** 2))
            thd = torch.clamp(thd + (-3 * 10.0 / 2 * torch.sin(th + math.pi) + 3.0 * u) * 0.05, -8.0, 8.0)
            th = th + thd * 0.05
            obs.append(x)
            acs.append(a)
            logps.append(lp)
            frames.append(ob())
        obs.append(torch.cat(frames[-F:], 1))   # the final observation (valued, never acted on)
    return torch.stack(obs), torch.stack(acs), torch.stack(logps), torch.stack(rews)


def path_adv(rews, vals, gamma=0.98, L=40):
    """PathAdv (process.py:46-66) for whole episodes (terminal at the end): rews [T, n], vals [T + 1, n]."""
    T = rews.shape[0]
    tgt = torch.zeros_like(rews)
    for i in range(T):
        h = min(i + L, T)
        disc = gamma ** torch.arange(h - i, dtype=rews.dtype)
        tgt[i] = (disc[:, None] * rews[i:h]).sum(0)
        if h != T:
            tgt[i] += gamma ** (h - i) * vals[h]
    return tgt, tgt - vals[:T]


def sched(i, a, b, init_t=100, end_t=3000):
    if i < init_t:
        return a
    if i > end_t:
        return b
    return a + (b - a) * (i - init_t) / (end_t - init_t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=300)
    ap.add_argument("--desired-kl", type=float, default=2e-3)
    ap.add_argument("--max-lr", type=float, default=0.1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--separate-local-init", action="store_true")
    ap.add_argument("--report", type=int, default=10)
    ap.add_argument("--frames", type=int, default=1, help="Framer depth (reference CLI default 1: the demo's 3-input actor)")
    a = ap.parse_args()
    torch.set_num_threads(2)
    torch.manual_seed(a.seed)
    gen = torch.Generator().manual_seed(a.seed + 1)
    D = 3 * a.frames
    actor, critic = Actor(D), Critic(D)
    local = Actor(D) if a.separate_local_init else actor
    aopt, copt = TFAdam(actor.parameters(), 5e-3), TFAdam(critic.parameters(), 1e-3)
    g_ent, beta = 0.01, 1.0
    for i in range(a.updates):
        obs, acs, logp_old, rews = pendulum_rollout(local, 6, 200, gen, a.frames)
        with torch.no_grad():
            vals = critic(obs.reshape(-1, D)).reshape(201, 6)
        tgt, adv = path_adv(rews, vals)
        X, A, LP = obs[:200].reshape(-1, D), acs.reshape(-1, 1), logp_old.reshape(-1)
        tgt, adv = tgt.reshape(-1), adv.reshape(-1)
        adv = (adv - adv.mean()) / (1e-8 + adv.std(unbiased=False))
        closs = ((critic(X) - tgt) ** 2).mean()
        copt.step(torch.autograd.grad(closs, list(critic.parameters())))
        src = local   # gradients at the local (rollout) parameters, applied to the global ones (process.py:84-89)
        mu, ls, pre = src(X)
        std = torch.exp(ls)
        lp = (-0.5 * ((A - mu) / std) ** 2 - ls - 0.5 * math.log(2 * math.pi)).sum(1)
        ent = (0.5 + 0.5 * math.log(2 * math.pi) + ls).sum() * torch.ones_like(lp)
        loss = -(adv * lp).mean() + beta * ((LP - lp) ** 2).mean() - g_ent * ent.mean()
        grads = [torch.clamp(g, -0.1, 0.1) for g in torch.autograd.grad(loss, list(src.parameters()))]
        aopt.step(grads)
        if local is not actor:
            local.load_state_dict(actor.state_dict())
        with torch.no_grad():
            mu2, ls2, pre2 = actor(X)
            lp2 = (-0.5 * ((A - mu2) / torch.exp(ls2)) ** 2 - ls2 - 0.5 * math.log(2 * math.pi)).sum(1)
            kl = float(((LP - lp2) ** 2).mean())
        if kl < a.desired_kl / 4:
            aopt.lr = min(a.max_lr, aopt.lr * 1.5)
        elif kl > a.desired_kl * 4:
            aopt.lr = max(1e-6, aopt.lr / 1.5)
        if i % 100 == 0:
            g_ent, beta = 10.0 ** sched(i, -2, -8), 10.0 ** sched(i, 0, -4)
        if i % a.report == 0 or i == a.updates - 1:
            print(json.dumps({"update": i + 1, "ret": round(float(rews.sum(0).mean()), 1), "lr": aopt.lr,
                              "kl": round(kl, 6), "log_std": round(float(actor.log_std.detach()), 4),
                              "mu_sat": round(float((pre2.abs() > 2).float().mean()), 4),
                              "pre_tanh": round(float(pre2.abs().mean()), 3)}), flush=True)


if __name__ == "__main__":
    main()
