"""Repeats the MLP train launch (SPEC path and the generic layer loop) on fixed inputs and reports any run whose
gradients differ from the first run of the same path (nondeterminism = a race) and the SPEC-vs-generic gap."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_mlp as T  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import distributions as D  # noqa: E402

cuda = torch.device("cuda:0")
for case in [(17, 6, False, "basic"), (4, 2, True, "basic")]:
    ob, ac, disc, variant = case
    m, ref, flat, eng = T._model(cuda, ob, ac, disc, variant, seed=3)
    Bfull, B = 300, 200
    obs = torch.randn(Bfull, ob, device=cuda)
    with torch.no_grad():
        pi, v0 = ref(obs)
        keys = torch.arange(Bfull, device=cuda, dtype=torch.int64)
        act, lp0, _ = (D.categorical_sample_ref(pi, keys, 7) if disc else D.gaussian_sample_ref(pi, ref.actor.log_std, keys, 7))
    lo = lp0 + 0.3 * torch.randn(Bfull, device=cuda)
    adv = torch.randn(Bfull, device=cuda)
    ret = v0 + torch.randn(Bfull, device=cuda)
    v_old = v0 + 0.1 * torch.randn(Bfull, device=cuda)
    idx = torch.randperm(Bfull, device=cuda)[:B]
    beta, ce = torch.tensor(0.7, device=cuda), torch.tensor(0.05, device=cuda)
    for ppo in (False, True):
        res = {}
        for spec in (True, False):
            eng.spec = spec
            first = None
            bad = 0
            for it in range(40):
                flat.grad.zero_()
                stats = torch.zeros(16, device=cuda)
                eng.train(obs, act, lo, adv, ret, ce, beta, B, idx=idx, v_old=v_old, ppo=ppo, ppo_clip=0.2,
                          v_clip=0.15 if ppo else 0.0, stats=stats, clips=(None, None), want_parts=True)
                torch.cuda.synchronize()
                g = flat.grad.clone()
                if first is None:
                    first = g
                elif not torch.equal(g, first):
                    bad += 1
                    d = (g - first).abs()
                    i = int(d.argmax())
                    names = [(n, p) for n, p in m.named_parameters()]
                    off = 0
                    where = "?"
                    for n, p in names:
                        o = flat.offsets[[id(x) for x in flat.params].index(id(p))]
                        if o <= i < o + p.numel():
                            where = f"{n}[{i - o}]"
                    if bad <= 3:
                        print(f"case {case} ppo {ppo} spec {spec} run {it}: max diff {float(d.max()):.3e} at {where}",
                              flush=True)
            res[spec] = first
            print(f"case {case} ppo {ppo} spec {spec}: {bad} / 39 runs differ from run 0", flush=True)
        print("  spec vs generic max rel:", float((res[True] - res[False]).abs().max() / res[False].abs().max()))
