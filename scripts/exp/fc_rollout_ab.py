"""Rollout fc product on the fragment-ordered Wfc (fc_rollout.hip): (1) every variant's planes vs an fp32 PyTorch
product of the same bf16 operands; (2) the captured pong_a2c update with each variant vs the general GEMM
(EngineOpts.fc_frag = -1), interleaved rounds so box drift hits every arm alike. GPU only.
python scripts/exp/fc_rollout_ab.py [--updates 400] [--rounds 3] [--variants -1,0,1,2,3,4,5,6]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order_kc  # noqa: E402


def check(variants):
    ops = _native.require()
    g = torch.Generator(device="cuda").manual_seed(0)
    out = {}
    for M in (32, 7):
        X = (torch.randn(M, 3136, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
        W = (torch.randn(3136, 512, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        Wf = frag_order_kc(W.float(), 3136, 512)
        ref = X.double() @ W.double()
        for v in variants:
            if v < 0:
                continue
            hp = torch.full((32 * M * 512,), float("nan"), device="cuda")
            S = ops.fc_rollout(X, Wf, hp, v)
            got = hp.view(32, M, 512)[:S].double().sum(0)
            err = float((got - ref).abs().max() / ref.abs().max())
            out[f"M{M}_v{v}"] = {"planes": S, "rel_err": err}
            assert err < 1e-5, (M, v, err)
    return out


def time_update(v, updates):
    cfg = preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0, seed=1,
                 engine_opts={"fc_frag": v})
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=2)
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(updates):
        tr.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / updates
    del tr
    return ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=400)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="-1,0,1,2,3,4,5,6")
    a = ap.parse_args()
    vs = [int(x) for x in a.variants.split(",")]
    print(json.dumps({"numerics": check(vs)}), flush=True)
    res = {v: [] for v in vs}
    for r in range(a.rounds):
        for v in vs:
            res[v].append(round(time_update(v, a.updates), 4))
            print(json.dumps({"round": r, "variant": v, "ms_per_update": res[v][-1]}), flush=True)
    print(json.dumps({"summary": {str(v): min(t) for v, t in res.items()}}))


if __name__ == "__main__":
    main()
