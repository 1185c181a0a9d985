"""Headline optimiser A/B: pong_a2c parameters (fp32 masters, bf16 shadow, fragment-ordered conv copies) after 6
graph-replayed updates, saved (--save) or compared bit for bit (--ref) across builds / unroll settings, and the
update time with each optimiser unroll (1, 2, 4 float4 groups per thread). GPU only."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def run(updates=6, time_updates=0):
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                                   seed=3))
    tr.capture(warmup=1)
    for _ in range(updates):
        tr.step()
    torch.cuda.synchronize()
    out = {"p": tr.flat.data.cpu().clone(), "shadow": tr.shadow.cpu().clone(),
           "frag": [f.cpu().clone() for f in tr.engine.frag], "stats": tr.stats_buf.cpu().clone()}
    ms = None
    if time_updates:
        t0 = time.perf_counter()
        for _ in range(time_updates):
            tr.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / time_updates
    return out, ms


def same(a, b):
    if isinstance(a, list):
        return all(torch.equal(x, y) for x, y in zip(a, b))
    return torch.equal(a, b)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--save")
    ap.add_argument("--ref")
    ap.add_argument("--unrolls", default="1")
    ap.add_argument("--time", type=int, default=0)
    a = ap.parse_args()
    ops = _native.require()
    for u in [int(x) for x in a.unrolls.split(",")]:
        if hasattr(ops, "opt_set_unroll"):
            ops.opt_set_unroll(u)
        out, ms = run(time_updates=a.time)
        if a.save:
            torch.save(out, a.save)
        res = {"unroll": u, "ms_per_update": ms}
        if a.ref:
            ref = torch.load(a.ref)
            res["bitwise"] = {k: same(out[k], ref[k]) for k in out}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
