"""Tune every GEMM shape the BASELINE configs issue on this GPU and write ops/gemm_plans.json (the measured plans
the package loads at import). Usage (GPU box): python scripts/dump_gemm_plans.py [--configs pong_a2c,breakout_ppo]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ACAMD_GEMM_PLANS"] = "0"   # measure afresh
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pong_a2c,breakout_ppo")
    ap.add_argument("--rounds", type=int, default=3, help="tune each shape this many times, keep the fastest plan")
    ap.add_argument("--out", default=None, help="write here instead of the package's plans file")
    ap.add_argument("--keep-existing", action="store_true",
                    help="shapes already in the package's plans file keep their plan (only new shapes are added)")
    a = ap.parse_args()
    best = {}
    for _ in range(a.rounds):
        G._TUNED.clear()
        for name in a.configs.split(","):
            tr = ActorCriticTrainer(preset(name, device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                           save_every=0, cuda_graph=False))
            for _ in range(2):
                tr.step()
            torch.cuda.synchronize()
            del tr
        for k, v in G._TUNED.items():
            if k not in best or v[3] < best[k][3]:
                best[k] = v
    G._TUNED.clear()
    G._TUNED.update(best)
    if a.keep_existing:
        import json
        with open(G.PLANS_FILE) as f:
            for r in json.load(f):
                G._TUNED[G._key_from_json(r["key"])] = tuple(r["plan"])
    out = a.out or G.PLANS_FILE
    n = G.save_plans(out)
    print("wrote", n, "plans to", out)


if __name__ == "__main__":
    main()
