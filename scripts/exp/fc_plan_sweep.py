"""In-pipeline sweep of the rollout fc GEMM plan (y3 [B, 3136] x Wfc -> split-K planes): the plans file holds the
winner of an isolated back-to-back timing; here every candidate (tile, BK, splits) runs inside the captured update
of the config (pong_a2c: B = 32; breakout_ppo: B = 128) and the update time decides. GPU only.
python scripts/exp/fc_plan_sweep.py [--config pong_a2c] [--updates 200]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="pong_a2c")
    ap.add_argument("--updates", type=int, default=200)
    a = ap.parse_args()
    B = {"pong_a2c": 32, "breakout_ppo": 128}[a.config]
    key = (B, 512, 3136, True, False, 3, True, True, (), (), 32)
    base = G._TUNED.get(key)
    cands = list(G._candidates(B, 512, 3136, True, 32))
    out = {"config": a.config, "plans_file": base, "results": []}
    for tile, bk, s in cands:
        G._TUNED[key] = (tile, bk, s, 0.0)
        tr = ActorCriticTrainer(preset(a.config, device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                       save_every=0, seed=1))
        tr.capture(warmup=2)
        n = a.updates if a.config == "pong_a2c" else max(3, a.updates // 40)
        for _ in range(max(2, n // 10)):
            tr.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            tr.step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / n
        out["results"].append({"tile": tile, "bm_bn": G.TILES[tile], "bk": bk, "splits": s,
                               "eff_splits": G.effective_splits(3136, bk, s), "ms_per_update": round(ms, 4)})
        print(json.dumps(out["results"][-1]), flush=True)
        del tr
    out["results"].sort(key=lambda r: r["ms_per_update"])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
