"""Breakout-shape PPO learning curves on the native engine (default EngineOpts) and the torch/autograd engine
(fraction of points won per report window), plus the native-vs-autograd gradient errors at the production batches
(per parameter relative norm) that set the bar of tests/test_gpu_learning.py. GPU only.
python scripts/exp/r5_learn_breakout.py [--updates 300] [--report 25] [--seeds 1,2]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def curve(engine, updates, report, seed):
    tr = ActorCriticTrainer(preset("breakout_ppo", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, seed=seed, engine=engine))
    if tr.cfg.cuda_graph:
        tr.capture(warmup=1)
    won = torch.zeros((), device=tr.device)
    lost = torch.zeros((), device=tr.device)
    rows = []
    for u in range(1, updates + 1):
        tr.step()
        r = tr.storage.rewards
        won += (r > 0).sum()
        lost += (r < 0).sum()
        if u % report == 0:
            w, l = float(won), float(lost)
            rows.append(round(w / max(w + l, 1.0), 4))
            won.zero_()
            lost.zero_()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--updates", type=int, default=300)
    ap.add_argument("--report", type=int, default=25)
    ap.add_argument("--seeds", default="1,2")
    ap.add_argument("--engines", default="native,torch")
    a = ap.parse_args()
    for eng in a.engines.split(","):
        for seed in [int(s) for s in a.seeds.split(",")]:
            rows = curve(eng, a.updates if eng == "native" else min(a.updates, 200), a.report, seed)
            print(json.dumps({"engine": eng, "seed": seed, "report_every": a.report, "win": rows}), flush=True)


if __name__ == "__main__":
    main()
