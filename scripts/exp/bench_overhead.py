"""Fixed per-window overhead of the headline bench: time K = 1, 2, 5, 20, 100, 400 captured updates with the
bench's bracketing (synchronize, timed loop, synchronize), the host time of one step() call, and the graph launch
alone. GPU only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def main():
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0))
    tr.capture(warmup=2)
    for _ in range(30):
        tr.step()
    torch.cuda.synchronize()
    out = {}
    for K in (1, 2, 5, 20, 100, 400, 20, 5, 1):
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(K):
                tr.step()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6)
        out[f"K{K}"] = round(min(ts), 1)
    # host cost of step() (the GPU queue is long: measured while it drains)
    torch.cuda.synchronize()
    for _ in range(50):
        tr.step()
    t0 = time.perf_counter()
    for _ in range(50):
        tr.step()
    out["host_us_per_step_queued"] = round((time.perf_counter() - t0) * 1e6 / 50, 1)
    torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
