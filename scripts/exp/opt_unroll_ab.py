"""Headline update time vs the single-segment optimiser's float4 groups per thread (aca_opt_set_unroll 1 / 2 / 4),
each captured fresh, A/B/A order; 200 timed replays after 20 warm-up."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402


def run(u):
    _native.require().opt_set_unroll(u)
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0))
    tr.capture(warmup=2)
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        tr.step()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) / 200 * 1e3, 2)


out = {}
for u in (1, 2, 4, 1):
    out.setdefault(f"U{u}", []).append(run(u))
print(json.dumps(out))
