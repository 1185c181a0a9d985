"""Micro-benchmark of the conv2 data-gradient GEMM (sub-pixel transposed conv, gather modes 5/6) at the A2C
(B=160) and PPO-minibatch (B=4096) batch sizes: with / without the fused bias column sums, per tile."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    _native.require()
    dev = torch.device("cuda:0")
    ws = G.GemmWorkspace(dev)
    out = {}
    for B in (160, 4096):
        dy2 = (torch.randn(B * 81, 64, device=dev) * 0.1).to(torch.bfloat16)
        W2 = (torch.randn(64 * 16 * 32, device=dev) * 0.1).to(torch.bfloat16)
        y1 = torch.randn(B * 400, 32, device=dev).to(torch.bfloat16)
        dy1 = torch.empty(B * 400, 32, device=dev, dtype=torch.bfloat16)
        gb1 = torch.zeros(32, device=dev)
        for cs in (True, False):
            for tile in (2, 0, 3):
                def run():
                    G.gemm(dy2, 0, True, W2, 0, False, dy1, 32, 1, B * 400, 32, 256, mask=y1, ldm=32,
                           colsum=gb1 if cs else None, workspace=ws, ga=[5, B, 64, 20, 20, 4, 4, 2],
                           gb=[6, 1, 64, 1, 32, 4, 4, 2], tile=tile, splits=1, bk=64)
                try:
                    out[f"B{B}_colsum{int(cs)}_tile{tile}"] = round(timeit(run), 2)
                except Exception as e:  # unsupported tile for this gather
                    out[f"B{B}_colsum{int(cs)}_tile{tile}"] = str(e)[:60]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
