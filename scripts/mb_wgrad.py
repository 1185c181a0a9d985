"""Isolated timing of the per-sample conv weight-gradient kernels (conv_wgrad.hip) vs the implicit-GEMM path."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000.0


def main():
    ops = _native.require()
    dev = torch.device("cuda:0")
    out = {}
    for B in (160, 4096):
        obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, device=dev)
        dy1 = torch.randn(B * 400, 32, device=dev).to(torch.bfloat16)
        y1 = torch.rand(B * 400, 32, device=dev).to(torch.bfloat16)
        dy2 = torch.randn(B * 81, 64, device=dev).to(torch.bfloat16)
        y2 = torch.rand(B * 81, 64, device=dev).to(torch.bfloat16)
        dy3 = torch.randn(B * 49, 64, device=dev).to(torch.bfloat16)
        pl = torch.zeros(256 * 64 * 576, device=dev)
        for P in (32, 64, 128):
            out[f"B{B}_conv1_P{P}"] = timeit(lambda: ops.conv1_wgrad(obs, dy1, pl, P, 1.0 / 255.0))
            out[f"B{B}_conv2_P{P}"] = timeit(lambda: ops.conv_wgrad_nhwc(2, y1, dy2, pl, P))
            out[f"B{B}_conv3_P{P}"] = timeit(lambda: ops.conv_wgrad_nhwc(3, y2, dy3, pl, P))
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
