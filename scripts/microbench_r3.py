"""Standalone timings (graph-captured back-to-back launches, warm caches) of the Breakout-PPO learner products at
the minibatch size B = 4096: conv2 / conv3 weight gradients (batched-position MFMA32 kernel vs per-sample kernel,
several plane counts) and the three fc-layer GEMMs (32x32x16-MFMA kernel vs the general GEMM with its tuned plan).
Prints one JSON object: {name: {"us": ..., "tflops": ...}}.

    python scripts/microbench_r3.py
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def time_fn(fn, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        t = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t) / reps * 1e6)
    return best


def main():
    ops = _native.require()
    dev = "cuda:0"
    B = 4096
    out = {}
    # conv weight gradients
    for layer, (H, C, KS, OH) in ((3, (9, 64, 3, 7)), (2, (20, 32, 4, 9))):
        img = torch.rand(B * H * H, C, device=dev).to(torch.bfloat16)
        dy = (torch.randn(B * OH * OH, 64, device=dev) * 0.1).to(torch.bfloat16)
        n = KS * KS * C
        flop = 2.0 * B * OH * OH * 64 * n
        planes = torch.zeros(1024 * 64 * n, device=dev)
        for P in (64, 128, 256, 512):
            us = time_fn(lambda: ops.conv_wgrad_gemm(layer, img, dy, planes, P))
            out[f"wgrad{layer}_gemm_P{P}"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    # fc GEMMs (PPO minibatch)
    y3 = torch.randn(B * 3136, device=dev).to(torch.bfloat16)
    dh = torch.randn(B * 512, device=dev).to(torch.bfloat16)
    Wfc = (torch.randn(3136 * 512, device=dev) * 0.02).to(torch.bfloat16)
    bfc = torch.zeros(512, device=dev)
    h = torch.empty(B * 512, dtype=torch.bfloat16, device=dev)
    dy3 = torch.empty(B * 3136, dtype=torch.bfloat16, device=dev)
    gW = torch.empty(3136 * 512, device=dev)
    ws = G.GemmWorkspace(torch.device(dev))
    shapes = {
        "fc_fwd": (y3, 3136, True, Wfc, 512, False, h, 512, 1, B, 512, 3136, dict(bias=bfc, relu=True)),
        "fc_dy3": (dh, 512, True, Wfc, 512, True, dy3, 3136, 1, B, 3136, 512, dict(mask=y3, ldm=3136)),
        "fc_dW": (y3, 3136, False, dh, 512, False, gW, 512, 0, 3136, 512, B, {}),
    }
    for name, (A, lda, ak, Bm, ldb, bk, Cm, ldc, om, M, N, K, kw) in shapes.items():
        flop = 2.0 * M * N * K
        us = time_fn(lambda: ops.gemm_mfma32(A, lda, ak, Bm, ldb, bk, Cm, ldc, om, M, N, K, 1.0, kw.get("bias"),
                                             bool(kw.get("relu", False)), kw.get("mask"), kw.get("ldm", 0), 1))
        out[f"{name}_mfma32"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
        G.GEMM32 = False
        us = time_fn(lambda: G.gemm(A, lda, ak, Bm, ldb, bk, Cm, ldc, om, M, N, K, workspace=ws, **kw))
        G.GEMM32 = True
        out[f"{name}_general"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
        # hipBLASLt (torch.matmul) on the plain product, as a yardstick only
        Am = (A.view(M, K) if ak else A.view(K, M).t())
        Bmm = (Bm.view(N, K).t() if bk else Bm.view(K, N))
        us = time_fn(lambda: torch.matmul(Am, Bmm))
        out[f"{name}_hipblaslt_ref"] = {"us": round(us, 2), "tflops": round(flop / us / 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
