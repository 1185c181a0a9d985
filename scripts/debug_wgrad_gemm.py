"""Repeat check of conv_wgrad_gemm (batched-position conv2/conv3 weight gradient) against the fp32 reference: runs
each case several times in one process and reports the mismatch pattern (rows / columns / planes) if any."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from test_gpu_r3 import _wgrad_ref  # noqa: E402

ops = _native.require()
cuda = torch.device("cuda:0")
for layer, B, P in [(2, 5, 3), (2, 7, 8), (3, 9, 4), (2, 300, 64)]:
    H, C, KS, OH = (20, 32, 4, 9) if layer == 2 else (9, 64, 3, 7)
    n = KS * KS * C
    g = torch.Generator(device="cpu").manual_seed(B * 7 + layer)
    img = torch.rand(B, H, H, C, generator=g).to(torch.bfloat16).to(cuda)
    dy = (torch.randn(B, OH, OH, 64, generator=g) * 0.1).to(torch.bfloat16).to(cuda)
    refs = {}
    for rep in range(6):
        planes = torch.full((P * 64 * n,), float("nan"), device=cuda)
        ops.conv_wgrad_gemm(layer, img.view(B * H * H, C), dy.view(B * OH * OH, 64), planes, P)
        torch.cuda.synchronize()
        pl = planes.view(P, 64, n)
        bad = []
        for gi in range(P):
            b0, b1 = gi * B // P, (gi + 1) * B // P
            if b1 == b0:
                continue
            if gi not in refs:
                refs[gi] = _wgrad_ref(layer, img[b0:b1], dy[b0:b1])
            d = (pl[gi] - refs[gi]).abs() > 1e-4 + 1e-4 * refs[gi].abs()
            if d.any():
                rows = torch.nonzero(d.any(1)).flatten().tolist()
                cols = torch.nonzero(d.any(0)).flatten().tolist()
                bad.append((gi, int(d.sum()), rows[:12], cols[:12], len(cols)))
        print(layer, B, P, "rep", rep, "ok" if not bad else bad, flush=True)
