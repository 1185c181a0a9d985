"""Instruction-mix driver for the PPO-learner trunk kernels: the per-env trunk forward (cnn_fused.hip
cnn_trunk_fwd_u8_kernel, mode 0) and the persistent trunk data-gradient kernel at B = 4096, 10 launches each, for
rocprofv3 --pmc passes (scripts/exp/r4m.sh). GPU only."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def main():
    ops = _native.require()
    dev, B = "cuda:0", 4096
    g = torch.Generator(device="cpu").manual_seed(0)
    bf = lambda *s: (torch.randn(*s, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    W1, W2, W3 = bf(32, 256), bf(64, 512), bf(64, 576)
    b1, b2, b3 = (torch.zeros(n, device=dev) for n in (32, 64, 64))
    y1 = torch.empty(B * 400, 32, dtype=torch.bfloat16, device=dev)
    y2 = torch.empty(B * 81, 64, dtype=torch.bfloat16, device=dev)
    y3 = torch.empty(B * 49, 64, dtype=torch.bfloat16, device=dev)
    dy3 = bf(B * 49, 64)
    dy2, dy1 = torch.empty_like(y2), torch.empty_like(y1)
    biasp = torch.empty(B * 160, device=dev)
    for _ in range(10):
        G.cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, y1, y2, y3, mode=int(os.environ.get("TRUNK_MODE", "3")))
    for _ in range(10):
        ops.cnn_trunk_bwd(dy3, W3.view(-1), y2, W2.view(-1), y1, dy2, dy1, biasp, None, 256)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
