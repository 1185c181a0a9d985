"""A/B of the per-env trunk forward forms at the PPO learner batch (B = 4096 through an index, as the minibatch
forward reads them): mode 0 (lean, bytes converted in conv1's loop) vs mode 3 (bf16-staged). Event-timed, 20
launches each after warm-up; mode 5 = mode 3 reading fragment-ordered weight copies (one contiguous 1 KB read per
wave fragment load), checked bitwise against mode 3. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def main():
    dev, R, B = "cuda:0", 16384, 4096
    g = torch.Generator(device="cpu").manual_seed(0)
    obs = torch.randint(0, 256, (R, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    idx = torch.randperm(R, generator=g)[:B].to(dev)
    bf = lambda *s: (torch.randn(*s, generator=g) * 0.05).to(torch.bfloat16).to(dev)
    W1, W2, W3 = bf(32, 256), bf(64, 512), bf(64, 576)
    b1, b2, b3 = (torch.zeros(n, device=dev) for n in (32, 64, 64))
    ys = [torch.empty(B * r, c, dtype=torch.bfloat16, device=dev) for r, c in ((400, 32), (81, 64), (49, 64))]
    # fragment order: [tile][k-step][lane = lg*16 + row16][8 elements]
    F1 = W1.view(2, 16, 8, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    F2 = W2.view(4, 16, 16, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    F3 = W3.view(4, 16, 18, 4, 8).permute(0, 2, 3, 1, 4).contiguous()
    G.cnn_trunk_fwd(obs, W1, b1, W2, b2, W3, b3, *ys, mode=3, obs_idx=idx)
    ref = [y.clone() for y in ys]
    G.cnn_trunk_fwd(obs, F1, b1, F2, b2, F3, b3, *ys, mode=5, obs_idx=idx)
    torch.cuda.synchronize()
    out = {"frag_bitwise": all(torch.equal(a, b) for a, b in zip(ref, ys))}
    for rep in range(2):
        for mode in (0, 3, 5):
            w = (F1, F2, F3) if mode == 5 else (W1, W2, W3)
            run = lambda: G.cnn_trunk_fwd(obs, w[0], b1, w[1], b2, w[2], b3, *ys, mode=mode, obs_idx=idx)
            for _ in range(3):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run()
            e1.record()
            torch.cuda.synchronize()
            out[f"mode{mode}_rep{rep}_us"] = round(e0.elapsed_time(e1) * 1e3 / 20, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
