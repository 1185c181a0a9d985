"""Times the three Nature-CNN fc products of the PPO learner (B = 4096) on gemm_big launch variants (XCD order x LDS
ring depth x split-K), the general gemm kernel and torch.matmul (hipBLASLt), plus gemm_big's per-workgroup phase
stamps. GPU only. Usage: python scripts/exp/gemm_big_bench.py [--B 4096]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def timeit(fn, reps=40):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    a = ap.parse_args()
    B, dev = a.B, "cuda:0"
    torch.manual_seed(0)
    y3 = torch.relu(torch.randn(B, 3136, device=dev)).bfloat16()
    W = (torch.randn(3136, 512, device=dev) * 0.02).bfloat16()
    dh = torch.randn(B, 512, device=dev).bfloat16()
    bias = torch.randn(512, device=dev)
    h = torch.empty(B, 512, device=dev, dtype=torch.bfloat16)
    dy3 = torch.empty(B, 3136, device=dev, dtype=torch.bfloat16)
    gW = torch.empty(3136, 512, device=dev)
    ws = G.GemmBigWorkspace(dev)
    shapes = {
        "fwd": (lambda v, s, st=None: G.gemm_big(y3, 3136, True, W, 512, False, h, 512, 1, B, 512, 3136, bias=bias,
                                                 relu=True, splits=s, workspace=ws, variant=v, stamps=st),
                lambda: G.gemm(y3, 3136, True, W, 512, False, h, 512, 1, B, 512, 3136, bias=bias, relu=True),
                lambda: torch.relu(y3 @ W + bias), 2.0 * B * 512 * 3136, (B, 512)),
        "dy3": (lambda v, s, st=None: G.gemm_big(dh, 512, True, W, 512, True, dy3, 3136, 1, B, 3136, 512, mask=y3,
                                                 ldm=3136, splits=s, workspace=ws, variant=v, stamps=st),
                lambda: G.gemm(dh, 512, True, W, 512, True, dy3, 3136, 1, B, 3136, 512, mask=y3, ldm=3136),
                lambda: (dh @ W.t()) * (y3 > 0), 2.0 * B * 512 * 3136, (B, 3136)),
        "dWfc": (lambda v, s, st=None: G.gemm_big(y3, 3136, False, dh, 512, False, gW, 512, 0, 3136, 512, B,
                                                  splits=s, workspace=ws, variant=v, stamps=st),
                 lambda: G.gemm(y3, 3136, False, dh, 512, False, gW, 512, 0, 3136, 512, B),
                 lambda: y3.t() @ dh, 2.0 * B * 512 * 3136, (3136, 512)),
    }
    for name, (big, gen, ref, flop, (M, N)) in shapes.items():
        t_gen = timeit(gen)
        t_ref = timeit(ref)
        print(f"{name}: general gemm {t_gen:.1f} us ({flop / t_gen / 1e6:.0f} TF/s)  torch {t_ref:.1f} us "
              f"({flop / t_ref / 1e6:.0f} TF/s)", flush=True)
        best = None
        for s in (1, 2):
            for v in (0, 1, 5, 9):
                try:
                    t = timeit(lambda: big(v, s))
                except RuntimeError as e:
                    print(f"  v{v} s{s}: {e}")
                    continue
                print(f"  gemm_big v{v} (xcd {v & 1}, ring {2 + ((v >> 1) & 3)}, scalar-epi {v >> 3}) splits {s}: {t:.1f} us "
                      f"({flop / t / 1e6:.0f} TF/s)", flush=True)
                if best is None or t < best[0]:
                    best = (t, v, s)
        t, v, s = best
        grid = -(-M // 128) * -(-N // 128) * s
        st = torch.zeros(grid, 8, dtype=torch.int64, device=dev)
        big(v, s)
        big(v, s, st)
        torch.cuda.synchronize()
        raw = st.cpu()
        x = raw[:, :4].double() * 10e-3   # 100 MHz realtime counter -> us
        t0 = x[:, 0].min()
        loop = x[:, 1] - x[:, 0]
        q = torch.quantile(loop, torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.float64)).tolist()
        fin = x[:, 3] > 0   # split-K: only the last arriver reaches the epilogue
        epi = (x[fin, 3] - x[fin, 1]).mean().item()
        hw, xcc = raw[:, 4], raw[:, 5]
        cu = (xcc & 0xF) * 256 + ((hw >> 13) & 7) * 32 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 0xF)
        _, counts = torch.unique(cu, return_counts=True)
        print(f"  best v{v} s{s} {t:.1f} us; stamps (grid {grid}): start spread {(x[:, 0].max() - t0).item():.1f} us, "
              f"loop min/med/p90/max {q[0]:.1f}/{q[1]:.1f}/{q[2]:.1f}/{q[3]:.1f}, reduce+epilogue {epi:.1f}, "
              f"span {(x[fin, 3].max() - t0).item():.1f} us; {len(counts)} distinct CUs, max {int(counts.max())} "
              f"workgroups on one CU, starts after t0+5us: {int(((x[:, 0] - t0) > 5).sum())}", flush=True)


if __name__ == "__main__":
    main()
