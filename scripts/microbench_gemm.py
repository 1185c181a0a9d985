"""Micro-benchmark: per-launch cost of the engine's GEMM shapes and of an empty kernel, in a captured hipGraph
chain (back-to-back dependent launches), to separate launch/boundary floors from kernel work."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def graph_time(fn, reps=200):
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
    t = time.perf_counter()
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / 5 / reps * 1e6


def main():
    ops = _native.require()
    dev = torch.device("cuda:0")
    res = {}
    x = torch.zeros(4, device=dev)
    y = torch.zeros(4, device=dev)
    res["normalize_4elems"] = graph_time(lambda: ops.normalize(x, y, 1e-8))
    tiny = torch.zeros(1024, device=dev)
    res["torch_add_1k"] = graph_time(lambda: tiny.add_(1.0))
    B = 32
    bf = torch.bfloat16
    obs = torch.randint(0, 255, (B, 4, 84, 84), dtype=torch.uint8, device=dev)
    y1 = torch.randn(B * 400, 32, device=dev).to(bf)
    y2 = torch.randn(B * 81, 64, device=dev).to(bf)
    y3 = torch.randn(B * 49, 64, device=dev).to(bf)
    h = torch.randn(B, 512, device=dev).to(bf)
    W1 = torch.randn(32 * 256, device=dev).to(bf)
    W2 = torch.randn(64 * 512, device=dev).to(bf)
    W3 = torch.randn(64 * 576, device=dev).to(bf)
    Wfc = torch.randn(3136 * 512, device=dev).to(bf)
    b = torch.zeros(512, device=dev)
    ws = G.GemmWorkspace(dev)
    shapes = {
        "conv1_fwd": lambda t, k, s: G.gemm(obs, 0, True, W1, 256, True, y1, 32, 1, B * 400, 32, 256, bias=b,
                                            relu=True, tile=t, bk=k, splits=s, workspace=ws,
                                            ga=[1, B, 4, 84, 84, 8, 8, 4], ga_scale=1 / 255),
        "conv2_fwd": lambda t, k, s: G.gemm(y1, 0, True, W2, 512, True, y2, 64, 1, B * 81, 64, 512, bias=b,
                                            relu=True, tile=t, bk=k, splits=s, workspace=ws,
                                            ga=[2, B, 32, 20, 20, 4, 4, 2]),
        "conv3_fwd": lambda t, k, s: G.gemm(y2, 0, True, W3, 576, True, y3, 64, 1, B * 49, 64, 576, bias=b,
                                            relu=True, tile=t, bk=k, splits=s, workspace=ws,
                                            ga=[2, B, 64, 9, 9, 3, 3, 1]),
        "fc_fwd": lambda t, k, s: G.gemm(y3, 3136, True, Wfc, 512, False, h, 512, 1, B, 512, 3136, bias=b,
                                         relu=True, tile=t, bk=k, splits=s, workspace=ws),
    }
    for name, f in shapes.items():
        best = None
        rows = []
        for tile, bks in G.BKS.items():
            for bk in bks:
                for s in (1, 2, 4, 8, 16):
                    try:
                        us = graph_time(lambda: f(tile, bk, s), reps=100)
                    except Exception as e:  # unsupported / too many splits
                        continue
                    rows.append((round(us, 2), tile, bk, s))
        rows.sort()
        res[name] = rows[:6]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
