"""Where the rollout fc launch's time goes (fc_rollout.hip): graph-chained time per launch and in-kernel wave stamps
(s_memrealtime, 100 MHz: entry, operands landed, MFMAs done, stores drained) under three cache conditions --
(a) launches back to back (operands warm in L2), (b) each launch after a kernel that rewrites X (as the fused
rollout step writes y3), (c) as (b) plus a 64 MB read between (cold L2 / MALL). Also an empty-kernel floor (a
1-element torch fill) in the same chain. GPU only. python scripts/exp/fc_rollout_stamps.py [--variants 1,5]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order_kc  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def stamps_summary(st, nwaves):
    s = st[:nwaves * 4].view(nwaves, 4).double().cpu()
    t0 = float(s[:, 0].min())
    us = (s - t0) / 100.0   # 100 MHz -> us
    return {"start_spread_us": round(float(us[:, 0].max()), 2),
            "load_us_median": round(float((us[:, 1] - us[:, 0]).median()), 2),
            "load_us_max": round(float((us[:, 1] - us[:, 0]).max()), 2),
            "mfma_us_median": round(float((us[:, 2] - us[:, 1]).median()), 2),
            "store_us_median": round(float((us[:, 3] - us[:, 2]).median()), 2),
            "end_from_first_start_us": round(float(us[:, 3].max()), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,5")
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    ops = _native.require()
    dev = "cuda:0"
    X = (torch.randn(32, 3136, device=dev) * 0.5).to(torch.bfloat16)
    Xsrc = X.clone()
    W = (torch.randn(3136, 512, device=dev) * 0.05).to(torch.bfloat16)
    Wf = frag_order_kc(W.float(), 3136, 512)
    hp = torch.zeros(32 * 32 * 512, device=dev)
    big = torch.zeros(16 * 1024 * 1024, device=dev)   # 64 MB
    dummy = torch.zeros(1, device=dev)
    stamps = torch.zeros(65536, dtype=torch.int64, device=dev)
    cfg = {0: (2, 7), 1: (4, 7), 2: (1, 14), 3: (7, 4), 4: (7, 2), 5: (2, 14), 6: (1, 7)}
    out = {}
    ws = G.GemmWorkspace(torch.device(dev))
    for v in [int(x) for x in a.variants.split(",")]:
        if v < 0:   # the general GEMM on the row-major operand (no stamps)
            kr, w, S, nwaves = 0, 0, 0, 0
            fc = lambda st=None: G.gemm(X, 3136, True, W, 512, False, hp, 512, 3, 32, 512, 3136,   # noqa: E731
                                        workspace=ws, max_planes=32)
        else:
            kr, w = cfg[v]
            S = 196 // (kr * w)
            nwaves = S * 16 * w
            fc = lambda st=None: ops.fc_rollout(X, Wf, hp, v, st)   # noqa: E731
        scen = {
            "warm": lambda: fc(),
            "after_x_write": lambda: (X.copy_(Xsrc), fc()),
            "cold": lambda: (X.copy_(Xsrc), big.sum(), fc()),
            "floor_fill": lambda: dummy.fill_(1.0),
            "floor_x_write": lambda: X.copy_(Xsrc),
            "floor_cold": lambda: (X.copy_(Xsrc), big.sum()),
        }
        res = {}
        for name, fn in scen.items():
            g = make_graph(fn, a.reps)
            res[name + "_us_per_rep"] = round(min(time_graph(g, a.reps) for _ in range(3)), 2)
            del g
        for name, pre in ((("warm", lambda: None), ("after_x_write", lambda: X.copy_(Xsrc)),
                           ("cold", lambda: (X.copy_(Xsrc), big.sum()))) if v >= 0 else ()):
            sm = []
            for _ in range(20):
                pre()
                fc(stamps)
                torch.cuda.synchronize()
                sm.append(stamps_summary(stamps, nwaves))
            res["stamps_" + name] = {k: statistics.median([d[k] for d in sm]) for k in sm[0]}
        out[f"variant{v}_KR{kr}_W{w}_S{S}"] = res
        print(json.dumps({f"variant{v}": res}), flush=True)


if __name__ == "__main__":
    main()
