"""Phase stamps of the persistent trunk data-gradient kernel (cnn_fused.hip cnn_trunk_bwd_persist_kernel) at the PPO
learner batch: per-workgroup s_memrealtime stamps of its first two samples, medians over workgroups, plus the
event-timed launch. GPU only. python scripts/exp/trunk_bwd_phases.py [--B 4096] [--persist 256]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--persist", type=int, default=256)
    ap.add_argument("--fold", action="store_true", help="conv1 weight gradient folded in (dy1 not stored)")
    a = ap.parse_args()
    ops = _native.require()
    dev, B = "cuda:0", a.B
    g = torch.Generator(device="cpu").manual_seed(0)
    bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(dev)
    dy3, W3, y2, W2, y1 = bf(B * 49, 64), bf(64 * 576), torch.relu(bf(B * 81, 64)), bf(64 * 512), torch.relu(bf(B * 400, 32))
    dy2 = torch.empty(B * 81, 64, dtype=torch.bfloat16, device=dev)
    dy1 = torch.empty(B * 400, 32, dtype=torch.bfloat16, device=dev)
    biasp = torch.empty(B * 160, device=dev)
    obs = torch.randint(0, 256, (B, 4, 84, 84), dtype=torch.uint8, generator=g).to(dev)
    planes = torch.empty(a.persist * 8192, device=dev)
    if a.fold:
        run = lambda st=None: ops.cnn_trunk_bwd(dy3, W3, y2, W2, y1, dy2, dy1, biasp, st, a.persist, obs, None, planes,
                                                1.0 / 255.0, True, True)
    else:
        run = lambda st=None: ops.cnn_trunk_bwd(dy3, W3, y2, W2, y1, dy2, dy1, biasp, st, a.persist)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e3 / 20
    st = torch.zeros(B * 16, dtype=torch.int64, device=dev)
    run(st)
    torch.cuda.synchronize()
    x = st.view(B, 16)[:a.persist].double().cpu() * 10e-3   # 100 MHz -> us
    names = ["stage+barrier", "dy2 mfma+epi+barrier", "dy2 out+dy1 mfma", "barrier+d1 write+barrier", "dy1 out+barrier (+ conv1 fold)"]
    out = {"B": B, "persist": a.persist, "fold": a.fold, "launch_us": round(t, 2), "per_sample_us": round(t / (B / a.persist), 3)}
    for it in (0, 1):
        ph = {}
        for k, n in enumerate(names):
            d = x[:, it * 8 + k + 1] - x[:, it * 8 + k]
            ph[n] = round(float(d.median()), 3)
        ph["total"] = round(float((x[:, it * 8 + 5] - x[:, it * 8]).median()), 3)
        ph["  of which dy2 mfma loop"] = round(float((x[:, it * 8 + 6] - x[:, it * 8 + 1]).median()), 3)
        ph["  of which dy2 epilogue+db3"] = round(float((x[:, it * 8 + 7] - x[:, it * 8 + 6]).median()), 3)
        ph["  of which barrier wait"] = round(float((x[:, it * 8 + 2] - x[:, it * 8 + 7]).median()), 3)
        out[f"sample{it}"] = ph
    out["loop_gap_us"] = round(float((x[:, 8] - x[:, 5]).median()), 3)
    out["start_spread_us"] = round(float(x[:, 0].max() - x[:, 0].min()), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
