"""Trunk data-gradient chain v1 (cnn_fused.hip per-sample / persistent kernels) vs v2 (trunk_bwd2.hip) at the
headline learner batch (B = 160, one workgroup per sample) and the Breakout minibatch (B = 4096, 256 workgroups
walking), graph-chained x20, plus v2's phase stamps (first sample of each workgroup). GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def main():
    ops = _native.require()
    dev = "cuda:0"
    out = {}
    for B, persist in ((160, 0), (4096, 256)):
        g = torch.Generator(device="cpu").manual_seed(0)
        bf = lambda *s: torch.randn(*s, generator=g).to(torch.bfloat16).to(dev)   # noqa: E731
        dy3, W3, y2, W2, y1 = (bf(B * 49, 64), bf(64 * 576), torch.relu(bf(B * 81, 64)), bf(64 * 512),
                               torch.relu(bf(B * 400, 32)))
        dy2 = torch.empty(B * 81, 64, dtype=torch.bfloat16, device=dev)
        dy1 = torch.empty(B * 400, 32, dtype=torch.bfloat16, device=dev)
        bp = torch.empty(B * 160, device=dev)
        v1 = lambda: ops.cnn_trunk_bwd(dy3, W3, y2, W2, y1, dy2, dy1, bp, None, persist)   # noqa: E731
        v2 = lambda: ops.cnn_trunk_bwd2(dy3, W3, y2, W2, y1, dy2, dy1, bp, None, persist)   # noqa: E731
        r = {}
        for name, fn in (("v1_us", v1), ("v2_us", v2)):
            gr = make_graph(fn, 20)
            r[name] = round(min(time_graph(gr, 20) for _ in range(3)), 2)
            del gr
        grid = persist if persist else B
        st = torch.zeros(grid * 16, dtype=torch.int64, device=dev)
        ops.cnn_trunk_bwd2(dy3, W3, y2, W2, y1, dy2, dy1, bp, st, persist)
        torch.cuda.synchronize()
        x = st.view(grid, 16).double().cpu() * 10e-3
        names = {1: "staged", 6: "dy2_mfma", 2: "dy2_epilogue", 3: "dy1_mfma", 5: "dy1_epilogue"}
        prev, ph = 0, {}
        for k in (1, 6, 2, 3, 5):
            ph[names[k]] = round(float((x[:, k] - x[:, prev]).median()), 3)
            prev = k
        ph["sample_total"] = round(float((x[:, 5] - x[:, 0]).median()), 3)
        if persist:
            ph["second_sample_total"] = round(float((x[:, 13] - x[:, 8]).median()), 3)
        r["v2_phases_first_sample"] = ph
        out[f"B{B}"] = r
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
