"""Headline learner fc backward at B = 160 (A2C Pong, 32 envs x 5 steps): dy3 = (dh Wfc^T) * (y3 > 0) and
dWfc = y3^T dh, alone and as the engine's grouped launch, vs torch.matmul (hipBLASLt) on the same shapes.
Event-timed, 50 launches after warm-up. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def timed(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / n, 2)


def main():
    dev = "cuda:0"
    g = torch.Generator(device="cpu").manual_seed(0)
    out = {}
    for B in (160, 4096):
        dh = (torch.randn(B, 512, generator=g) * 0.1).to(torch.bfloat16).to(dev)
        y3 = torch.relu(torch.randn(B, 3136, generator=g)).to(torch.bfloat16).to(dev)
        Wfc = (torch.randn(3136, 512, generator=g) * 0.02).to(torch.bfloat16).to(dev)
        dy3 = torch.empty(B, 3136, dtype=torch.bfloat16, device=dev)
        gW = torch.empty(3136, 512, dtype=torch.float32, device=dev)
        ws, ws2 = G.GemmWorkspace(dev), G.GemmWorkspace(dev)
        f_dy3 = lambda: G.gemm(dh, 512, True, Wfc, 512, True, dy3, 3136, 1, B, 3136, 512, mask=y3, ldm=3136,
                               workspace=ws)
        f_dw = lambda: G.gemm(y3, 3136, False, dh, 512, False, gW, 512, 0, 3136, 512, B, workspace=ws2)

        def f_group():
            with G.group():
                f_dy3()
                f_dw()
        r = {"dy3_us": timed(f_dy3), "dWfc_us": timed(f_dw), "group_us": timed(f_group)}
        r["torch_dy3_us"] = timed(lambda: torch.mm(dh, Wfc.t(), out=dy3))
        gWb = torch.empty(3136, 512, dtype=torch.bfloat16, device=dev)
        r["torch_dWfc_bf16out_us"] = timed(lambda: torch.mm(y3.t(), dh, out=gWb))
        r["torch_dWfc_f32_us"] = timed(lambda: torch.mm(y3.t().float(), dh.float(), out=gW))
        out[f"B{B}"] = r
    print(json.dumps(out))


if __name__ == "__main__":
    main()
