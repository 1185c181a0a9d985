"""Library GEMM (torch.matmul -> hipBLASLt / rocBLAS) on the Breakout learner's fc shapes (B = 4096, K = 3136,
N = 512), bf16 in, for comparison with the engine's own GEMM launches in the Breakout trace
(profiles/r3_breakout_ab2.txt: forward 47.3 us, dWfc 43.3 us, dy3 ~47 us).

Usage (GPU box): python scripts/probes/fc_gemm_library.py
"""
import json

import torch


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = "cuda"
    B, K, N = 4096, 3136, 512
    y3 = torch.randn(B, K, device=dev).bfloat16()
    W = torch.randn(N, K, device=dev).bfloat16()       # [N][K]
    dh = torch.randn(B, N, device=dev).bfloat16()
    out = {}
    f = 2 * B * K * N / 1e12
    out["fwd_y3_WT_bf16out_us"] = timeit(lambda: y3 @ W.t())
    out["dW_y3T_dh_bf16out_us"] = timeit(lambda: y3.t() @ dh)
    out["dW_y3T_dh_fp32out_us"] = timeit(lambda: torch.matmul(y3.t(), dh, out_dtype=torch.float32)
                                         if "out_dtype" in torch.matmul.__doc__ else (y3.t() @ dh).float())
    out["dy3_dh_W_bf16out_us"] = timeit(lambda: dh @ W)
    out["TF_per_s"] = {k: round(f / (v * 1e-6), 1) for k, v in out.items() if k.endswith("_us")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
