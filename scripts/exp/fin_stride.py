"""grad_finalize plane reduction vs plane stride: 256 planes of a 64 x 512 conv weight gradient (the Breakout conv2
shape) at the power-of-two stride the wgrad kernels write and at padded strides; plus 4096 per-sample bias rows."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops.optim import finalize_jobs  # noqa: E402


def timed(fn, n=30):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / n, 2)


def main():
    ops = _native.require()
    dev = "cuda:0"
    n, S = 32768, 256
    out = {}
    parts = torch.zeros(256, device=dev)
    dst = torch.zeros(n, device=dev)
    for pad in (0, 64, 256, 1024):
        st = n + pad
        planes = torch.randn(S * st, device=dev)
        for njobs_elems in (1024, 256):
            segs = []
            for a in range(0, n, njobs_elems):
                segs.append((dst.data_ptr() + 4 * a, planes.data_ptr() + 4 * a, min(njobs_elems, n - a), st, S))
            words = finalize_jobs(segs, dev)
            out[f"pad{pad}_ch{njobs_elems}_jobs{len(segs)}"] = timed(lambda: ops.grad_finalize(words, parts))
        ref = planes.view(S, st)[:, :n].sum(0)
        assert torch.allclose(dst, ref, rtol=1e-4, atol=1e-3)
        del planes
    rows = torch.randn(4096, 160, device=dev)
    b = torch.zeros(160, device=dev)
    for k in (1, 4, 16):
        # the 3 bias segments (64 | 64 | 32 columns), optionally split into k row ranges (partials not combined here)
        segs = []
        for c0, w in ((0, 64), (64, 64), (128, 32)):
            for j in range(k):
                r0 = j * 4096 // k
                segs.append((b.data_ptr() + 4 * c0, rows.data_ptr() + 4 * (r0 * 160 + c0), w, 160, 4096 // k))
        words = finalize_jobs(segs, dev)
        out[f"bias_rows_split{k}"] = timed(lambda: ops.grad_finalize(words, parts))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
