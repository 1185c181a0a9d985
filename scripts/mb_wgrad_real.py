"""Per-sample conv3 / conv2 weight-gradient kernels timed on the Breakout PPO learner's own buffers vs random data."""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from scripts.mb_wgrad import timeit  # noqa: E402


def main():
    ops = _native.require()
    tr = ActorCriticTrainer(preset("breakout_ppo", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, cuda_graph=False))
    tr.step()
    torch.cuda.synchronize()
    eng = tr.engine
    b = eng.bufs(4096, with_grad=True)
    pl = torch.zeros(64 * 64 * 576, device="cuda:0")
    out = {"real_conv3": timeit(lambda: ops.conv_wgrad_nhwc(3, b.y2, b.dy3, pl, 64)),
           "real_conv2": timeit(lambda: ops.conv_wgrad_nhwc(2, b.y1, b.dy2, pl, 64))}
    y2r, dy3r = torch.rand_like(b.y2.float()).to(torch.bfloat16), torch.randn_like(b.dy3.float()).to(torch.bfloat16)
    out["rand_conv3"] = timeit(lambda: ops.conv_wgrad_nhwc(3, y2r, dy3r, pl, 64))
    out["real_y2_rand_dy3"] = timeit(lambda: ops.conv_wgrad_nhwc(3, b.y2, dy3r, pl, 64))
    out["rand_y2_real_dy3"] = timeit(lambda: ops.conv_wgrad_nhwc(3, y2r, b.dy3, pl, 64))
    out["shapes"] = [list(b.y2.shape), list(b.dy3.shape), b.y2.stride(), b.dy3.stride()]
    z = b.dy3.float()
    out["dy3_zero_frac"] = float((z == 0).float().mean())
    out["dy3_absmax"] = float(z.abs().max())
    out["dy3_min_nonzero"] = float(z[z != 0].abs().min()) if bool((z != 0).any()) else 0.0
    print(json.dumps(out))


if __name__ == "__main__":
    main()
