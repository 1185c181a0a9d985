"""Headline learner conv weight gradients (B = 160): graph-chained x50 times of each product alone and of the grouped
launch the engine issues, for the implicit-GEMM path (default at this batch) and the dedicated kernels
(conv1_wgrad.hip per-sample planes, conv_wgrad_gemm batched positions) at several plane counts. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def main():
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0))
    tr.capture(warmup=2)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    eng = tr.engine
    B = tr.storage.T * tr.env.num_envs
    b = eng.bufs(B, with_grad=True)
    ws, ws2 = eng.ws, eng._side_ws()

    def t(fn):
        g = make_graph(fn, 50)
        r = round(min(time_graph(g, 50) for _ in range(3)), 2)
        del g
        return r

    out = {"gemm_W1": t(lambda: eng._wgrad_conv1(b, ws)),
           "gemm_W2": t(lambda: eng._wgrad_conv23("W2", b, ws2)),
           "gemm_W3": t(lambda: eng._wgrad_conv23("W3", b, ws2))}

    def grp():
        with G.group():
            eng._wgrad_conv1(b, ws)
            eng._wgrad_conv23("W2", b, ws2)
            eng._wgrad_conv23("W3", b, ws2)
    out["gemm_group"] = t(grp)
    out["planes"] = dict(eng._wsplits)
    eng.conv1_wgrad_min_b, eng.nhwc_wgrad_min_b = 1, 1
    for P in (16, 32, 64, 128):
        eng.conv1_planes = P
        out[f"conv1_wgrad_P{P}"] = t(lambda: eng._wgrad_conv1(b, ws))
    for P in (16, 32, 64, 160):
        eng.nhwc_planes, eng.nhwc3_planes = P, P
        out[f"wgrad_gemm_W2_P{P}"] = t(lambda: eng._wgrad_conv23("W2", b, ws2))
        out[f"wgrad_gemm_W3_P{P}"] = t(lambda: eng._wgrad_conv23("W3", b, ws2))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
