"""Headline learner fc backward (B = 160): fc_bwd.hip vs the grouped general-GEMM launch it replaces, graph-chained
x50 on the trained engine's buffers, plus fc_bwd's per-workgroup phase stamps (entry, operands in, MFMAs done,
stores issued) by job kind. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def main():
    ops = _native.require()
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0))
    tr.capture(warmup=2)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    eng = tr.engine
    B = tr.storage.T * tr.env.num_envs
    b = eng.bufs(B, with_grad=True)

    def fcb():
        ops.fc_bwd(b.dh, eng.sWfc, b.y3, b.dy3, eng.gWfc)

    def grp():
        with G.group():
            G.gemm(b.dh, 512, True, eng.sWfc, 512, True, b.dy3, 3136, 1, B, 3136, 512, mask=b.y3, ldm=3136,
                   workspace=eng.ws)
            G.gemm(b.y3, 3136, False, b.dh, 512, False, eng.gWfc, 512, 0, 3136, 512, B, workspace=eng._side_ws())

    out = {}
    for name, fn in (("fc_bwd_us", fcb), ("grouped_gemm_us", grp)):
        g = make_graph(fn, 50)
        out[name] = round(min(time_graph(g, 50) for _ in range(5)), 2)
        del g
    nwg = 392 + ((B + 31) // 32) * 49
    st = torch.zeros(nwg * 4 + 16, dtype=torch.int64, device="cuda:0")
    fcb()
    ops.fc_bwd(b.dh, eng.sWfc, b.y3, b.dy3, eng.gWfc, st)
    torch.cuda.synchronize()
    x = st[:nwg * 4].view(nwg, 4).double().cpu() * 10e-3
    t0 = float(x[:, 0].min())
    for kind, sl in (("dw", slice(0, 392)), ("dy", slice(392, nwg))):
        y = x[sl]
        out[kind] = {"start_med": round(float((y[:, 0] - t0).median()), 2),
                     "start_max": round(float((y[:, 0] - t0).max()), 2),
                     "operands_med": round(float((y[:, 1] - y[:, 0]).median()), 2),
                     "mfma_med": round(float((y[:, 2] - y[:, 1]).median()), 2),
                     "stores_med": round(float((y[:, 3] - y[:, 2]).median()), 2),
                     "end_max": round(float((y[:, 3] - t0).max()), 2)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
