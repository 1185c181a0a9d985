"""Per-workgroup timeline of the engine's GEMMs (s_memrealtime stamps from the kernel's diagnostic hook):
workgroup start spread (dispatch), prologue (first k-step's loads -> LDS), k-loop, epilogue, per product, on the
bench configuration's shapes with the tuned plans. Usage (GPU box): python scripts/microbench_gemm_stamps.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.ops import gemm as G  # noqa: E402


def timeline(name, fn, wgs):
    st = torch.zeros(wgs, 4, dtype=torch.int64, device="cuda")
    fn(None)
    torch.cuda.synchronize()
    fn(st)
    torch.cuda.synchronize()
    s = st.cpu().double() * 10e-3   # 100 MHz ticks -> us
    t0 = s[:, 0].min()
    q = lambda x: [round(float(v), 2) for v in torch.quantile(x, torch.tensor([0.1, 0.5, 0.9], dtype=x.dtype))]  # noqa
    return {"name": name, "wgs": wgs, "kernel_us": round(float(s[:, 3].max() - t0), 2),
            "start_offsets_p10_50_90": q(s[:, 0] - t0), "prologue": q(s[:, 1] - s[:, 0]),
            "kloop": q(s[:, 2] - s[:, 1]), "epilogue": q(s[:, 3] - s[:, 2]), "wg_total": q(s[:, 3] - s[:, 0])}


def main():
    cfg = preset("pong_a2c", num_envs=32, device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0)
    tr = ActorCriticTrainer(cfg)
    tr.capture(warmup=3)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    eng = tr.engine
    B = tr.storage.T * tr.env.num_envs
    b = eng.bufs(B, with_grad=True)
    plans = G.tuned_plans()
    out = []

    def run(name, M, N, K, key_match, call):
        hit = [(k, v) for k, v in plans.items() if k[0] == M and k[1] == N and k[2] == K and key_match(k)]
        if not hit:
            return
        tile, bk, splits = hit[0][1][:3]
        bm, bn = G.TILES[tile]
        wgs = G._cdiv(M, bm) * G._cdiv(N, bn) * G.effective_splits(K, bk, splits)
        out.append(timeline(name + f" tile{tile} bk{bk} s{splits}", lambda st: call(tile, bk, splits, st), wgs))

    ws = eng.ws
    run("conv2_dgrad_tconv", B * 400, 32, 1024, lambda k: k[8][:1] == (3,),
        lambda t, k, s, st: G.gemm(b.dy2, 0, True, eng.sW2, 0, False, b.dy1, 32, 1, B * 400, 32, 1024, mask=b.y1,
                                   ldm=32, workspace=ws, ga=[3, B, 64, 20, 20, 4, 4, 2],
                                   gb=[4, 1, 64, 1, 32, 4, 4, 1], tile=t, bk=k, splits=s, stamps=st))
    run("conv3_dgrad_tconv", B * 81, 64, 576, lambda k: k[8][:1] == (3,),
        lambda t, k, s, st: G.gemm(b.dy3, 0, True, eng.sW3, 0, False, b.dy2, 64, 1, B * 81, 64, 576, mask=b.y2,
                                   ldm=64, workspace=ws, ga=[3, B, 64, 9, 9, 3, 3, 1],
                                   gb=[4, 1, 64, 1, 64, 3, 3, 1], tile=t, bk=k, splits=s, stamps=st))
    run("dy3", B, 3136, 512, lambda k: True,
        lambda t, k, s, st: G.gemm(b.dh, 512, True, eng.sWfc, 512, True, b.dy3, 3136, 1, B, 3136, 512, mask=b.y3,
                                   ldm=3136, workspace=ws, tile=t, bk=k, splits=s, stamps=st))
    N = tr.env.num_envs
    hp = eng.hpart(N)
    run("fc_fwd_parts", N, 512, 3136, lambda k: k[5] == 3,
        lambda t, k, s, st: G.gemm(b.y3[:N * 49], 3136, True, eng.sWfc, 512, False, hp, 512, 3, N, 512, 3136,
                                   workspace=ws, tile=t, bk=k, splits=s, stamps=st))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
