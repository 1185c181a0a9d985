"""Compare one rollout of the per-env fused step against the unfused per-env trunk + policy/env launches."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from actor_critic_algs_on_tensorflow_amd import preset
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer
import actor_critic_algs_on_tensorflow_amd.ops.gemm as G
G.TUNE = False
res = []
for fused in (True, False):
    tr = ActorCriticTrainer(preset("pong_a2c", num_envs=72, n_steps=5, device="cuda:0", outdir=None, quiet=True,
                                   stdout_freq=0, save_every=0, seed=5, cuda_graph=False,
                                   engine_opts=dict(fused_step=fused)))
    tr.env.max_episode_steps = 7
    tr.collect()
    torch.cuda.synchronize()
    st = tr.storage
    lb = tr.engine.bufs(st.T * 72, with_grad=True)
    res.append(dict(act=st.actions[:].clone(), logp=st.logp[:].clone(), ent=st.entropy[:].clone(),
                    val=st.values[:].clone(), z=lb.z.clone(), h=lb.h.clone(), y3=lb.y3.clone(),
                    obs=st.obs[:].clone()))
for k in res[0]:
    a, b = res[0][k], res[1][k]
    d = (a.float() - b.float()).abs()
    print(k, "equal" if torch.equal(a, b) else f"max diff {d.max().item():.3e} n_diff {(d > 0).sum().item()} / {d.numel()}")
    if not torch.equal(a, b) and k in ("logp", "z"):
        idx = (d > 0).nonzero()[:5]
        print("  first diffs at", idx.tolist())
