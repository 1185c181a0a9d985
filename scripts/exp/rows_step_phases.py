"""Phase stamps of the row-split fused rollout step (cnn_fused.hip pong_fused_step_kernel, 7 workgroups per env) at
the headline bank (Pong, 32 envs): per-workgroup s_memrealtime stamps, medians over workgroups; conv2 / conv3 weights
fragment-ordered (EngineOpts.frag_weights) and row-major. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer, KEY_ENV_BITS  # noqa: E402

# stamp order in time: 0 start, 8 staged + barrier, 9 sampled + barrier, 1 rendered + barrier, 2 conv1 + barrier,
# 3 conv2 + barrier, 4 conv3 + owned rows issued
ORDER = [(0, 8, "loads + head + staging + barrier"), (8, 9, "sampling + barrier"), (9, 1, "commit + render + barrier"),
         (1, 2, "conv1 + barrier"), (2, 3, "conv2 + barrier"), (3, 4, "conv3 + y stores issued")]


def main():
    ops = _native.require()
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, cuda_graph=False, seed=3))
    tr.step()
    st, env, eng = tr.storage, tr.env, tr.engine
    N = env.num_envs
    b = eng.bufs(N)
    eng.forward(st.obs[0], b, head=False, shift_out=st.obs[1], fc_parts=True)
    out = {}
    _, F2, F3, _ = eng.trunk_w()
    for frag in (True, False):
        W2, W3 = (F2, F3) if frag else (eng.sW2, eng.sW3)
        out["frag" if frag else "rowmajor"] = phases(ops, tr, st, env, eng, N, b, W2, W3, frag)
    print(json.dumps(out, indent=1))


def phases(ops, tr, st, env, eng, N, b, W2, W3, frag):
    sts = torch.zeros(N * 7 * 16, dtype=torch.int64, device="cuda:0")
    res = {}
    for rep in range(6):
        hp, S = eng.last_fc
        sn, tn, tgn, ern = env.next_state()
        ops.pong_fused_step(b.h, eng.sWh, eng.bh, b.z, st.actions[0], st.logp[0], st.entropy[0], st.values[0],
                            KEY_ENV_BITS, tr.policy_seed, env.state, env.t, env.tg, env.ep_ret, sn, tn, tgn, ern,
                            env.ep_stats, env.env_ids, st.obs[0], st.obs[1], st.rewards[0], st.dones[0],
                            st.truncated[0], env.seed, env.max_episode_steps, hp, S, eng.bfc, eng.sW1, eng.b1,
                            W2, eng.b2, W3, eng.b3, b.y1, b.y2, b.y3, 1.0 / 255.0, st.obs[2],
                            sts if rep == 5 else None, frag)
        env.flip()
    torch.cuda.synchronize()
    x = sts.view(N * 7, 16).double().cpu() * 10e-3
    for a, c, name in ORDER:
        res[name] = round(float((x[:, c] - x[:, a]).median()), 2)
    res["  of conv1: MFMAs + epilogue (to the W2/W3 issue)"] = round(float((x[:, 10] - x[:, 1]).median()), 2)
    res["total (start -> conv3 issued)"] = round(float((x[:, 4] - x[:, 0]).median()), 2)
    res["start spread us"] = round(float(x[:, 0].max() - x[:, 0].min()), 2)
    res["first start -> last end us"] = round(float(x[:, 4].max() - x[:, 0].min()), 2)
    return res


if __name__ == "__main__":
    main()
