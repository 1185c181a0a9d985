"""The fused step's in-launch fc product (EngineOpts.fused_fc) at the headline bank: graph-chained time of
[fused step with the fc tail] vs [fused step ; fc_rollout], and phase stamps of the tail (slot 4 conv3 issued, 11 row
published + arrival, 12 slice wait passed, 13 planes stored), medians / extremes over workgroups. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer, KEY_ENV_BITS  # noqa: E402
from microbench_r2 import make_graph, time_graph  # noqa: E402


def main():
    ops = _native.require()
    tr = ActorCriticTrainer(preset("pong_a2c", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, cuda_graph=False, seed=3))
    tr.step()
    st, env, eng = tr.storage, tr.env, tr.engine
    N = env.num_envs
    b = eng.bufs(N)
    eng.forward(st.obs[0], b, head=False, shift_out=st.obs[1], fc_parts=True)
    _, F2, F3, _ = eng.trunk_w()
    hp0, S0 = eng.last_fc
    fw, fo, fcnt = eng.fused_fc_args(N)

    def step(ffc, stamps=None):
        sn, tn, tgn, ern = env.next_state()
        ops.pong_fused_step(b.h, eng.sWh, eng.bh, b.z, st.actions[0], st.logp[0], st.entropy[0], st.values[0],
                            KEY_ENV_BITS, tr.policy_seed, env.state, env.t, env.tg, env.ep_ret, sn, tn, tgn, ern,
                            env.ep_stats, env.env_ids, st.obs[0], st.obs[1], st.rewards[0], st.dones[0],
                            st.truncated[0], env.seed, env.max_episode_steps, hp0, S0, eng.bfc, eng.sW1, eng.b1,
                            F2, eng.b2, F3, eng.b3, b.y1, b.y2, b.y3, 1.0 / 255.0, st.obs[2], stamps, True,
                            fw if ffc else None, fo if ffc else None, fcnt if ffc else None)
        env.flip()
        if not ffc:
            eng.fc_planes(b)

    out = {}
    for name, ffc in (("step_with_fc_tail_us", True), ("step_then_fc_rollout_us", False)):
        g = make_graph(lambda: step(ffc), 50)
        out[name] = round(min(time_graph(g, 50) for _ in range(5)), 2)
        del g
    for ffc in (True, False):
        sts = torch.zeros(N * 7 * 16, dtype=torch.int64, device="cuda:0")
        step(ffc)
        step(ffc, sts)
        torch.cuda.synchronize()
        x = sts.view(N * 7, 16).double().cpu() * 10e-3
        t0 = float(x[:, 0].min())
        res = {"start_spread": round(float(x[:, 0].max()) - t0, 2),
               "conv3_issued_med": round(float((x[:, 4] - t0).median()), 2),
               "conv3_issued_max": round(float((x[:, 4] - t0).max()), 2)}
        if ffc:
            for slot, nm in ((11, "published"), (12, "wait_passed"), (13, "planes_stored")):
                res[nm + "_med"] = round(float((x[:, slot] - t0).median()), 2)
                res[nm + "_max"] = round(float((x[:, slot] - t0).max()), 2)
                res[nm + "_min"] = round(float((x[:, slot] - t0).min()), 2)
        out["stamps_fc_tail" if ffc else "stamps_plain"] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
