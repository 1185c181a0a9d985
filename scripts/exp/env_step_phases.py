"""Phase stamps of the per-env fused rollout step (cnn_fused.hip pong_fused_env_step_kernel) at the Breakout-shape
bank (128 envs), split (two workgroups per env) and whole-env forms: event-timed launches plus per-workgroup
s_memrealtime stamps, medians over workgroups (per half for the split form); conv2 / conv3 weights fragment-ordered
(EngineOpts.frag_weights) or row-major. GPU only."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch  # noqa: E402

from actor_critic_algs_on_tensorflow_amd import _native, preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer, KEY_ENV_BITS  # noqa: E402

NAMES = ["loads landed (DMA, fragments, fc planes) + barrier", "sampling + barrier", "commit + render + barrier",
         "shift copy", "conv1 + W3 frags + barrier", "conv2 + barrier", "conv3 + stores"]


def main():
    ops = _native.require()
    tr = ActorCriticTrainer(preset("breakout_ppo", device="cuda:0", outdir=None, quiet=True, stdout_freq=0,
                                   save_every=0, cuda_graph=False, seed=3))
    tr.step()
    st, env, eng = tr.storage, tr.env, tr.engine
    N = env.num_envs
    b = eng.bufs(N)
    eng.forward(st.obs[0], b, head=False, shift_out=st.obs[1], fc_parts=True)
    out = {}
    _, F2, F3, _ = eng.trunk_w()
    for split, frag in ((True, True), (True, False), (False, True)):
        if frag and eng.frag is None:
            continue
        W2, W3 = (F2, F3) if frag else (eng.sW2, eng.sW3)

        def launch(stamps=None):
            hp, S = eng.last_fc
            ops.pong_fused_env_step(b.h, eng.sWh, eng.bh, b.z, st.actions[0], st.logp[0], st.entropy[0],
                                    st.values[0], KEY_ENV_BITS, tr.policy_seed, env.state, env.t, env.tg,
                                    env.ep_ret, env.ep_stats, env.env_ids, st.obs[1], st.rewards[0], st.dones[0],
                                    st.truncated[0], env.seed, env.max_episode_steps, hp, S, eng.bfc, eng.sW1,
                                    eng.b1, W2, eng.b2, W3, eng.b3, b.y1, b.y2, b.y3, 1.0 / 255.0,
                                    st.obs[2], list(env.next_state()) if split else None, stamps, frag)
            if split:
                env.flip()
        for _ in range(5):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            launch()
        e1.record()
        torch.cuda.synchronize()
        nb = 2 * N if split else N
        sts = torch.zeros(nb * 16, dtype=torch.int64, device="cuda:0")
        launch(sts)
        torch.cuda.synchronize()
        x = sts.view(nb, 16).double().cpu() * 10e-3   # 100 MHz -> us
        res = {"launch_us (50 back to back)": round(e0.elapsed_time(e1) * 1e3 / 50, 2)}
        parts = [("half0", x[0::2]), ("half1", x[1::2])] if split else [("whole", x)]
        for name, y in parts:
            ph = {n: round(float((y[:, k + 1] - y[:, k]).median()), 2) for k, n in enumerate(NAMES)}
            ph["total (first stamp .. last)"] = round(float((y[:, 7] - y[:, 0]).median()), 2)
            ph["  start -> fc planes summed (wave 0)"] = round(float((y[:, 8] - y[:, 0]).median()), 2)
            ph["  start -> head partials written (wave 0)"] = round(float((y[:, 9] - y[:, 0]).median()), 2)
            ph["  start -> physics candidates (wave 1)"] = round(float((y[:, 10] - y[:, 0]).median()), 2)
            res[name] = ph
        res["start spread us"] = round(float(x[:, 0].max() - x[:, 0].min()), 2)
        res["end spread us (last - first end)"] = round(float(x[:, 7].max() - x[:, 7].min()), 2)
        out[("split" if split else "whole") + ("_frag" if frag else "_rowmajor")] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
