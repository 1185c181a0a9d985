"""Phase timings of the fused MLP rollout kernel (mlp_rollout_kernel) from its s_memrealtime stamps (100 MHz):
per step, the end of each actor layer, of the parallel Gaussian head and of the env step, as seen by wave 0 of
workgroup 0 after each barrier. Median over steps 1..15 of the MuJoCo-shape config (64 envs)."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from actor_critic_algs_on_tensorflow_amd import preset  # noqa: E402
from actor_critic_algs_on_tensorflow_amd.algos.trainer import ActorCriticTrainer, KEY_ENV_BITS  # noqa: E402


def main():
    cfg = preset("mujoco_ppo_dp8", device="cuda:0", outdir=None, quiet=True, stdout_freq=0, save_every=0,
                 cuda_graph=False)
    tr = ActorCriticTrainer(cfg)
    eng, st, env = tr.mlp, tr.storage, tr.env
    stamps = torch.zeros(256, dtype=torch.int64, device="cuda:0")
    out = {"wlds": eng.rollout_weights_in_lds(), "T": st.T, "N": env.num_envs}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.rollout_linear(env, st, KEY_ENV_BITS, tr.policy_seed, stamps=stamps)
        torch.cuda.synchronize()
        out[f"host_ms_{rep}"] = round((time.perf_counter() - t0) * 1e3, 3)
    allst = stamps.cpu().tolist()
    if len(sys.argv) > 1 and sys.argv[1] == "--layers-only":   # diagnostics: actor layers alone in the step loop
        st2 = torch.zeros(256, dtype=torch.int64, device="cuda:0")
        st2[255] = 1
        eng.rollout_linear(env, st, KEY_ENV_BITS, tr.policy_seed, stamps=st2)
        torch.cuda.synchronize()
        a2 = st2.cpu().tolist()
        s2 = [a2[8 * k:8 * k + 8] for k in range(16)]
        out["layers_only_layer_us"] = [round((s2[8][i] - (s2[8][i - 1] if i else s2[7][6])) * 0.01, 2) for i in range(4)]
    s = [allst[8 * k:8 * k + 8] for k in range(16)]
    names = ["layer0", "layer1", "layer2", "layer3", "-", "head", "env"]
    ph = {n: [] for n in names if n != "-"}
    for k in range(1, 16):
        prev = s[k - 1][6]
        for i, n in enumerate(names):
            if n == "-":
                continue
            ph[n].append((s[k][i] - prev) * 10 / 1000.0)   # 10 ns ticks -> us
            prev = s[k][i]
    out["phase_us_median"] = {n: round(sorted(v)[len(v) // 2], 3) for n, v in ph.items()}
    out["step_us_median"] = round(sorted((s[k][6] - s[k - 1][6]) * 0.01 for k in range(1, 16))[7], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
