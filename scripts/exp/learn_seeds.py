"""MuJoCo-shape PPO learning curves (the test_gpu_learning no-decay setting: actor 1e-4, critic 1e-3, linear decay,
300 updates) on several seeds: per seed the returns every 30 updates, peak, last-third mean and their ratio."""
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_learning as T  # noqa: E402

seeds = [int(s) for s in (sys.argv[1:] or ["1", "2", "3", "4"])]
for seed in seeds:
    tr, rows = T._curve("mujoco_ppo_dp8", 300, 30, lr=1e-4, critic_lr=1e-3, lr_schedule="linear", total_updates=300,
                        seed=seed)
    rets = [round(r["ret"], 1) for r in rows]
    peak, last = max(rets), sum(rets[-3:]) / 3
    print(f"seed {seed}: {rets} peak {peak} last-third {last:.1f} ratio {last / peak:.3f}", flush=True)
