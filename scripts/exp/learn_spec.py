import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_learning as T
from actor_critic_algs_on_tensorflow_amd.ops import mlp as M
for spec in (False, True):
    orig = M.MLPEngine.__init__
    def init(self, *a, _o=orig, _s=spec, **k):
        _o(self, *a, **k); self.spec = _s
    M.MLPEngine.__init__ = init
    tr, rows = T._curve("mujoco_ppo_dp8", 300, 30, lr=1e-4, critic_lr=1e-3, lr_schedule="linear", total_updates=300)
    M.MLPEngine.__init__ = orig
    rets = [round(r["ret"], 1) for r in rows]
    print("spec", spec, rets, flush=True)
