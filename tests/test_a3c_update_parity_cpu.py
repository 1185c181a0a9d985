"""The reference A3C worker update (A3C/process.py:217-278, A3C/policies.py:34-104) in this framework vs an
independent plain-PyTorch oracle (tests/oracles/a3c_oracle.py, written from the reference's equations with no code from
this package), from the same parameters on the same 1200-step Pendulum batch: PathAdv targets, the actor gradient
(policy gradient + beta KL + gamma entropy, value-clipped), TF-Adam parameters, the KL proxy and the adaptive lr."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracles"))


def test_a3c_update_matches_independent_oracle():
    import a3c_update_parity as P
    torch.set_num_threads(2)
    rows = P.run(updates=3, num_envs=3, verbose=False)
    for r in rows:
        assert r["target_max"] < 1e-3, r
        assert r["logp_consistency"] < 1e-5, r
        assert r["grad_rel"] < 1e-4, r
        assert r["param_max"] < 1e-5, r
        assert abs(r["kl"][0] - r["kl"][1]) <= 1e-4 * max(1.0, abs(r["kl"][1])), r
        assert r["lr"][0] == r["lr"][1] or abs(r["lr"][0] - r["lr"][1]) < 1e-9, r
