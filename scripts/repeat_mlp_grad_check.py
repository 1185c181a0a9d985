"""Repeats the MLP train-kernel gradient check (tests/test_gpu_mlp.py test_mlp_train_gradients_match_autograd, PPO,
case 0) N times in one process and counts mismatches: a race shows up as an occasional large mismatch."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import test_gpu_mlp as T  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    bad = 0
    for i in range(n):
        try:
            T.test_mlp_train_gradients_match_autograd(torch.device("cuda:0"), T.CASES[0], True)
        except AssertionError as e:
            bad += 1
            print("mismatch", i, str(e).splitlines()[0][:160], flush=True)
    print(f"{bad} / {n} mismatched", flush=True)


if __name__ == "__main__":
    main()
