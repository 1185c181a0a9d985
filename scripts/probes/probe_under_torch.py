"""Runs the MFMA probe (scripts/probes/mfma_f32_rate.hip built as a shared library) inside a process that has
initialised PyTorch's HIP context and launched kernels on its stream, to compare with the standalone binary."""
import ctypes
import sys

import torch

x = torch.randn(1024, 1024, device="cuda:0")
(x @ x).sum().item()
lib = ctypes.CDLL(sys.argv[1])
sys.stdout.flush()
lib.run_probe()
