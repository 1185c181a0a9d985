"""Source-level invariants of the HIP kernels that the compiler does not enforce.

Dynamic LDS (``extern __shared__``) starts right after a kernel's static LDS segment, aligned only to the declared
type: a float array after a 1,720-byte static segment began at 8 mod 16 bytes, and every ``ds_read_b128`` of the
MLP rollout kernel's weights and activations was misaligned (its 128 x 128 layer ran at 8-9 k instead of ~2.5 k
shader cycles; profiles/r2_probe_mfma_f32_rate.txt). Every dynamic LDS array must therefore be declared 16-byte
aligned."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dynamic_lds_arrays_are_16_byte_aligned():
    offenders = []
    for path in glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")) + \
            glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.h")):
        for i, line in enumerate(open(path), 1):
            if re.search(r"extern\s+__shared__", line) and "aligned(16)" not in line:
                offenders.append(f"{os.path.basename(path)}:{i}: {line.strip()}")
    assert not offenders, offenders


def test_no_cuda_compat_layers():
    """CDNA4 code only: no CUDA shims, hipify markers or dual-platform paths in the kernels."""
    bad = []
    for path in glob.glob(os.path.join(ROOT, "csrc", "**", "*.*"), recursive=True):
        if not path.endswith((".hip", ".h", ".cpp")):
            continue
        txt = open(path, errors="ignore").read()
        for pat in ("__HIP_PLATFORM_NVIDIA__", "#include <cuda", "cudaStream_t", "__CUDA_ARCH__"):
            if pat in txt:
                bad.append((os.path.basename(path), pat))
    assert not bad, bad


def test_fused_head_gate_matches_kernel_limits():
    """the Python gate of the fused A2C head (engine.head_ok) applies the same limits as the kernel's
    launcher (loss.hip aca_head_bwd: B <= 512 rows, N <= 256 envs, 2..7 actions), so e.g. n_steps=1 with 300 envs
    takes the loss + GEMM path instead of failing at launch."""
    from actor_critic_algs_on_tensorflow_amd.algos.engine import CNNEngine
    eng = CNNEngine.__new__(CNNEngine)
    eng.fused_head, eng.A = True, 6
    assert eng.head_ok(160, 32)
    assert eng.head_ok(512, 256)
    assert not eng.head_ok(300, 300)     # one step of 300 envs: N > 256
    assert not eng.head_ok(640, 128)     # B > 512
    eng.A = 8
    assert not eng.head_ok(160, 32)
    src = open(os.path.join(ROOT, "csrc", "kernels", "loss.hip")).read()
    assert "B > aca::HB_MAXB || N > 256" in src and "constexpr int HB_MAXB = 512;" in src
