"""Counter-based RNG shared bit-for-bit by the PyTorch env oracles and the HIP env-bank kernels.

``hash_u32(seed, env, step, stream)`` mixes four 32-bit words with the lowbias32 finaliser (two rounds); it is
stateless, so every env / step / draw gets an independent stream and the result does not depend on how envs
are partitioned across GPUs or ranks. ``csrc/kernels/env_common.h`` implements the
identical function; ``tests/test_envs.py`` pins a few values so the two never drift apart.
"""
from __future__ import annotations

import torch

M32 = 0xFFFFFFFF
C1 = 0x7FEB352D
C2 = 0x846CA68B
GOLD = 0x9E3779B9


def _mix(x):
    x = x & M32
    x = x ^ (x >> 16)
    x = (x * C1) & M32
    x = x ^ (x >> 15)
    x = (x * C2) & M32
    x = x ^ (x >> 16)
    return x


def hash_u32(seed, env, step, stream):
    """All args int64 tensors (or ints) holding values < 2**32; returns an int64 tensor in [0, 2**32)."""
    h = _mix(torch.as_tensor(seed, dtype=torch.int64) ^ GOLD)
    h = _mix(h ^ (torch.as_tensor(env, dtype=torch.int64) & M32))
    h = _mix(h ^ ((torch.as_tensor(step, dtype=torch.int64) * 0x27D4EB2F) & M32))
    h = _mix(h ^ ((torch.as_tensor(stream, dtype=torch.int64) * 0x165667B1) & M32))
    return h


def uniform(seed, env, step, stream):
    """Uniform float32 in [0, 1) with 24 random bits (exact in fp32 on both CPU and GPU)."""
    return (hash_u32(seed, env, step, stream) >> 8).to(torch.float32) * (1.0 / 16777216.0)


_PRP_MULTS = (0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D)


def minibatch_key(seed, update_counter, epoch):
    """Key of the PPO minibatch permutation of ``epoch`` in update ``update_counter`` (a tensor, so the key is
    derived on the device inside a captured graph). Identical to ``minibatch_key`` in csrc/kernels/common.h."""
    uc = torch.as_tensor(update_counter, dtype=torch.int64)
    return hash_u32(seed, (uc * 64 + epoch) & M32, 7, 11)


def prp(i, n, key):
    """Keyed pseudo-random permutation of ``[0, n)`` applied to the int64 tensor ``i`` (values < n): three rounds of
    xor-key / odd multiply / xorshift, each a bijection of the k-bit domain (k = ceil(log2 n)), with cycle walking
    back into ``[0, n)``. Bit-identical to ``prp_index`` in csrc/kernels/common.h."""
    k = 1
    while k < 32 and (1 << k) < n:
        k += 1
    mask = (1 << k) - 1
    sh = (k + 1) >> 1
    key = torch.as_tensor(key, dtype=torch.int64)
    cs = [hash_u32(key, r, 0x5BD1, 3) & mask for r in range(3)]

    def rounds(x):
        for c, m in zip(cs, _PRP_MULTS):
            x = ((x ^ c) * m) & mask
            x = x ^ (x >> sh)
        return x

    x = rounds(torch.as_tensor(i, dtype=torch.int64))
    while bool((x >= n).any()):
        x = torch.where(x >= n, rounds(x), x)
    return x


def hash_u32_py(seed, env, step, stream):
    """Pure-Python reference (used to pin test vectors)."""
    def mix(x):
        x &= M32
        x ^= x >> 16
        x = (x * C1) & M32
        x ^= x >> 15
        x = (x * C2) & M32
        x ^= x >> 16
        return x
    h = mix(seed ^ GOLD)
    h = mix(h ^ (env & M32))
    h = mix(h ^ ((step * 0x27D4EB2F) & M32))
    h = mix(h ^ ((stream * 0x165667B1) & M32))
    return h
