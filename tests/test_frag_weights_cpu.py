"""Fragment-ordered conv weight copies (EngineOpts.frag_weights), host side: the torch permutation
(ops/optim.py frag_order), the optimiser kernel's per-element index (optim.hip write_trans, ldt < 0) and the
kernels' per-lane fragment reads (cnn_fused.hip frag_w1..3) all describe the same layout, and the torch optimiser
path keeps the copies current."""
import numpy as np
import torch

from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order


def _elem_index(k, c, N):
    # optim.hip write_trans: element (k, c) of a row-major [K][N] weight
    return ((((k >> 4) * (N >> 5) + (c >> 5)) * 64 + ((c >> 3) & 3) * 16 + (k & 15)) * 8 + (c & 7))


def test_frag_order_matches_the_optimiser_element_index():
    for K, N in ((32, 256), (64, 512), (64, 576)):
        W = torch.arange(K * N, dtype=torch.float32).view(K, N)
        F = frag_order(W.double(), K, N).double()   # bf16 is exact only below 256: compare positions instead
        k, c = np.meshgrid(np.arange(K), np.arange(N), indexing="ij")
        idx = _elem_index(k, c, N)
        assert sorted(idx.reshape(-1).tolist()) == list(range(K * N))   # a permutation
        src = torch.arange(K * N, dtype=torch.int64).view(K, N)
        perm = src.reshape(K // 16, 16, N // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1)
        inv = torch.empty_like(perm)
        inv[perm] = torch.arange(K * N)
        assert torch.equal(inv.view(K, N), torch.from_numpy(idx).long())
        assert F.numel() == K * N


def test_frag_order_matches_the_kernel_fragment_reads():
    # frag_w2 / frag_w3: wave wid, k-step ks, lane l reads 8 elements at ((wid * KS + ks) * 64 + l) * 8, which must be
    # the MFMA B fragment of output channel wid * 16 + (l & 15), k = ks * 32 + (l >> 4) * 8 .. + 8
    for K, N in ((32, 256), (64, 512), (64, 576)):
        W = torch.arange(K * N, dtype=torch.int64).view(K, N)
        F = W.reshape(K // 16, 16, N // 32, 4, 8).permute(0, 2, 3, 1, 4).reshape(-1)
        KS = N // 32
        for tile in range(K // 16):
            for ks in range(KS):
                for lane in (0, 5, 16, 31, 47, 63):
                    o = ((tile * KS + ks) * 64 + lane) * 8
                    row, col = tile * 16 + (lane & 15), ks * 32 + (lane >> 4) * 8
                    assert torch.equal(F[o:o + 8], W[row, col:col + 8])


def test_torch_optimiser_path_rewrites_the_copies():
    from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams, FusedAdam, FusedRMSprop
    for cls in (FusedAdam, FusedRMSprop):
        W = torch.nn.Parameter(torch.randn(64, 512))
        flat = FlatParams({"shared": [W]})
        opt = cls(flat, "shared", lr=1e-2)
        F = torch.empty(64 * 512, dtype=torch.bfloat16)
        view = flat.data[flat.offsets[0]:flat.offsets[0] + W.numel()]
        opt.set_frag([(view, 64, 512, F)])
        flat.grad.normal_()
        opt.step()
        assert torch.equal(F, frag_order(view, 64, 512))

