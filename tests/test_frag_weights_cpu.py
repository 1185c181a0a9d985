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



def test_kc_fragment_layout_matches_the_mfma_b_operand_and_the_optimiser_wave_items():
    """Wfc's k-contiguous copy (frag_order_kc, fc_rollout.hip): fragment (kb, nb) lane l holds the 8 consecutive k of
    column nb * 32 + (l & 31) starting at kb * 16 + 8 (l >> 5) -- the 32x32x16 MFMA B operand; the optimiser's wave
    item (k octet kq, column block nb) writes the 512-byte run at ((kq / 2) * NB + nb) * 512 + (kq % 2) * 256 from
    its LDS image [32 columns][8 k] (optim.hip opt_body)."""
    from actor_critic_algs_on_tensorflow_amd.ops.optim import frag_order_kc
    K, N = 64, 96
    NB = N // 32
    W = torch.arange(K * N, dtype=torch.int64).view(K, N)
    F = W.reshape(K // 16, 2, 8, NB, 32).permute(0, 3, 1, 4, 2).reshape(-1)
    for kb in range(K // 16):
        for nb in range(NB):
            for lane in (0, 7, 31, 32, 50, 63):
                o = ((kb * NB + nb) * 64 + lane) * 8
                k0, col = kb * 16 + 8 * (lane >> 5), nb * 32 + (lane & 31)
                assert torch.equal(F[o:o + 8], W[k0:k0 + 8, col])
    for kq in range(K // 8):
        for nb in range(NB):
            img = W[kq * 8:kq * 8 + 8, nb * 32:nb * 32 + 32].t().reshape(-1)   # [32 columns][8 k]
            base = ((kq // 2) * NB + nb) * 512 + (kq % 2) * 256
            assert torch.equal(F[base:base + 256], img)
    Wf = torch.randn(K, N)
    assert torch.equal(frag_order_kc(Wf, K, N), Wf.reshape(-1)[F].to(torch.bfloat16))


def test_torch_optimiser_path_rewrites_the_kc_copy():
    from actor_critic_algs_on_tensorflow_amd.ops.optim import FlatParams, FusedRMSprop, frag_order_kc
    Wc = torch.nn.Parameter(torch.randn(64, 512))
    Wk = torch.nn.Parameter(torch.randn(128, 64))
    flat = FlatParams({"shared": [Wc, Wk]})
    opt = FusedRMSprop(flat, "shared", lr=1e-2)
    Fc = torch.empty(64 * 512, dtype=torch.bfloat16)
    Fk = torch.empty(128 * 64, dtype=torch.bfloat16)
    vc = flat.data[flat.offsets[0]:flat.offsets[0] + Wc.numel()]
    vk = flat.data[flat.offsets[1]:flat.offsets[1] + Wk.numel()]
    opt.set_frag([(vc, 64, 512, Fc), (vk, 128, 64, Fk, -2)])
    assert opt._frag_table[1, 3] == -2
    flat.grad.normal_()
    opt.step()
    assert torch.equal(Fc, frag_order(vc, 64, 512)) and torch.equal(Fk, frag_order_kc(vk, 128, 64))
