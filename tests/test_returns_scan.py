"""Chunked associative returns scan (reference Basic_AC/run_AC.py:63-75): the GPU kernel against
the fp64 PyTorch oracles at T in {5, 128, 2048}, fused EV / moments / advantage normalisation, bitwise repeat; and
on the CPU a numpy emulation of the kernel's algorithm (chunk maps -> suffix scan -> replay, prefix-sum window
form) against the same oracles."""
import numpy as np
import pytest
import torch

from actor_critic_algs_on_tensorflow_amd.ops import returns as R


def _rollout(T, N, seed, p_done=0.05, device="cpu"):
    g = torch.Generator().manual_seed(seed)
    r = torch.randn(T, N, generator=g)
    v = torch.randn(T + 1, N, generator=g) * 2.0
    d = (torch.rand(T, N, generator=g) < p_done).to(torch.uint8)
    return r.to(device), v.to(device), d.to(device)


def _emulate(r, v, d, mode, gamma, lam, L, CH):
    """The kernel's algorithm in numpy (fp64), one env column at a time."""
    T, N = r.shape
    K = -(-T // CH)
    out_ret, out_adv = np.zeros((T, N)), np.zeros((T, N))
    gae = mode == "gae"
    window = not gae and L < T
    for n in range(N):
        maps, fts = [], []
        for ch in range(CH):
            t0, t1 = min(ch * K, T), min(ch * K + K, T)
            a, c, ft = 0.0, 1.0, T
            for t in range(t1 - 1, t0 - 1, -1):
                nd = 0.0 if d[t, n] else 1.0
                ft = t if d[t, n] else ft
                x = r[t, n] + gamma * v[t + 1, n] * nd - v[t, n] if gae else r[t, n]
                cc = (gamma * lam if gae else gamma) * nd
                a, c = x + cc * a, cc * c
            maps.append((a, c))
            fts.append(ft)
        init = 0.0 if (gae or window) else v[T, n]
        gz = np.zeros(T + 1)
        for ch in range(CH):   # carry = composition of the later chunks' maps applied to init
            x = init
            for j in range(CH - 1, ch, -1):
                x = maps[j][0] + maps[j][1] * x
            nt = min(fts[ch + 1:], default=T)
            t0, t1 = min(ch * K, T), min(ch * K + K, T)
            for t in range(t1 - 1, t0 - 1, -1):
                nd = 0.0 if d[t, n] else 1.0
                if gae:
                    x = r[t, n] + gamma * v[t + 1, n] * nd - v[t, n] + gamma * lam * nd * x
                    out_adv[t, n], out_ret[t, n] = x, x + v[t, n]
                else:
                    x = r[t, n] + gamma * nd * x
                    gz[t] = x
                    out_ret[t, n], out_adv[t, n] = x, x - v[t, n]
        if window:
            nt = T
            for t in range(T - 1, -1, -1):
                nt = t if d[t, n] else nt
                h = min(t + L, T)
                tg = gz[t]
                if nt >= h:
                    tg += gamma ** (h - t) * (v[h, n] - (gz[h] if h < T else 0.0))
                out_ret[t, n], out_adv[t, n] = tg, tg - v[t, n]
    return out_ret, out_adv


@pytest.mark.parametrize("mode,L,T,CH", [("gae", None, 37, 8), ("nstep", None, 37, 8), ("nstep", 7, 37, 8),
                                         ("nstep", 1, 12, 4), ("nstep", 5, 5, 2), ("gae", None, 5, 2)])
def test_scan_algorithm_emulation_matches_oracle(mode, L, T, CH):
    N = 6
    r, v, d = _rollout(T, N, seed=T + (L or 0), p_done=0.15)
    LL = T if L is None else L
    if mode == "gae":
        ret_o, adv_o = R.gae_ref(r, v, d, 0.97, 0.9)
    else:
        ret_o, adv_o = R.nstep_returns_ref(r, v, d, 0.97, LL)
    ret_e, adv_e = _emulate(r.double().numpy(), v.double().numpy(), d.numpy(), mode, 0.97, 0.9, LL, CH)
    np.testing.assert_allclose(ret_e, ret_o.numpy(), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(adv_e, adv_o.numpy(), rtol=1e-5, atol=1e-5)


def test_returns_scan_cpu_path_matches_oracles():
    r, v, d = _rollout(16, 5, seed=3)
    ev = torch.zeros(1)
    ret, adv, mom = R.returns_scan(r, v, d, "gae", 0.99, 0.95, norm=True, ev_out=ev)
    ret_o, adv_o = R.gae_ref(r, v, d, 0.99, 0.95)
    torch.testing.assert_close(ret, ret_o)
    torch.testing.assert_close(adv, R.normalize_advantages(adv_o))
    assert float(mom[0]) == 80.0
    assert abs(float(mom[1]) - float(adv_o.double().sum())) < 1e-4


CASES = [(5, 32, "nstep", None), (5, 32, "gae", None), (128, 128, "gae", None), (128, 128, "nstep", None),
         (128, 128, "nstep", 30), (2048, 4, "gae", None), (2048, 4, "nstep", None), (2048, 4, "nstep", 64),
         (2048, 1, "nstep", 2047), (100, 300, "gae", None), (64, 8, "nstep", 1)]


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,mode,L", CASES)
def test_returns_scan_gpu_matches_oracle(cuda, T, N, mode, L):
    from actor_critic_algs_on_tensorflow_amd.utils.stats import var_accounted_for_tensor
    r, v, d = _rollout(T, N, seed=T * 7 + N)
    LL = T if L is None else L
    if mode == "gae":
        ret_o, adv_o = R.gae_ref(r, v, d, 0.99, 0.95)
    else:
        ret_o, adv_o = R.nstep_returns_ref(r, v, d, 0.99, LL)
    ws = R.ScanWorkspace(cuda, T, N)
    ev = torch.zeros(1, device=cuda)
    ret, adv, mom = R.returns_scan(r.to(cuda), v.to(cuda), d.to(cuda), mode, 0.99, 0.95, look_ahead=L, norm=False,
                                   ws=ws, ev_out=ev)
    torch.cuda.synchronize()
    torch.testing.assert_close(ret.cpu(), ret_o, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(adv.cpu(), adv_o, rtol=1e-5, atol=1e-4)
    ev_o = float(var_accounted_for_tensor(ret_o.double(), v[:T].double()))
    assert abs(float(ev) - ev_o) < 1e-4
    m = mom.cpu()
    assert float(m[0]) == T * N
    a64, r64, v64 = adv_o.double(), ret_o.double(), v[:T].double()
    ref = [a64.sum(), (a64 * a64).sum(), r64.sum(), (r64 * r64).sum(), v64.sum(), (v64 * v64).sum(), (r64 * v64).sum()]
    for k in range(7):
        assert abs(float(m[1 + k]) - float(ref[k])) < 1e-3 * (1 + abs(float(ref[k]))), k
    # fused normalisation == oracle normalisation; a second launch is bitwise identical (fixed-order reductions,
    # self-cleaning ticket)
    ret2, adv2, _ = R.returns_scan(r.to(cuda), v.to(cuda), d.to(cuda), mode, 0.99, 0.95, look_ahead=L, norm=True,
                                   ws=ws)
    torch.testing.assert_close(adv2.cpu(), R.normalize_advantages(adv_o), rtol=1e-4, atol=1e-4)
    ret3, adv3, _ = R.returns_scan(r.to(cuda), v.to(cuda), d.to(cuda), mode, 0.99, 0.95, look_ahead=L, norm=True,
                                   ws=ws)
    assert torch.equal(adv2, adv3) and torch.equal(ret2, ret3)


@pytest.mark.gpu
def test_normalize_mom_and_ev_multi(cuda):
    from actor_critic_algs_on_tensorflow_amd import _native
    from actor_critic_algs_on_tensorflow_amd.utils.stats import var_accounted_for_tensor
    ops = _native.require()
    r, v, d = _rollout(128, 128, seed=5)
    ws = R.ScanWorkspace(cuda, 128, 128)
    ret, adv, mom = R.returns_scan(r.to(cuda), v.to(cuda), d.to(cuda), "gae", 0.99, 0.95, ws=ws)
    out = torch.empty_like(adv)
    ops.normalize_mom(adv, out, mom, 1e-8)
    torch.testing.assert_close(out.cpu(), R.normalize_advantages(adv.cpu()), rtol=1e-4, atol=1e-4)
    for n in (1000, 16384, 300000):
        x = torch.randn(n, device=cuda)
        y = x * 0.5 + torch.randn(n, device=cuda)
        e1 = torch.zeros(1, device=cuda)
        ops.ev(x, y, e1, ws.ev_part, ws.ev_ticket)
        e2 = torch.zeros(1, device=cuda)
        ops.ev(x, y, e2, ws.ev_part, ws.ev_ticket)
        assert torch.equal(e1, e2)
        assert abs(float(e1) - float(var_accounted_for_tensor(x.double(), y.double()))) < 1e-5
