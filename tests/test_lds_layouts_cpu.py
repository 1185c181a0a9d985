"""LDS bank model of the GEMM operand tiles (csrc/kernels/gemm_impl.h), checked on the CPU.

gfx950 LDS: 64 banks of 4 bytes. A wave64 access is served in fixed lane groups, one LDS cycle per group when no two
distinct dwords of the group share a bank (docs: MI355X_MICROARCH.md, LDS table):
  ds_read_b128          4 groups of 16 lanes {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32), bank = dword % 64
  ds_read_b64_tr_b16    2 groups of 32 lanes, bank = dword % 64
  ds_write_b128         8 groups of 8 consecutive lanes, bank = dword % 32
The kernel's layouts: k-contiguous tiles padded by GEMM_PAD_K elements per row, m/n-contiguous tiles unpadded with
the 16-byte chunk index XOR-swizzled by gemm_tr_swz<W>(k row). This test mirrors both in Python, checks that every
fragment read and staging store is conflict-free under the model, and that the header still holds the same
constants and swizzle terms (profiles/r3_gemm_swizzle_ab.txt: SQ_LDS_BANK_CONFLICT 0.0 % on the GPU).
"""
import os
import re

import pytest

HDR = os.path.join(os.path.dirname(__file__), "..", "csrc", "kernels", "gemm_impl.h")

G128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G128 += [[lane + 32 for lane in g] for g in G128]


def cycles(groups, width_dw, nbanks):
    """LDS cycles of one wave instruction: per group, the largest number of distinct dwords on one bank."""
    tot = 0
    for g in groups:
        banks = {}
        for byte_addr in g:
            d0 = byte_addr // 4
            for d in range(width_dw):
                banks.setdefault((d0 + d) % nbanks, set()).add(d0 + d)
        tot += max(len(v) for v in banks.values())
    return tot


def tr_swz(w, row):
    """Python mirror of gemm_tr_swz<W>."""
    if w == 32:
        return ((row >> 3) & 1) << 1
    if w == 64:
        return (((row >> 1) & 1) << 1) ^ (((row >> 3) & 1) << 2)
    return ((row & 1) << 1) ^ (((row >> 1) & 1) << 2) ^ (((row >> 3) & 1) << 3)


def header_consts():
    src = open(HDR).read()
    pad_k = int(re.search(r"constexpr int GEMM_PAD_K = (\d+);", src).group(1))
    pad = int(re.search(r"constexpr int GEMM_PAD = (\d+);", src).group(1))
    return src, pad_k, pad


def test_header_matches_model():
    src, pad_k, pad = header_consts()
    assert pad_k == 16 and pad == 0
    body = src[src.index("__device__ __forceinline__ int gemm_tr_swz"):]
    body = body[:body.index("\n}\n")]
    for term in ("if constexpr (W == 32) return ((row >> 3) & 1) << 1;",
                 "(((row >> 1) & 1) << 1) ^ (((row >> 3) & 1) << 2)",
                 "((row & 1) << 1) ^ (((row >> 1) & 1) << 2) ^ (((row >> 3) & 1) << 3)"):
        assert term in body, term


@pytest.mark.parametrize("bk", [64, 128, 256])
def test_k_contiguous_fragment_reads_conflict_free(bk):
    _, pad_k, _ = header_consts()
    ld = bk + pad_k
    for ks in range(bk // 32):
        for rowbase in (0, 16):
            # frag(): lane (lr16, lg) reads 16 bytes at row rowbase + lr16, k = ks*32 + lg*8
            addrs = [2 * ((rowbase + (lane & 15)) * ld + ks * 32 + (lane >> 4) * 8) for lane in range(64)]
            assert cycles([[addrs[lane] for lane in g] for g in G128], 4, 64) == 4


@pytest.mark.parametrize("w", [32, 64, 128, 256])
@pytest.mark.parametrize("bk", [64, 128])
def test_transposed_tiles_conflict_free(w, bk):
    _, _, pad = header_consts()
    ld = w + pad

    def phys(k, col):
        return 2 * (k * ld + (((col >> 3) ^ tr_swz(w, k)) << 3) + (col & 7))

    for ks in range(bk // 32):
        for rowbase in range(0, w, 16):
            groups = []
            for half in range(2):
                g = []
                for lane in range(32 * half, 32 * half + 32):
                    lr16, lg = lane & 15, lane >> 4
                    q, p = lr16 >> 2, lr16 & 3
                    g.append(phys(ks * 32 + lg * 8 + q, rowbase + 4 * p))
                groups.append(g)
            assert cycles(groups, 2, 64) == 2
    # 16-byte staging stores: thread ch -> k row ch / (W/8), chunk ch % (W/8)
    per_row = w // 8
    for base in range(0, bk * per_row, 64):
        groups = [[phys((base + g8 * 8 + i) // per_row, ((base + g8 * 8 + i) % per_row) * 8) for i in range(8)]
                  for g8 in range(8)]
        assert cycles(groups, 4, 32) == 8
    # the swizzle is a permutation of each row's chunks (no two columns share a slot)
    for k in range(bk):
        assert sorted(c ^ tr_swz(w, k) for c in range(per_row)) == list(range(per_row))


# ---------------------------------------------------------------------------------------------- trunk backward
CNN = os.path.join(os.path.dirname(__file__), "..", "csrc", "kernels", "cnn_fused.hip")
GTR = [list(range(32)), list(range(32, 64))]


def _bw_consts():
    src = open(CNN).read()
    c = {k: int(re.search(r"\b%s = (\d+)" % k, src).group(1)) for k in
         ("BW_LDW3", "BW_LDW2", "BW_PS", "BW_P3W", "BW_P2W")}
    assert "(((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2)" in src and "return ((r >> 3) & 1) << 1;" in src
    return c


def test_trunk_bwd_image_reads_are_conflict_free():
    """cnn_trunk_bwd(_persist): the A fragments of dy2 (dy3 image, 9-wide output) and dy1 (dy2 image, 10-wide
    sub-pixel classes) read at one LDS cycle per lane group under the model."""
    c = _bw_consts()
    ps = c["BW_PS"] * 2   # bytes per pixel
    for wid in range(8):
        mh = (wid >> 2) * 3
        for ks in range(18):
            for mt in range(3):
                addr = []
                for lane in range(64):
                    l16, lg = lane & 15, lane >> 4
                    kb = ks * 32 + lg * 8
                    t, o0 = kb >> 6, kb & 63
                    ti, tj = t // 3, t % 3
                    m = min((mh + mt) * 16 + l16, 80)
                    a, cc = m // 9, m % 9
                    addr.append(((a - ti + 2) * c["BW_P3W"] + (cc - tj + 2)) * ps + o0 * 2)
                assert cycles([[addr[l] for l in g] for g in G128], 4, 64) == 4, (wid, ks, mt)
    for ks in range(8):
        d = ks >> 1
        di, dj, ob = d >> 1, d & 1, (ks & 1) * 32
        for i in range(7):
            addr = []
            for lane in range(64):
                l16, lg = lane & 15, lane >> 4
                u = min(i * 16 + l16, 99)
                yy, xx = u // 10, u % 10
                addr.append(((yy - di + 1) * c["BW_P2W"] + (xx - dj + 1)) * ps + (ob + lg * 8) * 2)
            assert cycles([[addr[l] for l in g] for g in G128], 4, 64) == 4, (ks, i)


def test_trunk_bwd_weight_reads_are_conflict_free():
    """W3 / W2 B rows, unpadded with XOR-swizzled 16-byte chunks: every ds_read_b64_tr_b16 of tr_frag_sw at one
    LDS cycle per 32-lane group."""
    c = _bw_consts()
    sw3 = lambda r: (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2)
    sw2 = lambda r: ((r >> 3) & 1) << 1
    for ld, sw, col0s, row0s in ((c["BW_LDW3"], sw3, (0, 16, 32, 48), [ks * 32 for ks in range(18)]),
                                 (c["BW_LDW2"], sw2, (0, 16), [t * 64 + ob for t in range(16) for ob in (0, 32)])):
        for col0 in col0s:
            for row0 in row0s:
                for half in (0, 4):
                    addr = []
                    for lane in range(64):
                        lr16, lg = lane & 15, lane >> 4
                        q, p = lr16 >> 2, lr16 & 3
                        r, col = row0 + lg * 8 + half + q, col0 + 4 * p
                        addr.append((r * ld + (((col >> 3) ^ sw(r)) << 3) + (col & 7)) * 2)
                    assert cycles([[addr[l] for l in g] for g in GTR], 2, 64) == 2, (ld, col0, row0, half)


def test_per_env_trunk_forward_reads_are_conflict_free():
    """trunk_env_convs (per-env trunk forward and the fused rollout step): the conv2 A fragments over the y1 image
    (pixel stride Y1_LD, row pitch E1_W) and the conv3 ones over the y2 image (Y2_LD, E2_W) at one LDS cycle per
    lane group."""
    src = open(CNN).read()
    y1_ld, y2_ld = (int(v) for v in re.search(r"constexpr int Y1_LD = (\d+), Y2_LD = (\d+);", src).groups())
    e1_w, e2_w = (int(v) for v in re.search(r"constexpr int E1_W = (\d+), E2_W = (\d+);", src).groups())
    a = src.index("void trunk_env_convs(")
    body = src[a:src.index("\n}\n", a)]
    assert "((oh * 2 + i) * E1_W + ow * 2 + j) * Y1_LD + c0" in body and "((oh + i) * E2_W + ow + j) * Y2_LD + c0" in body
    for ks in range(16):
        for mt in range(6):
            addr = []
            for lane in range(64):
                l16, lg = lane & 15, lane >> 4
                k = ks * 32 + lg * 8
                i, j, c0 = k >> 7, (k >> 5) & 3, k & 31
                m = min(mt * 16 + l16, 80)
                oh, ow = m // 9, m % 9
                addr.append((((oh * 2 + i) * e1_w + ow * 2 + j) * y1_ld + c0) * 2)
            assert cycles([[addr[l] for l in g] for g in G128], 4, 64) == 4, ("conv2", ks, mt)
    for ks in range(18):
        for mt in range(4):
            addr = []
            for lane in range(64):
                l16, lg = lane & 15, lane >> 4
                k = ks * 32 + lg * 8
                i, j, c0 = k // 192, (k >> 6) % 3, k & 63
                m = min(mt * 16 + l16, 48)
                oh, ow = m // 7, m % 7
                addr.append((((oh + i) * e2_w + ow + j) * y2_ld + c0) * 2)
            assert cycles([[addr[l] for l in g] for g in G128], 4, 64) == 4, ("conv3", ks, mt)


def test_w1_lds_image_is_a_permutation_and_fragment_reads_are_conflict_free():
    """w1_lds_dma / w1_frags_from_lds (cnn_fused.hip, the fused rollout step): W1's 16-byte chunks land XOR-swizzled
    by (row & 15) -- every chunk exactly once -- and the conv1 fragment reads (16 rows at one column per lane group)
    take one LDS cycle per group."""
    src = open(CNN).read()
    assert "lc = (q & 31) ^ (row & 15);" in src and "pc = (ks * 4 + lg) ^ (row & 15);" in src
    placed = {}
    for q in range(1024):                 # LDS chunk q <- source chunk row * 32 + lc
        row, lc = q >> 5, (q & 31) ^ ((q >> 5) & 15)
        placed[row * 32 + lc] = q
    assert sorted(placed) == list(range(1024))
    for nt in range(2):
        for ks in range(8):
            addr = []
            for lane in range(64):
                l16, lg = lane & 15, lane >> 4
                row = nt * 16 + l16
                pc = (ks * 4 + lg) ^ (row & 15)
                assert placed[row * 32 + ks * 4 + lg] == row * 32 + pc
                addr.append((row * 256 + pc * 8) * 2)
            assert cycles([[addr[l] for l in g] for g in G128], 4, 64) == 4, (nt, ks)


def test_fast_divisions_are_exact_over_their_ranges():
    """cnn_fused.hip div9 / div10 / div7 (multiply-shift) == integer division over the ranges the kernels use."""
    src = open(CNN).read()
    for name, d, lim in (("div9", 9, 200), ("div10", 10, 1029), ("div7", 7, 64)):
        m = re.search(name + r"\(int n\) \{ return \(int\)\(\(\(unsigned\)n \* (\d+)u\) >> (\d+)\); \}", src)
        mul, sh = int(m.group(1)), int(m.group(2))
        assert all((n * mul) >> sh == n // d for n in range(lim)), name


def _wgrad_src():
    return open(os.path.join(os.path.dirname(__file__), "..", "csrc", "kernels", "conv_wgrad.hip")).read()


@pytest.mark.parametrize("geom", [(20, 20, 32, 4, 2, 9, 9, 2), (9, 9, 64, 3, 1, 7, 7, 2)])
def test_conv_wgrad_gemm_dy_reads_are_conflict_free_and_image_reads_bounded(geom):
    """conv_wgrad_gemm: the dy A fragments (192-byte rows) at one cycle per 32-lane group; the implicit-im2col B
    fragments within 1.35x of ideal (only reads whose 4 positions wrap an output row conflict; 1.9x before)."""
    H, W, C, KS, S, OH, OW, SB = geom
    src = _wgrad_src()
    assert "constexpr int LDI = S == 2 ? C + 16 : C + 32, LDD = 96, IMG_E = H * W * LDI;" in src
    LDI, LDD = (C + 16 if S == 2 else C + 32), 96
    NPOS, NCOL = OH * OW, KS * KS * C
    GP = SB * NPOS
    KST = (GP + 15) // 16
    IMG_E = H * W * LDI

    def pos_off(pk):
        if pk >= GP:
            return SB * IMG_E
        sm, pp = pk // NPOS, pk % NPOS
        oy, ox = pp // OW, pp % OW
        return sm * IMG_E + (S * oy * W + S * ox) * LDI
    tot = n = 0
    for ks in range(KST):
        for mt in range(2):
            for hi in (0, 4):
                addr = []
                for lane in range(64):
                    gl, q, p4 = lane >> 4, (lane >> 2) & 3, lane & 3
                    addr.append(((ks * 16 + 8 * (gl >> 1) + hi + q) * LDD + mt * 32 + (gl & 1) * 16 + 4 * p4) * 2)
                assert cycles([[addr[x] for x in g] for g in GTR], 2, 64) == 2, ("dy", ks, mt, hi)
        for nt in range(NCOL // 32):
            for hi in (0, 4):
                addr = []
                for lane in range(64):
                    gl, q, p4 = lane >> 4, (lane >> 2) & 3, lane & 3
                    n0 = nt * 32 + (gl & 1) * 16 + 4 * p4
                    kyx, c0 = n0 // C, n0 % C
                    ky, kx = kyx // KS, kyx % KS
                    po = pos_off(ks * 16 + 8 * (gl >> 1) + hi + q)
                    addr.append((po if po == SB * IMG_E else po + (ky * W + kx) * LDI + c0) * 2)
                tot += cycles([[addr[x] for x in g] for g in GTR], 2, 64)
                n += 1
    assert tot / n / 2 < 1.35
