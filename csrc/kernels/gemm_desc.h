// Plain-C description of one GEMM launch, shared by the HIP launchers and the torch bindings.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// Implicit-im2col operand gather (convolution as GEMM without materialising the column matrix).
//   mode 1: uint8 NCHW source [B, C, H, W], k order (c, i, j), values scaled by `scale` (the /255 of the frames);
//           requires KW % 8 == 0, S % 4 == 0, W % 4 == 0 (8 k = two aligned 4-byte loads)
//   mode 2: bf16 NHWC source [B, H, W, C], k order (i, j, c); requires C % 8 == 0 (8 k = one 16-byte load)
// Row index m = (b, oh, ow) of the conv output, column index k as above.
//   mode 3: transposed conv / data gradient: source = output gradient bf16 NHWC [B, OH, OW, C]; row m = (b, h, w) of
//           the conv INPUT [H, W]; k order (i, j, c); zero where (h - i, w - j) is off the stride grid or outside
//           the output; requires C % 8 == 0
//   mode 4: (B operand) OHWI weight [C][KH][KW][W] read as B[k = (i, j, o)][n]: the transposed-conv weight operand
//           without materialising the transpose; spec fields C = conv output channels, W = input channels
//   mode 5: sub-pixel transposed conv (stride S, KH % S == KW % S == H % S == W % S == 0): the rows are the input
//           pixels grouped by stride phase (ph, pw), m = (((ph * S + pw) * B + b) * H/S + a) * W/S + c for pixel
//           (a*S + ph, c*S + pw), k = (di, dj, o) over (KH/S) x (KW/S) x C: only the taps i = ph + S*di,
//           j = pw + S*dj that land on the stride grid, so K shrinks by S^2 and no zero products are computed;
//           the epilogue writes row m back to its natural NHWC position. Pairs with
//   mode 6: (B operand) OHWI weight read as B[k = (di, dj, o)][n] = W[o][ph + S*di][pw + S*dj][n] for the phase of
//           the workgroup's rows (tiles never straddle phases: (B * H/S * W/S) % BM == 0)
// n / d for 0 <= n < 2^31 as (umulhi(n, m) + n) >> s (Granlund-Montgomery, computed on the host by
// aca_fastdiv_init): the gathers decode their (b, h, w) / (i, j, c) indices without integer division sequences.
typedef struct {
  unsigned int m, s;
} AcaFastDiv;

typedef struct {
  const void* src;
  int mode;  // 0 none, 1 u8 nchw, 2 bf16 nhwc, 3 transposed-conv gather, 4 OHWI weight transpose,
             // 5 sub-pixel transposed conv, 6 phase-selected OHWI weight
  int B, C, H, W, KH, KW, S, OH, OW;
  float scale;
  AcaFastDiv fd_ohw, fd_ow, fd_hw, fd_w, fd_khw, fd_kw, fd_kwc, fd_c, fd_s;
  // modes 5/6 (sub-pixel): HS = H/S, WS = W/S, KHS = KH/S, KWS = KW/S
  int HS, WS, KHS, KWS;
  AcaFastDiv fd_phase, fd_hsws, fd_ws, fd_kwsc, fd_kws;
} AcaConvGather;

static inline AcaFastDiv aca_fastdiv_init(unsigned int d) {
  AcaFastDiv f;
  unsigned int l = 0;
  while (l < 32 && (1ull << l) < d) ++l;   // l = ceil(log2 d)
  f.m = (unsigned int)((((unsigned long long)1 << 32) * (((unsigned long long)1 << l) - d)) / d + 1);
  f.s = l;
  return f;
}

// fills the fast divisors of a gather whose geometry fields are set
static inline void aca_gather_prepare(AcaConvGather* g) {
  g->fd_ohw = aca_fastdiv_init((unsigned int)(g->OH * g->OW > 0 ? g->OH * g->OW : 1));
  g->fd_ow = aca_fastdiv_init((unsigned int)(g->OW > 0 ? g->OW : 1));
  g->fd_hw = aca_fastdiv_init((unsigned int)(g->H * g->W > 0 ? g->H * g->W : 1));
  g->fd_w = aca_fastdiv_init((unsigned int)(g->W > 0 ? g->W : 1));
  g->fd_khw = aca_fastdiv_init((unsigned int)(g->KH * g->KW > 0 ? g->KH * g->KW : 1));
  g->fd_kw = aca_fastdiv_init((unsigned int)(g->KW > 0 ? g->KW : 1));
  g->fd_kwc = aca_fastdiv_init((unsigned int)(g->KW * g->C > 0 ? g->KW * g->C : 1));
  g->fd_c = aca_fastdiv_init((unsigned int)(g->C > 0 ? g->C : 1));
  g->fd_s = aca_fastdiv_init((unsigned int)(g->S > 0 ? g->S : 1));
  if (g->S > 0) {
    g->HS = g->H / g->S; g->WS = g->W / g->S; g->KHS = g->KH / g->S; g->KWS = g->KW / g->S;
    g->fd_phase = aca_fastdiv_init((unsigned int)(g->B * g->HS * g->WS > 0 ? g->B * g->HS * g->WS : 1));
    g->fd_hsws = aca_fastdiv_init((unsigned int)(g->HS * g->WS > 0 ? g->HS * g->WS : 1));
    g->fd_ws = aca_fastdiv_init((unsigned int)(g->WS > 0 ? g->WS : 1));
    g->fd_kwsc = aca_fastdiv_init((unsigned int)(g->KWS * g->C > 0 ? g->KWS * g->C : 1));
    g->fd_kws = aca_fastdiv_init((unsigned int)(g->KWS > 0 ? g->KWS : 1));
  }
}

typedef struct {
  const void* A;
  const void* B;
  void* C;
  const float* bias;
  const void* mask;
  float* colsum;
  float* ws;
  unsigned int* tickets;
  int64_t lda, ldb, ldc, ldm;
  int M, N, K;
  int a_k, b_k;       // operand storage (see gemm_impl.h)
  int out_mode;       // 0 fp32, 1 bf16, 2 fp32 atomic add, 3 fp32 split-K partial planes
  int relu;
  int colsum_mod;
  float alpha;
  int tile;           // 0 64x64, 1 32x64, 2 64x32, 3 128x64, 4 32x32
  int bk;             // 64 | 128 | 256
  int splits;
  AcaConvGather ga;   // gather for A (requires a_k)
  AcaConvGather gb;   // gather for B (requires !b_k): B[k = conv row m][n = conv column k]
  unsigned long long* stamps;   // diagnostics (null in production): per workgroup [start, k-loop, epilogue, end]
  // column sums as per-row-tile partials (plain stores to colsum_part[(m0 / BM) * N + n], no atomics; reduced into
  // colsum by aca_colsum_reduce): thousands of workgroups adding into the same few bias addresses serialise in L2
  float* colsum_part;
} AcaGemmDesc;

#ifdef __cplusplus
}
#endif
