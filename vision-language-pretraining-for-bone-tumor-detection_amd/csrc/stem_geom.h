// Geometry of the single-channel stem's input layout (shared by conv_ops.hip's
// K = 64 stem GEMMs and stem_ops.hip's fused stem + max-pool kernels).
//
// conv(x replicated to 3 channels, w) = conv(x, w1) with w1 = sum_c w[:, c]: a
// K = (kh:8, kw:8) = 64 GEMM.  A 16-B chunk (8 bf16 / 4 fp32) is 8 (4)
// consecutive kw of one kh; to keep every chunk 16-B aligned the zero-padded
// image is stored in 4 copies shifted by 0, 2, 4, 6 pixels: output column wo
// reads copy s = wo & 3 at column 2wo - 2s (a multiple of 8).
// Xs[s][n][Hp][Wp1], Wp1 = round8(2Wo + 8), zero outside the image.
#pragma once
#include "common.h"

namespace vlp {

struct Stem1Geom {
  int N, Ho, Wo, Hp, Wp1, M;
  size_t copy;   // elements per shifted copy
  FastDiv fd_howo, fd_wo;
};

static inline Stem1Geom make_stem1(int N, int H, int W) {
  Stem1Geom g;
  g.N = N;
  g.Ho = (H + 6 - 7) / 2 + 1;
  g.Wo = (W + 6 - 7) / 2 + 1;
  g.Hp = 2 * g.Ho + 6;
  g.Wp1 = (2 * g.Wo + 8 + 7) / 8 * 8;
  g.M = N * g.Ho * g.Wo;
  g.copy = (size_t)N * g.Hp * g.Wp1;
  g.fd_howo = make_fastdiv(g.Ho * g.Wo);
  g.fd_wo = make_fastdiv(g.Wo);
  return g;
}

// element offset of output pixel (n, ho, wo)'s patch row kh = 0 (Xs copy wo & 3)
__device__ __forceinline__ size_t stem1_pix(const Stem1Geom& g, int n, int ho, int wo) {
  const int sh = wo & 3;
  return (size_t)sh * g.copy + ((size_t)n * g.Hp + 2 * ho) * g.Wp1 + 2 * wo - 2 * sh;
}

}  // namespace vlp
