// Implicit-GEMM convolutions for the ResNet34 image tower (timm `resnet34`,
// called from the reference at src/models/pretrain/VisionLanguageModule.py:30-35).
//
// Layout: activations NHWC (channels innermost), weights packed per step from
// the fp32 master tensors (timm [Co][C][KH][KW]) into
//   Wp[Co][KH][KW][C]  (forward operand, K-contiguous)
//   Wt[C][KH][KW][Co]  (data-gradient operand, K-contiguous)
// so every operand streams as 16-byte chunks along the channel dimension.
//
//   fwd   : y[m=(n,ho,wo)][co]  = sum_{kh,kw,ci} x[n][ho*S-P+kh][wo*S-P+kw][ci] Wp[co][kh][kw][ci]
//   dgrad : dx[m=(n,h,w)][ci]   = sum_{kh,kw,co} dy[n][(h+P-kh)/S][(w+P-kw)/S][co] Wt[ci][kh][kw][co]
//   wgrad : dW[co][(kh,kw,ci)]  = sum_{m} dy[m][co] * x_patch[m][(kh,kw,ci)]     (split-K over m)
//
// Fusions: the forward epilogue accumulates train-mode BatchNorm batch
// statistics (sum, sum of squares per channel, fp64 atomics); the forward and
// weight-gradient loaders can apply the previous layer's BN+ReLU on load, so
// the post-activation tensor is never materialised; the data-gradient epilogue
// can apply the ReLU mask of the producer layer and accumulate that BN's
// backward statistics, or add a residual-branch gradient.
#include "gemm.h"
#include "stem_geom.h"

namespace vlp {

struct ConvGeom {
  int N, H, W, C, Co, KH, KW, S, P, Ho, Wo;
  int M;      // rows of the GEMM
  int K;      // reduction length
  FastDiv fd_howo, fd_wo, fd_hw, fd_w, fd_c, fd_co, fd_kw;
};

static ConvGeom make_geom(int N, int H, int W, int C, int Co, int KH, int KW, int S, int P) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Co = Co; g.KH = KH; g.KW = KW; g.S = S; g.P = P;
  g.Ho = (H + 2 * P - KH) / S + 1;
  g.Wo = (W + 2 * P - KW) / S + 1;
  g.M = 0; g.K = 0;
  g.fd_howo = make_fastdiv(g.Ho * g.Wo);
  g.fd_wo = make_fastdiv(g.Wo);
  g.fd_hw = make_fastdiv(H * W);
  g.fd_w = make_fastdiv(W);
  g.fd_c = make_fastdiv(C);
  g.fd_co = make_fastdiv(Co);
  g.fd_kw = make_fastdiv(KW);
  return g;
}

// Optional per-channel affine + ReLU applied to a loaded chunk (BN-apply on load).
template <typename T>
__device__ __forceinline__ uint4 xform_chunk(uint4 v, const float* sc, const float* sh, int c) {
  constexpr int E = Chunk<T>::N;
  float f[E];
  Chunk<T>::unpack(v, f);
#pragma unroll
  for (int j = 0; j < E; ++j) f[j] = fmaxf(fmaf(f[j], sc[c + j], sh[c + j]), 0.f);
  return Chunk<T>::pack(f);
}

// Loaders carry two protocols (gemm.h): fixed/load (register staging: fp32
// parity mode, BN-on-load) and start/next (incremental direct-to-LDS, bf16).
// The direct path requires the channel count to be a multiple of the K-step
// (64), so a K-step never straddles a filter tap and (kh, kw, channel offset)
// are wave-uniform scalars; every ResNet34 conv except the stem satisfies it
// (the stem has its own loaders).

// K-step order of the bf16 buffer-protocol convolutions (VLP_KPERM = 1):
// channel chunk major, filter tap minor -- the 9 taps of one 64-channel chunk
// are consecutive K-steps, so a tile's shifted re-reads of the same input rows
// follow each other and hit L2 (tap-major order re-read them every C/64 steps,
// and 32 tiles x C/64 steps x 32 KB per XCD overflowed its 4 MB L2)
#ifndef VLP_KPERM
#define VLP_KPERM 1
#endif
__device__ __forceinline__ int conv_kperm(int k, int K, int taps, int nch) {
  if (k >= K) return k;
  const int s = k >> 6;
  const int chunk = s / taps, tap = s - chunk * taps;
  return (tap * nch + chunk) << 6;
}

// ---- forward A operand: input patches, K-contiguous ----
template <typename T, bool XF>
struct ConvFwdA {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = !XF;
  static constexpr bool kKPerm = VLP_KPERM && std::is_same<T, bf16>::value && !XF;
  __device__ int kperm(int k) const {
    return g.C % 64 ? k : conv_kperm(k, g.K, g.KH * g.KW, g.C >> 6);
  }
  struct State { const T* base; int hi0, wi0; bool ok; };
  ConvGeom g; const T* x; const float* sc; const float* sh;
  __device__ State fixed(int m) const {
    State s;
    s.ok = m < g.M;
    int mm = s.ok ? m : 0;
    int n = fdiv(mm, g.fd_howo);
    int r = mm - n * g.Ho * g.Wo;
    int ho = fdiv(r, g.fd_wo);
    int wo = r - ho * g.Wo;
    s.base = x + (size_t)n * g.H * g.W * g.C;
    s.hi0 = ho * g.S - g.P;
    s.wi0 = wo * g.S - g.P;
    return s;
  }
  __device__ uint4 load(const State& s, int k) const {
    if (!s.ok || k >= g.K) return zero4();
    int tap = fdiv(k, g.fd_c);
    int ci = k - tap * g.C;
    int kh = fdiv(tap, g.fd_kw);
    int kw = tap - kh * g.KW;
    int hi = s.hi0 + kh, wi = s.wi0 + kw;
    if ((unsigned)hi >= (unsigned)g.H || (unsigned)wi >= (unsigned)g.W) return zero4();
    uint4 v = ldg16(s.base + ((size_t)hi * g.W + wi) * g.C + ci);
    if constexpr (XF) v = xform_chunk<T>(v, sc, sh, ci);
    return v;
  }
  struct DState { long long off; int hi0, wi0; bool ok; };
  __device__ DState start(int m, int koff, int) const {
    State f = fixed(m);
    DState d;
    d.ok = f.ok; d.hi0 = f.hi0; d.wi0 = f.wi0;
    d.off = (long long)(f.base - x) + ((long long)f.hi0 * g.W + f.wi0) * g.C + koff;
    return d;
  }
  struct Step { long long delta; int kh, kw; bool kv; };   // K-step-uniform tap
  __device__ Step step(int k0) const {
    const int tap = fdiv(k0, g.fd_c), ci0 = k0 - tap * g.C;
    const int kh = fdiv(tap, g.fd_kw), kw = tap - kh * g.KW;
    return Step{((long long)kh * g.W + kw) * g.C + ci0, kh, kw, k0 < g.K};
  }
  __device__ const void* next(DState& d, const Step& s) const {
    const bool v = d.ok & s.kv & ((unsigned)(d.hi0 + s.kh) < (unsigned)g.H) &
                   ((unsigned)(d.wi0 + s.kw) < (unsigned)g.W);
    return v ? (const void*)(x + d.off + s.delta) : zero_page();
  }
  // buffer protocol (gemm_bk / gemm_big): the chunk's row is fixed, so the
  // validity of all KH*KW taps is one bit mask computed once; a K-step is
  // (tap, channel offset) -> one scalar byte delta
  static constexpr bool kBuf = !XF;
  struct BState { unsigned base; unsigned mask; };
  struct BStep { unsigned delta; unsigned tap; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(x, (unsigned)((size_t)g.N * g.H * g.W * g.C * sizeof(T))); }
  __device__ BState bstart(int m, int koff, int) const {
    const State f = fixed(m);
    unsigned mask = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
        if (kh < g.KH && kw < g.KW && (unsigned)(f.hi0 + kh) < (unsigned)g.H && (unsigned)(f.wi0 + kw) < (unsigned)g.W)
          mask |= 1u << (kh * g.KW + kw);
    const long long e = (long long)(f.base - x) + ((long long)f.hi0 * g.W + f.wi0) * g.C + koff;
    return BState{opaque_base((unsigned)(e * (long long)sizeof(T))), f.ok ? mask : 0u};
  }
  __device__ BStep bstep(int k0) const {
    const int tap = fdiv(k0, g.fd_c), ci0 = k0 - tap * g.C;
    const int kh = fdiv(tap, g.fd_kw), kw = tap - kh * g.KW;
    return BStep{(unsigned)((((long long)kh * g.W + kw) * g.C + ci0) * (long long)sizeof(T)), (unsigned)tap};
  }
  __device__ unsigned boff(BState& s, const BStep& st) const {
    return ((s.mask >> st.tap) & 1u) ? s.base + st.delta : kOOB;
  }
};
// BN-apply + ReLU on load for the ping-pong kernel (gemm_pp_kernel applies
// relu(sc*a + sh) to its A fragments; C <= 512 channels in its LDS table)
struct ConvFwdABn : ConvFwdA<bf16, false> {
  static constexpr bool kXformA = true;
  __device__ int xchannels() const { return g.C; }
  __device__ unsigned xrow_mask(int m) const { return bstart(m, 0, 0).mask; }
  __device__ unsigned xtap(int k0, int& ci0) const {
    const int tap = fdiv(k0, g.fd_c);
    ci0 = k0 - tap * g.C;
    return (unsigned)tap;
  }
};
// the same operand through register staging only (per-chunk filter tap): for
// channel counts the one-tap-per-K-step LDS-DMA / direct loaders cannot take
template <typename T>
struct ConvFwdAReg : ConvFwdA<T, false> {
  static constexpr bool kDirect = false;
  static constexpr bool kBuf = false;
};

// ---- data-gradient A operand (stride 1): output-gradient "patches", K-contiguous ----
template <typename T>
struct ConvDgradA {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = true;
  // the chunk-major order measured slower here (layer 3/4 +7-8 % per launch, r4d): tap-major kept
  static constexpr bool kKPerm = false;
  __device__ int kperm(int k) const { return k; }
  struct State { const T* base; int hp, wp; bool ok; };
  ConvGeom g; const T* dy;
  __device__ State fixed(int m) const {
    State s;
    s.ok = m < g.M;
    int mm = s.ok ? m : 0;
    int n = fdiv(mm, g.fd_hw);
    int r = mm - n * g.H * g.W;
    int h = fdiv(r, g.fd_w);
    int w = r - h * g.W;
    s.base = dy + (size_t)n * g.Ho * g.Wo * g.Co;
    s.hp = h + g.P;
    s.wp = w + g.P;
    return s;
  }
  __device__ uint4 load(const State& s, int k) const {
    if (!s.ok || k >= g.K) return zero4();
    int tap = fdiv(k, g.fd_co);
    int co = k - tap * g.Co;
    int kh = fdiv(tap, g.fd_kw);
    int kw = tap - kh * g.KW;
    int th = s.hp - kh, tw = s.wp - kw;
    if (th < 0 || tw < 0) return zero4();
    int ho = th, wo = tw;
    if (g.S != 1) {
      if ((th % g.S) | (tw % g.S)) return zero4();
      ho = th / g.S; wo = tw / g.S;
    }
    if (ho >= g.Ho || wo >= g.Wo) return zero4();
    return ldg16(s.base + ((size_t)ho * g.Wo + wo) * g.Co + co);
  }
  struct DState { long long off; int hp, wp; bool ok; };
  __device__ DState start(int m, int koff, int) const {
    State f = fixed(m);
    DState d;
    d.ok = f.ok; d.hp = f.hp; d.wp = f.wp;
    d.off = (long long)(f.base - dy) + ((long long)f.hp * g.Wo + f.wp) * g.Co + koff;
    return d;
  }
  struct Step { long long delta; int kh, kw; bool kv; };
  __device__ Step step(int k0) const {   // stride-1 only (S=2: ConvDgradS2A)
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int kh = fdiv(tap, g.fd_kw), kw = tap - kh * g.KW;
    return Step{co0 - ((long long)kh * g.Wo + kw) * g.Co, kh, kw, k0 < g.K};
  }
  __device__ const void* next(DState& d, const Step& s) const {
    const bool v = d.ok & s.kv & ((unsigned)(d.hp - s.kh) < (unsigned)g.Ho) &
                   ((unsigned)(d.wp - s.kw) < (unsigned)g.Wo);
    return v ? (const void*)(dy + d.off + s.delta) : zero_page();
  }
  // buffer protocol (stride 1): per-chunk tap mask, scalar byte delta per K-step
  static constexpr bool kBuf = true;
  struct BState { unsigned base; unsigned mask; };
  struct BStep { unsigned delta; unsigned tap; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(dy, (unsigned)((size_t)g.N * g.Ho * g.Wo * g.Co * sizeof(T))); }
  __device__ BState bstart(int m, int koff, int) const {
    const State f = fixed(m);
    unsigned mask = 0;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
        if (kh < g.KH && kw < g.KW && (unsigned)(f.hp - kh) < (unsigned)g.Ho && (unsigned)(f.wp - kw) < (unsigned)g.Wo)
          mask |= 1u << (kh * g.KW + kw);
    const long long e = (long long)(f.base - dy) + ((long long)f.hp * g.Wo + f.wp) * g.Co + koff;
    return BState{opaque_base((unsigned)(e * (long long)sizeof(T))), f.ok ? mask : 0u};
  }
  __device__ BStep bstep(int k0) const {
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int kh = fdiv(tap, g.fd_kw), kw = tap - kh * g.KW;
    return BStep{(unsigned)((co0 - ((long long)kh * g.Wo + kw) * g.Co) * (long long)sizeof(T)), (unsigned)tap};
  }
  __device__ unsigned boff(BState& s, const BStep& st) const {
    return ((s.mask >> st.tap) & 1u) ? s.base + st.delta : kOOB;
  }
};

// ---- stride-2 data gradient, one pixel-parity class (ph, pw) per launch ----
// dx pixels h = 2i + ph receive only taps kh = (ph + P) mod 2 + 2a, so the class
// GEMM has K = ntaps_h * ntaps_w * Co with no masked (zero) MFMA work.
struct S2Class {
  int ph, pw, kh0, kw0, nth, ntw, Hc, Wc;
  FastDiv fd_hwc, fd_wc, fd_ntw;
};
static S2Class make_s2class(const ConvGeom& g, int ph, int pw) {
  S2Class c;
  c.ph = ph; c.pw = pw;
  c.kh0 = (ph + g.P) & 1;
  c.kw0 = (pw + g.P) & 1;
  c.nth = g.KH > c.kh0 ? (g.KH - c.kh0 + 1) / 2 : 0;
  c.ntw = g.KW > c.kw0 ? (g.KW - c.kw0 + 1) / 2 : 0;
  c.Hc = (g.H - ph + 1) / 2;
  c.Wc = (g.W - pw + 1) / 2;
  c.fd_hwc = make_fastdiv(c.Hc * c.Wc > 0 ? c.Hc * c.Wc : 1);
  c.fd_wc = make_fastdiv(c.Wc > 0 ? c.Wc : 1);
  c.fd_ntw = make_fastdiv(c.ntw > 0 ? c.ntw : 1);
  return c;
}
// Downsample fold (class (0, 0) of a 3x3/2 conv beside its 1x1/2 downsample):
// the K-steps past Kc1 read the downsample's output gradient dyd (same pixel
// grid, placed dd_off elements after dy in one allocation) against the
// downsample's packed weights (wd_off elements after wt) -- the two data
// gradients sum in one GEMM, no separate launch and no addend pass.
template <typename T>
struct ConvDgradS2A {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = true;
  struct State { const T* base; int hb, wb; bool ok; };   // hb = (h + P - kh0) / 2
  ConvGeom g; S2Class c; const T* dy; int Mc, Kc;
  int Kc1 = 1 << 30; long long dd_off = 0;                // downsample segment (buffer protocol only)
  __device__ State fixed(int m) const {
    State s;
    s.ok = m < Mc;
    int mm = s.ok ? m : 0;
    int n = fdiv(mm, c.fd_hwc);
    int r = mm - n * c.Hc * c.Wc;
    int i = fdiv(r, c.fd_wc);
    int j = r - i * c.Wc;
    s.base = dy + (size_t)n * g.Ho * g.Wo * g.Co;
    s.hb = (2 * i + c.ph + g.P - c.kh0) >> 1;
    s.wb = (2 * j + c.pw + g.P - c.kw0) >> 1;
    return s;
  }
  __device__ uint4 load(const State& s, int k) const {
    if (!s.ok || k >= Kc) return zero4();
    int tap = fdiv(k, g.fd_co);
    int co = k - tap * g.Co;
    int a = fdiv(tap, c.fd_ntw);
    int b = tap - a * c.ntw;
    int ho = s.hb - a, wo = s.wb - b;
    if ((unsigned)ho >= (unsigned)g.Ho || (unsigned)wo >= (unsigned)g.Wo) return zero4();
    return ldg16(s.base + ((size_t)ho * g.Wo + wo) * g.Co + co);
  }
  struct DState { long long off; int hb, wb; bool ok; };
  __device__ DState start(int m, int koff, int) const {
    State f = fixed(m);
    DState d;
    d.ok = f.ok; d.hb = f.hb; d.wb = f.wb;
    d.off = (long long)(f.base - dy) + ((long long)f.hb * g.Wo + f.wb) * g.Co + koff;
    return d;
  }
  struct Step { long long delta; int a, b; bool kv; };
  __device__ Step step(int k0) const {
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int a = fdiv(tap, c.fd_ntw), b = tap - a * c.ntw;
    return Step{co0 - ((long long)a * g.Wo + b) * g.Co, a, b, k0 < Kc};
  }
  __device__ const void* next(DState& d, const Step& s) const {
    const bool v = d.ok & s.kv & ((unsigned)(d.hb - s.a) < (unsigned)g.Ho) &
                   ((unsigned)(d.wb - s.b) < (unsigned)g.Wo);
    return v ? (const void*)(dy + d.off + s.delta) : zero_page();
  }
  // buffer protocol: tap (a, b) of the class -> bit a*ntw + b
  static constexpr bool kBuf = true;
  struct BState { unsigned base; unsigned mask; };
  struct BStep { unsigned delta; unsigned tap; };
  __device__ rsrc_t rsrc() const {
    return buf_rsrc(dy, (unsigned)(((size_t)dd_off + (size_t)g.N * g.Ho * g.Wo * g.Co) * sizeof(T)));
  }
  __device__ BState bstart(int m, int koff, int) const {
    const State f = fixed(m);
    unsigned mask = 0;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
        if (a < c.nth && b < c.ntw && (unsigned)(f.hb - a) < (unsigned)g.Ho && (unsigned)(f.wb - b) < (unsigned)g.Wo)
          mask |= 1u << (a * c.ntw + b);
    const long long e = (long long)(f.base - dy) + ((long long)f.hb * g.Wo + f.wb) * g.Co + koff;
    return BState{opaque_base((unsigned)(e * (long long)sizeof(T))), f.ok ? mask : 0u};
  }
  __device__ BStep bstep(int k0) const {
    if (k0 >= Kc1)   // downsample segment: dyd at the class pixel itself (tap 0 of class (0, 0))
      return BStep{(unsigned)((dd_off + (k0 - Kc1)) * (long long)sizeof(T)), 0u};
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int a = fdiv(tap, c.fd_ntw), b = tap - a * c.ntw;
    return BStep{(unsigned)((co0 - ((long long)a * g.Wo + b) * g.Co) * (long long)sizeof(T)), (unsigned)tap};
  }
  __device__ unsigned boff(BState& s, const BStep& st) const {
    return ((s.mask >> st.tap) & 1u) ? s.base + st.delta : kOOB;
  }
};
// class-local row -> global NHWC row, then the wrapped epilogue
template <class EP>
struct EpiS2Remap {
  static constexpr bool kStats = EP::kStats;
  double* stat1; double* stat2; int stat_rep;
  EP inner; S2Class c; int H, W;
  __device__ int grow(int row) const {
    int n = fdiv(row, c.fd_hwc);
    int r = row - n * c.Hc * c.Wc;
    int i = fdiv(r, c.fd_wc);
    int j = r - i * c.Wc;
    return (n * H + 2 * i + c.ph) * W + 2 * j + c.pw;
  }
  __device__ void operator()(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    inner(grow(row), col, v, s1, s2);
  }
  static constexpr bool kStage = StageTrait<EP>::value;
  static constexpr bool kRow = RowTrait<EP>::value;
  __device__ v4f value(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    return inner.value(grow(row), col, v, s1, s2);
  }
  __device__ void pre8(int row, int col, RowPre& p) const { inner.pre8(grow(row), col, p); }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                       float (&s2)[8]) const {
    inner.row8(grow(row), col, v, p, s1, s2);
  }
  static constexpr int kCoefs = CoefTrait<EP>::value;
  static constexpr int kPreDepth = PreDepthTrait<EP>::value;
  __device__ const float* coef(int k) const { return inner.coef(k); }
  template <int NC>
  __device__ void row8r(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                        float (&s2)[8], const float (&cf)[NC][8]) const {
    inner.row8r(grow(row), col, v, p, s1, s2, cf);
  }
  __device__ void store8(int row, int col, const uint4& u) const { inner.store8(grow(row), col, u); }
};
// class B operand: B(ci, k = (a, b, co)) = Wt[ci][kh0 + 2a][kw0 + 2b][co]
template <typename T>
struct WtS2B {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = true;
  struct State { const T* p; bool ok; };
  const T* wt; ConvGeom g; S2Class c; int Kc;
  int Kc1 = 1 << 30; long long wd_off = 0;                // downsample segment (buffer protocol only)
  __device__ State fixed(int ci) const {
    return State{wt + (size_t)(ci < g.C ? ci : 0) * g.KH * g.KW * g.Co, ci < g.C};
  }
  __device__ uint4 load(const State& s, int k) const {
    if (!s.ok || k >= Kc) return zero4();
    int tap = fdiv(k, g.fd_co);
    int co = k - tap * g.Co;
    int a = fdiv(tap, c.fd_ntw);
    int b = tap - a * c.ntw;
    return ldg16(s.p + ((size_t)(c.kh0 + 2 * a) * g.KW + c.kw0 + 2 * b) * g.Co + co);
  }
  struct DState { const T* p; bool ok; };
  __device__ DState start(int ci, int koff, int) const {
    State f = fixed(ci);
    return DState{f.p + koff, f.ok};
  }
  struct Step { long long delta; bool kv; };
  __device__ Step step(int k0) const {
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int a = fdiv(tap, c.fd_ntw), b = tap - a * c.ntw;
    return Step{((long long)(c.kh0 + 2 * a) * g.KW + c.kw0 + 2 * b) * g.Co + co0, k0 < Kc};
  }
  __device__ const void* next(DState& d, const Step& s) const {
    return (d.ok & s.kv) ? (const void*)(d.p + s.delta) : zero_page();
  }
  // buffer protocol (Kc is a multiple of the K-step: no per-chunk k check)
  static constexpr bool kBuf = true;
  struct BState { unsigned o, od; };
  struct BStep { unsigned delta; unsigned ds; };
  __device__ rsrc_t rsrc() const {
    const size_t n = wd_off ? (size_t)wd_off + (size_t)g.C * g.Co : (size_t)g.C * g.KH * g.KW * g.Co;
    return buf_rsrc(wt, (unsigned)(n * sizeof(T)));
  }
  __device__ BState bstart(int ci, int koff, int) const {
    if (ci >= g.C) return BState{kOOB, kOOB};
    return BState{(unsigned)(((size_t)ci * g.KH * g.KW * g.Co + koff) * sizeof(T)),
                  (unsigned)(((size_t)wd_off + (size_t)ci * g.Co + koff) * sizeof(T))};
  }
  __device__ BStep bstep(int k0) const {
    if (k0 >= Kc1) return BStep{(unsigned)((k0 - Kc1) * (long long)sizeof(T)), 1u};
    const int tap = fdiv(k0, g.fd_co), co0 = k0 - tap * g.Co;
    const int a = fdiv(tap, c.fd_ntw), b = tap - a * c.ntw;
    return BStep{(unsigned)((((long long)(c.kh0 + 2 * a) * g.KW + c.kw0 + 2 * b) * g.Co + co0) * (long long)sizeof(T)),
                 0u};
  }
  __device__ unsigned boff(BState& s, const BStep& st) const {
    // bitwise select on the uniform flag: a ?: over the two members was lowered
    // to a dynamically indexed scratch copy of the state (4 scratch loads per
    // K-step in the main loop, each one counted in the LDS-DMA vmcnt waits)
    const unsigned m = 0u - st.ds;
    const unsigned b = (s.o & ~m) | (s.od & m);
    return b == kOOB ? kOOB : b + st.delta;
  }
};

// ---- weight-gradient B operand: input patches, MN-contiguous over (kh,kw,ci) ----
// The reduction runs over output pixels; the direct path walks each chunk's
// pixel (n, ho, wo) incrementally, BK pixels per K-step (constant carries).
struct PixStep {
  int dwo, dho;          // BK = dho*Wo + dwo
  int dpoff;             // element delta of (dho, dwo) in the input image
  int carry_w, carry_h;  // deltas applied when wo / ho wrap
  int small;             // Ho*Wo <= BK: recompute by division instead
};
template <typename T, bool XF>
struct ConvWgradB {
  static constexpr bool kKContig = false;
  static constexpr bool kDirect = !XF;
  struct State { int kh, kw, ci; bool ok; };
  ConvGeom g; const T* x; const float* sc; const float* sh; int Kcols; PixStep ps;
  __device__ State fixed(int col) const {
    State s;
    s.ok = col < Kcols;
    int c = s.ok ? col : 0;
    int tap = fdiv(c, g.fd_c);
    s.ci = c - tap * g.C;
    s.kh = fdiv(tap, g.fd_kw);
    s.kw = tap - s.kh * g.KW;
    return s;
  }
  __device__ uint4 load(const State& s, int m) const {
    if (!s.ok || m >= g.M) return zero4();
    int n = fdiv(m, g.fd_howo);
    int r = m - n * g.Ho * g.Wo;
    int ho = fdiv(r, g.fd_wo);
    int wo = r - ho * g.Wo;
    int hi = ho * g.S - g.P + s.kh, wi = wo * g.S - g.P + s.kw;
    if ((unsigned)hi >= (unsigned)g.H || (unsigned)wi >= (unsigned)g.W) return zero4();
    uint4 v = ldg16(x + (((size_t)n * g.H + hi) * g.W + wi) * g.C + s.ci);
    if constexpr (XF) v = xform_chunk<T>(v, sc, sh, s.ci);
    return v;
  }
  // direct staging (GStagerN, MN-contig): one output-pixel walk per thread
  // (RState, 32-bit element offsets; x < 2^31 elements is checked on the
  // host) combined with a fixed (tap, channel) offset per chunk column.
  struct RState { int poff, ho, wo, mm; };     // poff = ((n*H + ho*S)*W + wo*S)*C
  struct CState { int colofs, khp, kwp; bool ok; };
  __device__ void locate(RState& r) const {
    const int mm = r.mm < g.M ? r.mm : 0;
    const int n = fdiv(mm, g.fd_howo);
    const int rr = mm - n * g.Ho * g.Wo;
    r.ho = fdiv(rr, g.fd_wo);
    r.wo = rr - r.ho * g.Wo;
    r.poff = ((n * g.H + r.ho * g.S) * g.W + r.wo * g.S) * g.C;
  }
  __device__ RState rstart(int k, int kb) const {
    RState r;
    r.mm = kb + k;
    locate(r);
    return r;
  }
  __device__ CState cstart(int col) const {
    const State f = fixed(col);
    return CState{((f.kh - g.P) * g.W + (f.kw - g.P)) * g.C + f.ci, f.kh - g.P, f.kw - g.P, f.ok};
  }
  __device__ const void* addr(const RState& r, const CState& c) const {
    const int hi = r.ho * g.S + c.khp, wi = r.wo * g.S + c.kwp;
    const bool v = c.ok & (r.mm < g.M) & ((unsigned)hi < (unsigned)g.H) & ((unsigned)wi < (unsigned)g.W);
    return v ? (const void*)(x + (r.poff + c.colofs)) : zero_page();
  }
  __device__ void radvance(RState& r) const {
    r.mm += Elem<T>::BK;
    if (ps.small) {   // tiny images (Ho*Wo <= BK): recompute
      locate(r);
      return;
    }
    r.wo += ps.dwo;
    r.ho += ps.dho;
    r.poff += ps.dpoff;
    const bool cw = r.wo >= g.Wo;
    r.wo = cw ? r.wo - g.Wo : r.wo;
    r.ho = cw ? r.ho + 1 : r.ho;
    r.poff = cw ? r.poff + ps.carry_w : r.poff;
    const bool ch = r.ho >= g.Ho;
    r.ho = ch ? r.ho - g.Ho : r.ho;
    r.poff = ch ? r.poff + ps.carry_h : r.poff;
  }
  // buffer protocol: per pixel row a KH*KW tap-validity mask (recomputed as
  // the row walks), per chunk column a fixed byte offset and tap index
  static constexpr bool kBuf = !XF;
  struct BRow { int poff, hs, ws, mm; unsigned tmask; };   // poff: bytes of (n, ho*S, wo*S)
  struct BCol { unsigned ofs, tap; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(x, (unsigned)((size_t)g.N * g.H * g.W * g.C * sizeof(T))); }
  __device__ unsigned tapmask(int hs, int ws, int mm) const {
    unsigned wm = 0, m = 0;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw)
      if (kw < g.KW && (unsigned)(ws - g.P + kw) < (unsigned)g.W) wm |= 1u << kw;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
      if (kh < g.KH && (unsigned)(hs - g.P + kh) < (unsigned)g.H) m |= wm << (kh * g.KW);
    return mm < g.M ? m : 0u;
  }
  __device__ void blocate(BRow& r) const {
    const int mm = r.mm < g.M ? r.mm : 0;
    const int n = fdiv(mm, g.fd_howo);
    const int rr = mm - n * g.Ho * g.Wo;
    const int ho = fdiv(rr, g.fd_wo);
    const int wo = rr - ho * g.Wo;
    r.hs = ho * g.S;
    r.ws = wo * g.S;
    r.poff = ((n * g.H + r.hs) * g.W + r.ws) * g.C * (int)sizeof(T);
    r.tmask = tapmask(r.hs, r.ws, r.mm);
  }
  __device__ BRow brstart(int k, int kb) const {
    BRow r;
    r.mm = kb + k;
    blocate(r);
    return r;
  }
  __device__ BCol bcstart(int col) const {
    const State f = fixed(col);
    return BCol{(unsigned)((((f.kh - g.P) * g.W + (f.kw - g.P)) * g.C + f.ci) * (int)sizeof(T)),
                f.ok ? (unsigned)(f.kh * g.KW + f.kw) : 31u};
  }
  __device__ unsigned boff(const BRow& r, const BCol& c) const {
    return ((r.tmask >> c.tap) & 1u) ? (unsigned)r.poff + c.ofs : kOOB;
  }
  __device__ void bradvance(BRow& r) const {
    r.mm += Elem<T>::BK;
    if (ps.small) {
      blocate(r);
      return;
    }
    r.ws += ps.dwo * g.S;
    r.hs += ps.dho * g.S;
    r.poff += ps.dpoff * (int)sizeof(T);
    const bool cw = r.ws >= g.Wo * g.S;
    r.ws = cw ? r.ws - g.Wo * g.S : r.ws;
    r.hs = cw ? r.hs + g.S : r.hs;
    r.poff = cw ? r.poff + ps.carry_w * (int)sizeof(T) : r.poff;
    const bool ch = r.hs >= g.Ho * g.S;
    r.hs = ch ? r.hs - g.Ho * g.S : r.hs;
    r.poff = ch ? r.poff + ps.carry_h * (int)sizeof(T) : r.poff;
    r.tmask = tapmask(r.hs, r.ws, r.mm);
  }
};
static PixStep make_pixstep(const ConvGeom& g, int BK) {
  PixStep p;
  p.small = g.Ho * g.Wo <= BK;
  p.dho = BK / g.Wo;
  p.dwo = BK % g.Wo;
  p.dpoff = p.dwo * g.S * g.C + p.dho * g.S * g.W * g.C;
  p.carry_w = g.S * g.W * g.C - g.Wo * g.S * g.C;            // wo -= Wo, ho += 1
  p.carry_h = g.H * g.W * g.C - g.Ho * g.S * g.W * g.C;      // ho -= Ho, n += 1
  return p;
}

// ---- stem (7x7/2, 3 input channels) on a zero-padded NHWC4 image ----
// Xp[n][Hp][Wp][4] with the 3-pixel top/left padding materialised; K layout
// (kh:8, kw:8, c:4) = 256, of which kh<7, kw<7, c<3 carry weights.
struct StemGeom {
  int N, Ho, Wo, Hp, Wp, M;
  FastDiv fd_howo, fd_wo;
};
template <typename T>
struct StemA {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = true;
  struct State { const T* base; bool ok; };
  StemGeom g; const T* xp;
  __device__ State fixed(int m) const {
    State s;
    s.ok = m < g.M;
    int mm = s.ok ? m : 0;
    int n = fdiv(mm, g.fd_howo);
    int r = mm - n * g.Ho * g.Wo;
    int ho = fdiv(r, g.fd_wo);
    int wo = r - ho * g.Wo;
    s.base = xp + (((size_t)n * g.Hp + 2 * ho) * g.Wp + 2 * wo) * 4;
    return s;
  }
  __device__ uint4 load(const State& s, int k) const {
    int kh = k >> 5, kw = (k & 31) >> 2;
    if (!s.ok || kh >= 7) return zero4();
    return ldg16(s.base + ((size_t)kh * g.Wp + kw) * 4);
  }
  struct DState { const T* p; int khc; bool ok; };
  __device__ DState start(int m, int koff, int) const {
    State f = fixed(m);
    return DState{f.base + ((size_t)(koff >> 5) * g.Wp + ((koff & 31) >> 2)) * 4, koff >> 5, f.ok};
  }
  struct Step { int kh; long long delta; };
  __device__ Step step(int k0) const { return Step{k0 >> 5, (long long)(k0 >> 5) * g.Wp * 4}; }
  __device__ const void* next(DState& d, const Step& s) const {
    return (d.ok & (s.kh + d.khc < 7)) ? (const void*)(d.p + s.delta) : zero_page();
  }
  // buffer protocol: a chunk is valid while kh = k0/32 + its own kh stays < 7
  static constexpr bool kBuf = true;
  struct BState { unsigned base; int khlim; };
  struct BStep { unsigned delta; int kh; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(xp, (unsigned)((size_t)g.N * g.Hp * g.Wp * 4 * sizeof(T))); }
  __device__ BState bstart(int m, int koff, int) const {
    const State f = fixed(m);
    const size_t e = (size_t)(f.base - xp) + ((size_t)(koff >> 5) * g.Wp + ((koff & 31) >> 2)) * 4;
    return BState{(unsigned)(e * sizeof(T)), f.ok ? 7 - (koff >> 5) : -1000};
  }
  __device__ BStep bstep(int k0) const { return BStep{(unsigned)((size_t)(k0 >> 5) * g.Wp * 4 * sizeof(T)), k0 >> 5}; }
  __device__ unsigned boff(BState& s, const BStep& st) const { return st.kh < s.khlim ? s.base + st.delta : kOOB; }
};
template <typename T>
struct StemWgradB {
  static constexpr bool kKContig = false;
  static constexpr bool kDirect = true;
  struct State { int off; bool ok; };
  StemGeom g; const T* xp;
  __device__ State fixed(int col) const {
    int kh = col >> 5, kw = (col & 31) >> 2;
    return State{(kh * g.Wp + kw) * 4, kh < 7};
  }
  __device__ uint4 load(const State& s, int m) const {
    if (!s.ok || m >= g.M) return zero4();
    int n = fdiv(m, g.fd_howo);
    int r = m - n * g.Ho * g.Wo;
    int ho = fdiv(r, g.fd_wo);
    int wo = r - ho * g.Wo;
    return ldg16(xp + (((size_t)n * g.Hp + 2 * ho) * g.Wp + 2 * wo) * 4 + s.off);
  }
  struct RState { int poff, mm; };   // pixel (n, 2ho, 2wo) of the padded image, x 4 channels
  struct CState { int off; bool ok; };
  __device__ RState rstart(int k, int kb) const {
    RState r;
    r.mm = kb + k;
    locate(r);
    return r;
  }
  __device__ void locate(RState& r) const {
    const int m = r.mm < g.M ? r.mm : 0;
    const int n = fdiv(m, g.fd_howo);
    const int rr = m - n * g.Ho * g.Wo;
    const int ho = fdiv(rr, g.fd_wo);
    const int wo = rr - ho * g.Wo;
    r.poff = ((n * g.Hp + 2 * ho) * g.Wp + 2 * wo) * 4;
  }
  __device__ CState cstart(int col) const {
    const State f = fixed(col);
    return CState{f.off, f.ok};
  }
  __device__ const void* addr(const RState& r, const CState& c) const {
    return (c.ok & (r.mm < g.M)) ? (const void*)(xp + (r.poff + c.off)) : zero_page();
  }
  __device__ void radvance(RState& r) const {
    r.mm += Elem<T>::BK;
    locate(r);
  }
  // buffer protocol: incremental pixel walk over (n, ho, wo) in the padded image
  static constexpr bool kBuf = true;
  PixStep ps;   // deltas in padded-image elements (make_stem_pixstep)
  struct BRow { int poff, ho, wo, mm; };
  typedef unsigned BCol;
  __device__ rsrc_t rsrc() const { return buf_rsrc(xp, (unsigned)((size_t)g.N * g.Hp * g.Wp * 4 * sizeof(T))); }
  __device__ void blocate(BRow& r) const {
    const int m = r.mm < g.M ? r.mm : 0;
    const int n = fdiv(m, g.fd_howo);
    const int rr = m - n * g.Ho * g.Wo;
    r.ho = fdiv(rr, g.fd_wo);
    r.wo = rr - r.ho * g.Wo;
    r.poff = ((n * g.Hp + 2 * r.ho) * g.Wp + 2 * r.wo) * 4 * (int)sizeof(T);
  }
  __device__ BRow brstart(int k, int kb) const {
    BRow r;
    r.mm = kb + k;
    blocate(r);
    return r;
  }
  __device__ BCol bcstart(int col) const {
    const State f = fixed(col);
    return f.ok ? (unsigned)(f.off * (int)sizeof(T)) : kOOB;
  }
  __device__ unsigned boff(const BRow& r, const BCol& c) const { return r.mm < g.M ? (unsigned)r.poff + c : kOOB; }
  __device__ void bradvance(BRow& r) const {
    r.mm += Elem<T>::BK;
    if (ps.small) {
      blocate(r);
      return;
    }
    r.wo += ps.dwo;
    r.ho += ps.dho;
    r.poff += ps.dpoff * (int)sizeof(T);
    const bool cw = r.wo >= g.Wo;
    r.wo = cw ? r.wo - g.Wo : r.wo;
    r.ho = cw ? r.ho + 1 : r.ho;
    r.poff = cw ? r.poff + ps.carry_w * (int)sizeof(T) : r.poff;
    const bool ch = r.ho >= g.Ho;
    r.ho = ch ? r.ho - g.Ho : r.ho;
    r.poff = ch ? r.poff + ps.carry_h * (int)sizeof(T) : r.poff;
  }
};
// pixel-walk deltas of the stem's padded NHWC4 image (output pixel (n, ho, wo)
// starts at padded (n, 2ho, 2wo))
static PixStep make_stem_pixstep(const StemGeom& g, int BK) {
  PixStep p;
  p.small = g.Ho * g.Wo <= BK;
  p.dho = BK / g.Wo;
  p.dwo = BK % g.Wo;
  p.dpoff = (p.dwo * 2 + p.dho * 2 * g.Wp) * 4;
  p.carry_w = (2 * g.Wp - 2 * g.Wo) * 4;                 // wo -= Wo, ho += 1
  p.carry_h = (g.Hp * g.Wp - 2 * g.Ho * g.Wp) * 4;       // ho -= Ho, n += 1
  return p;
}

// ---- single-channel stem (the grayscale radiograph's 3 identical channels) ----
// conv(x replicated to 3 channels, w) = conv(x, w1) with w1 = sum_c w[:, c]: a
// K = (kh:8, kw:8) = 64 GEMM instead of the 4-channel K = 256 one.  A 16-B chunk
// (8 bf16 / 4 fp32) is 8 (4) consecutive kw of one kh; to keep every chunk 16-B
// aligned for LDS-DMA the padded image is stored in 4 copies shifted by 0, 2, 4,
// 6 pixels: output column wo reads copy s = wo & 3 at column 2wo - 2s (a multiple
// of 8).  Xs[s][n][Hp][Wp1], Wp1 = round8(2Wo + 8), zero outside the image.
// Requires Wo % 4 == 0 (then s is constant along the pixel walk of a K-step).
template <typename T>
struct Stem1A {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = false;
  Stem1Geom g; const T* xs;
  struct State { const T* base; bool ok; };
  __device__ size_t pix(int m) const {   // element offset of (copy, n, 2ho, 2wo - 2s)
    const int n = fdiv(m, g.fd_howo);
    const int r = m - n * g.Ho * g.Wo;
    const int ho = fdiv(r, g.fd_wo);
    const int wo = r - ho * g.Wo;
    const int sh = wo & 3;
    return (size_t)sh * g.copy + ((size_t)n * g.Hp + 2 * ho) * g.Wp1 + 2 * wo - 2 * sh;
  }
  __device__ State fixed(int m) const {
    State s;
    s.ok = m < g.M;
    s.base = xs + pix(s.ok ? m : 0);
    return s;
  }
  __device__ uint4 load(const State& s, int k) const {   // k = kh * 8 + kw0
    const int kh = k >> 3, kw = k & 7;
    if (!s.ok || kh >= 7) return zero4();
    return ldg16(s.base + (size_t)kh * g.Wp1 + kw);
  }
  static constexpr bool kBuf = true;
  struct BState { unsigned base; int khlim; };
  struct BStep { unsigned delta; int kh; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(xs, (unsigned)(4 * g.copy * sizeof(T))); }
  __device__ BState bstart(int m, int koff, int) const {
    const bool ok = m < g.M;
    const size_t e = pix(ok ? m : 0) + (size_t)(koff >> 3) * g.Wp1;
    return BState{(unsigned)(e * sizeof(T)), ok ? 7 - (koff >> 3) : -1000};
  }
  __device__ BStep bstep(int k0) const { return BStep{(unsigned)((size_t)(k0 >> 3) * g.Wp1 * sizeof(T)), k0 >> 3}; }
  __device__ unsigned boff(BState& s, const BStep& st) const { return st.kh < s.khlim ? s.base + st.delta : kOOB; }
};
template <typename T>
struct Stem1WgradB {   // B(n = kh*8 + kw, k = pixel m), MN-contiguous chunks of 8 (4) kw
  static constexpr bool kKContig = false;
  static constexpr bool kDirect = false;
  Stem1Geom g; const T* xs;
  struct State { int off; bool ok; };
  __device__ State fixed(int col) const { return State{(col >> 3) * g.Wp1 + (col & 7), (col >> 3) < 7}; }
  __device__ uint4 load(const State& s, int m) const {
    if (!s.ok || m >= g.M) return zero4();
    const int n = fdiv(m, g.fd_howo);
    const int r = m - n * g.Ho * g.Wo;
    const int ho = fdiv(r, g.fd_wo);
    const int wo = r - ho * g.Wo;
    const int sh = wo & 3;
    return ldg16(xs + (size_t)sh * g.copy + ((size_t)n * g.Hp + 2 * ho) * g.Wp1 + 2 * wo - 2 * sh + s.off);
  }
  static constexpr bool kBuf = true;
  PixStep ps;   // deltas in elements of one copy (make_stem1_pixstep)
  struct BRow { unsigned poff; int ho, wo, mm; };
  typedef unsigned BCol;
  __device__ rsrc_t rsrc() const { return buf_rsrc(xs, (unsigned)(4 * g.copy * sizeof(T))); }
  __device__ void blocate(BRow& r) const {
    const int m = r.mm < g.M ? r.mm : 0;
    const int n = fdiv(m, g.fd_howo);
    const int rr = m - n * g.Ho * g.Wo;
    r.ho = fdiv(rr, g.fd_wo);
    r.wo = rr - r.ho * g.Wo;
    const int sh = r.wo & 3;
    r.poff = (unsigned)(((size_t)sh * g.copy + ((size_t)n * g.Hp + 2 * r.ho) * g.Wp1 + 2 * r.wo - 2 * sh) * sizeof(T));
  }
  __device__ BRow brstart(int k, int kb) const {
    BRow r;
    r.mm = kb + k;
    blocate(r);
    return r;
  }
  __device__ BCol bcstart(int col) const {
    const State f = fixed(col);
    return f.ok ? (unsigned)(f.off * (int)sizeof(T)) : kOOB;
  }
  __device__ unsigned boff(const BRow& r, const BCol& c) const { return r.mm < g.M ? r.poff + c : kOOB; }
  __device__ void bradvance(BRow& r) const {
    r.mm += Elem<T>::BK;
    if (ps.small) {
      blocate(r);
      return;
    }
    // Wo % 4 == 0 and BK % 4 == 0: the copy index (wo & 3) never changes along the walk
    r.wo += ps.dwo;
    r.ho += ps.dho;
    r.poff += ps.dpoff * (int)sizeof(T);
    const bool cw = r.wo >= g.Wo;
    r.wo = cw ? r.wo - g.Wo : r.wo;
    r.ho = cw ? r.ho + 1 : r.ho;
    r.poff = cw ? r.poff + ps.carry_w * (int)sizeof(T) : r.poff;
    const bool ch = r.ho >= g.Ho;
    r.ho = ch ? r.ho - g.Ho : r.ho;
    r.poff = ch ? r.poff + ps.carry_h * (int)sizeof(T) : r.poff;
  }
};
static PixStep make_stem1_pixstep(const Stem1Geom& g, int BK) {
  PixStep p;
  p.small = g.Ho * g.Wo <= BK;
  p.dho = BK / g.Wo;
  p.dwo = BK % g.Wo;
  p.dpoff = p.dwo * 2 + p.dho * 2 * g.Wp1;
  p.carry_w = 2 * g.Wp1 - 2 * g.Wo;                  // wo -= Wo, ho += 1
  p.carry_h = g.Hp * g.Wp1 - 2 * g.Ho * g.Wp1;       // ho -= Ho, n += 1
  return p;
}

typedef const __attribute__((address_space(3))) float* lds_fp;

// 8 consecutive per-channel coefficients as two 16-B loads
__device__ __forceinline__ void ld8f(const float* p, float (&o)[8]) {
  const v4f a = *reinterpret_cast<const v4f*>(p), b = *reinterpret_cast<const v4f*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = a[j]; o[4 + j] = b[j]; }
}

// ---------------- epilogues ----------------
// raw conv output + BN batch statistics (sum, sum of squares)
template <typename T>
struct EpiConvFwd {
  static constexpr bool kStats = true;
  double* stat1; double* stat2; int stat_rep;
  T* y; int Co;
  __device__ void operator()(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    store4(y + (size_t)row * Co + col, v);
    s1 = v;
    s2 = v * v;
  }
  // staged form (multi-stage kernel): value() -> LDS tile -> 16-B row stores
  static constexpr bool kStage = true;
  __device__ v4f value(int, int, v4f v, v4f& s1, v4f& s2) const {
    s1 = v;
    s2 = v * v;
    return v;
  }
  __device__ void store8(int row, int col, const uint4& u) const { stg16(y + (size_t)row * Co + col, u); }
};
// data gradient through the producer's ReLU (mask from BN-applied y), plus
// that BN's backward statistics: sum(g), sum(g * xhat).
// 16-B store of a row-chunk epilogue (VLP_ROW_NT: non-temporal, streaming past the caches)
#ifndef VLP_ROW_NT
#define VLP_ROW_NT 1   // r4: measured +0.35 % per step (2 interleaved pairs), dgrad epilogues -1..-7 %
#endif
__device__ __forceinline__ void stg16_row(void* p, const uint4& v) {
#if VLP_ROW_NT
  typedef unsigned v4u_nt __attribute__((ext_vector_type(4)));
  __builtin_nontemporal_store(v4u_nt{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u_nt*>(p));
#else
  stg16(p, v);
#endif
}
template <typename T>
struct EpiDgradBN {
  static constexpr bool kStats = true;
  double* stat1; double* stat2; int stat_rep;
  T* g_out; int C;
  const T* y; const float* sc; const float* sh; const float* mean; const float* invstd;
  __device__ void operator()(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    v4f yv = load4(y + (size_t)row * C + col);
    v4f sc4 = *reinterpret_cast<const v4f*>(sc + col);
    v4f sh4 = *reinterpret_cast<const v4f*>(sh + col);
    v4f mu = *reinterpret_cast<const v4f*>(mean + col);
    v4f is = *reinterpret_cast<const v4f*>(invstd + col);
    v4f g;
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = (fmaf(yv[j], sc4[j], sh4[j]) > 0.f) ? v[j] : 0.f;
    store4(g_out + (size_t)row * C + col, g);
    s1 = g;
    s2 = g * ((yv - mu) * is);
  }
  static constexpr bool kRow = true;
  __device__ void pre8(int row, int col, RowPre& p) const { p.u[0] = ldg16(y + (size_t)row * C + col); }
  // y may come from an LDS image of the tile (the window kernel stages it during the last chunk)
  static constexpr int kLdsSlot = 0;
  __device__ const T* lds_operand() const { return y; }
  __device__ void pre8_rest(int, int, RowPre&) const {}
  // per-channel coefficient arrays (a caller may stage them in LDS: row8 with lds_fp)
  static constexpr int kCoefs = 4;
  __device__ const float* coef(int k) const { return k == 0 ? sc : k == 1 ? sh : k == 2 ? mean : invstd; }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                       float (&s2)[8]) const {
    row8c(row, col, v, p, s1, s2, sc, sh, mean, invstd);
  }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                       float (&s2)[8], lds_fp cf) const {
    row8c(row, col, v, p, s1, s2, cf, cf + 64, cf + 128, cf + 192);
  }
  static constexpr int kPreDepth = 16;   // one 16-B operand per row chunk
  __device__ void row8r(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                        float (&s2)[8], const float (&cf)[4][8]) const {
    row8c(row, col, v, p, s1, s2, RegCoef{cf[0], col}, RegCoef{cf[1], col}, RegCoef{cf[2], col},
          RegCoef{cf[3], col});
  }
  template <class FP>
  __device__ void row8c(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                        float (&s2)[8], FP csc, FP csh, FP cmu, FP cis) const {
    const size_t o = (size_t)row * C + col;
    float yv[8], g[8];
    Chunk<bf16>::unpack(p.u[0], yv);
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // 4 channels at a time: 16 coefficient registers live, not 32
      v4f a, b, mu, is;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        a[jj] = csc[col + 4 * h + jj]; b[jj] = csh[col + 4 * h + jj];
        mu[jj] = cmu[col + 4 * h + jj]; is[jj] = cis[col + 4 * h + jj];
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = 4 * h + jj;
        g[j] = fmaf(yv[j], a[jj], b[jj]) > 0.f ? v[j] : 0.f;
        s1[j] += g[j];
        s2[j] += g[j] * ((yv[j] - mu[jj]) * is[jj]);
      }
    }
    stg16_row(g_out + o, Chunk<bf16>::pack(g));
  }
  static constexpr bool kStage = false;
  __device__ v4f value(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    v4f yv = load4(y + (size_t)row * C + col);
    v4f sc4 = *reinterpret_cast<const v4f*>(sc + col);
    v4f sh4 = *reinterpret_cast<const v4f*>(sh + col);
    v4f mu = *reinterpret_cast<const v4f*>(mean + col);
    v4f is = *reinterpret_cast<const v4f*>(invstd + col);
    v4f g;
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = (fmaf(yv[j], sc4[j], sh4[j]) > 0.f) ? v[j] : 0.f;
    s1 = g;
    s2 = g * ((yv - mu) * is);
    return g;
  }
  __device__ void store8(int row, int col, const uint4& u) const { stg16(g_out + (size_t)row * C + col, u); }
};
// data gradient plus a residual-branch gradient
template <typename T>
struct EpiDgradAdd {
  static constexpr bool kStats = false;
  double* stat1 = nullptr; double* stat2 = nullptr;
  T* dx; const T* addend; int C;
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    size_t o = (size_t)row * C + col;
    if (addend) v += load4(addend + o);
    store4(dx + o, v);
  }
  static constexpr bool kRow = true;
  __device__ void pre8(int row, int col, RowPre& p) const {
    if (addend) p.u[0] = ldg16(addend + (size_t)row * C + col);
  }
  static constexpr int kPreDepth = 16;
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&)[8], float (&)[8]) const {
    const size_t o = (size_t)row * C + col;
    float d[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] = v[j];
    if (addend) {
      float a[8];
      Chunk<bf16>::unpack(p.u[0], a);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] += a[j];
    }
    stg16_row(dx + o, Chunk<bf16>::pack(d));
  }
  static constexpr bool kStage = false;
  __device__ v4f value(int row, int col, v4f v, v4f&, v4f&) const {
    if (addend) v += load4(addend + (size_t)row * C + col);
    return v;
  }
  __device__ void store8(int row, int col, const uint4& u) const { stg16(dx + (size_t)row * C + col, u); }
};

// data gradient (+ residual-branch addend) through the NEXT block's output
// ReLU, plus that block's BN2 backward sums: the gradient reaching block b-1
// is g = (conv_dgrad + addend) * (out_{b-1} > 0), and its bn2 needs sum(g),
// sum(g * xhat(y2_{b-1})).  Fusing this here removes the separate reduction
// pass over (dx, out, y2) and lets the next BN-backward apply read g directly.
// BITS: the ReLU sign comes from a bit mask (1/16 of the activation's bytes);
// a separate instantiation, so the activation path's registers are not shared
template <typename T, bool BITS = false>
struct EpiDgradRelu {
  static constexpr bool kStats = true;
  double* stat1; double* stat2; int stat_rep;
  T* g_out; const T* addend; int C;
  const T* relu_out; const T* y; const float* mean; const float* invstd;
  const uint8_t* rmask;   // when set: bit (o & 7) of byte o >> 3 replaces relu_out[o] > 0
  __device__ v4f grad(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    const size_t o = (size_t)row * C + col;
    if (addend) v += load4(addend + o);
    bool pos[4];
    if constexpr (BITS) {
      const unsigned b = rmask[o >> 3] >> (o & 7);
#pragma unroll
      for (int j = 0; j < 4; ++j) pos[j] = (b >> j) & 1u;
    } else {
      const v4f r = load4(relu_out + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) pos[j] = r[j] > 0.f;
    }
    const v4f yv = load4(y + o);
    const v4f mu = *reinterpret_cast<const v4f*>(mean + col);
    const v4f is = *reinterpret_cast<const v4f*>(invstd + col);
    v4f g;
#pragma unroll
    for (int j = 0; j < 4; ++j) g[j] = pos[j] ? v[j] : 0.f;
    s1 = g;
    s2 = g * ((yv - mu) * is);
    return g;
  }
  __device__ void operator()(int row, int col, v4f v, v4f& s1, v4f& s2) const {
    store4(g_out + (size_t)row * C + col, grad(row, col, v, s1, s2));
  }
  static constexpr bool kRow = true;
  __device__ void pre8(int row, int col, RowPre& p) const {
    const size_t o = (size_t)row * C + col;
    p.u[0] = addend ? ldg16(addend + o) : zero4();
    if constexpr (BITS) {
      p.u[1].x = rmask[o >> 3];
    } else {
      p.u[1] = ldg16(relu_out + o);
    }
    p.u[2] = ldg16(y + o);
  }
  // y could come from LDS as EpiDgradBN's does (kLdsSlot = 2 + lds_operand()); measured
  // slower (lock-step: layer 2 504 -> 528 us, profiles/r5l_lds_operand_ab.txt; ping-pong:
  // 494 -> 507, profiles/r5u_relu_lds_ab.txt): the addend and the mask still make the
  // epilogue wait on global loads, now behind 64 KB more DMA
  static constexpr int kLdsSlotOff = 2;
  __device__ void pre8_rest(int row, int col, RowPre& p) const {
    const size_t o = (size_t)row * C + col;
    p.u[0] = addend ? ldg16(addend + o) : zero4();
    if constexpr (BITS) {
      p.u[1].x = rmask[o >> 3];
    } else {
      p.u[1] = ldg16(relu_out + o);
    }
  }
  static constexpr int kCoefs = 2;
  __device__ const float* coef(int k) const { return k == 0 ? mean : invstd; }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                       float (&s2)[8]) const {
    row8c(row, col, v, p, s1, s2, mean, invstd);
  }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                       float (&s2)[8], lds_fp cf) const {
    row8c(row, col, v, p, s1, s2, cf, cf + 64);
  }
  static constexpr int kPreDepth = BITS ? 8 : 6;
  __device__ void row8r(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                        float (&s2)[8], const float (&cf)[2][8]) const {
    row8c(row, col, v, p, s1, s2, RegCoef{cf[0], col}, RegCoef{cf[1], col});
  }
  template <class FP>
  __device__ void row8c(int row, int col, const float (&v)[8], const RowPre& p, float (&s1)[8],
                        float (&s2)[8], FP cmu, FP cis) const {
    const size_t o = (size_t)row * C + col;
    float a[8], yv[8], g[8], mu[8], is[8];
    bool pos[8];
    Chunk<bf16>::unpack(p.u[0], a);
    if constexpr (BITS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) pos[j] = (p.u[1].x >> j) & 1u;
    } else {
      float r[8];
      Chunk<bf16>::unpack(p.u[1], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) pos[j] = r[j] > 0.f;
    }
    Chunk<bf16>::unpack(p.u[2], yv);
#pragma unroll
    for (int j = 0; j < 8; ++j) { mu[j] = cmu[col + j]; is[j] = cis[col + j]; }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = pos[j] ? v[j] + a[j] : 0.f;
      s1[j] += g[j];
      s2[j] += g[j] * ((yv[j] - mu[j]) * is[j]);
    }
    stg16_row(g_out + o, Chunk<bf16>::pack(g));
  }
  static constexpr bool kStage = false;
  __device__ v4f value(int row, int col, v4f v, v4f& s1, v4f& s2) const { return grad(row, col, v, s1, s2); }
  __device__ void store8(int row, int col, const uint4& u) const { stg16(g_out + (size_t)row * C + col, u); }
};

// data gradient (+ residual-branch addend) through the output ReLU of a block
// whose output feeds BOTH its bn2 and its downsample BN (the first block of
// layers 2-4): g = (dgrad + addend) * (out > 0) (sign bits), plus that block's
// three backward sums sum(g), sum(g * xhat2), sum(g * xhatd) -- replaces the
// separate bn_bwd_reduce pass over (dout, out, y2, yd) and the masked copy of g.
// Row-chunk epilogue only (the host routes it to the LDS-DMA kernels).
template <typename T>
struct EpiDgradRelu2 {
  static constexpr bool kStats = true;
  static constexpr bool kStats3 = true;
  double* stat1; double* stat2; int stat_rep; double* stat3;
  T* g_out; const T* addend; int C;
  const uint8_t* rmask; const T* y; const T* yd;
  const float* mean; const float* invstd; const float* meand; const float* invstdd;
  struct Pre { uint4 u[4]; };
  static constexpr bool kRow = true;
  static constexpr int kCoefs = 4;
  static constexpr int kPreDepth = 6;
  __device__ const float* coef(int k) const { return k == 0 ? mean : k == 1 ? invstd : k == 2 ? meand : invstdd; }
  __device__ void pre8(int row, int col, Pre& p) const {
    const size_t o = (size_t)row * C + col;
    p.u[0] = addend ? ldg16(addend + o) : zero4();
    p.u[1].x = rmask[o >> 3];
    p.u[2] = ldg16(y + o);
    p.u[3] = ldg16(yd + o);
  }
  __device__ void row8r3(int row, int col, const float (&v)[8], const Pre& p, float (&s1)[8], float (&s2)[8],
                         float (&s3)[8], const float (&cf)[4][8]) const {
    const size_t o = (size_t)row * C + col;
    float a[8], y2[8], y3[8], g[8];
    Chunk<bf16>::unpack(p.u[0], a);
    Chunk<bf16>::unpack(p.u[2], y2);
    Chunk<bf16>::unpack(p.u[3], y3);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      g[j] = ((p.u[1].x >> j) & 1u) ? v[j] + a[j] : 0.f;
      s1[j] += g[j];
      s2[j] += g[j] * ((y2[j] - cf[0][j]) * cf[1][j]);
      s3[j] += g[j] * ((y3[j] - cf[2][j]) * cf[3][j]);
    }
    stg16_row(g_out + o, Chunk<bf16>::pack(g));
  }
  // non-row epilogue forms (instantiated by the dispatch, never launched: the
  // host entry point refuses shapes that would not take a row-chunk kernel).
  // They cannot form the three sums, so reaching one is a dispatch bug: trap
  // (the launch fails loudly) instead of returning unmasked values and zero sums
  static constexpr bool kStage = false;
  __device__ v4f value(int, int, v4f v, v4f& s1, v4f& s2) const {
    __builtin_trap();
    s1 = s2 = v4f{0.f, 0.f, 0.f, 0.f};
    return v;
  }
  __device__ void operator()(int, int, v4f, v4f& s1, v4f& s2) const {
    __builtin_trap();
    s1 = s2 = v4f{0.f, 0.f, 0.f, 0.f};
  }
  __device__ void store8(int row, int col, const uint4& u) const { stg16(g_out + (size_t)row * C + col, u); }
};

// ---------------- tile-config dispatch ----------------
template <typename T, class LA, class LB, class EP>
static int gemm_auto(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                     hipStream_t st) {
  if (N <= 64) return gemm_narrow<T>(M, N, K, ksplit, la, lb, ep, st);
  return gemm_conv_wide<T>(M, N, K, ksplit, la, lb, ep, st);
}
// stride-2 data-gradient parity classes (short K: 1..4 taps of Co channels)
template <typename T, class LA, class LB, class EP>
static int gemm_s2(int M, int N, int K, const LA& la, const LB& lb, const EP& ep, hipStream_t st) {
  if constexpr (use_bk<T, LA, LB>()) {
    // 256x64 on the two-tiles-in-flight engine: +3 % over the one-tile ring
    constexpr int s2v = 1;
    if (N <= 64 && s2v == 1) return launch_gemm_big<256, 64, 4, 1>(M, N, K, 1, la, lb, ep, st);
    if (N <= 64 && s2v == 2) return launch_gemm_big<128, 64, 2, 1>(M, N, K, 1, la, lb, ep, st);
  }
  return gemm_auto<T>(M, N, K, 1, la, lb, ep, st);
}
// weight-gradient GEMMs: rows = Co, cols = KH*KW*C, reduction = pixels.
//  Co = 64 (stem, layer1): 64 x 128 tiles, split-K chosen by the launcher to
//    fill whole rounds of resident workgroups (ksplit = -2048: >= 2048 pixels)
//  Co >= 128: ~1024 workgroups, >= 4096 pixels each, splits in multiples of 8
//    so each XCD owns whole splits (GemmShape::xsplit); measured faster than
//    the slot-balanced split for these shapes (r1: 21.1 vs 26.1 ms per step)
template <typename T, class LA, class LB, class EP>
static int gemm_wgrad(int M, int N, int K, const LA& la, const LB& lb, const EP& ep, hipStream_t st) {
  if (M <= 64) return gemm_short<T>(M, N, K, -2048, la, lb, ep, st);
  if constexpr (use_bk<T, LA, LB>()) {   // large tiles, one workgroup per CU: slot-balanced split
    constexpr int mink5 = 2048;
    if (gemm_variant() >= 5) return gemm_conv_wide<T>(M, N, K, -mink5, la, lb, ep, st);
  }
  constexpr int balanced = 0;
  if (balanced) return gemm_wide<T>(M, N, K, -balanced, la, lb, ep, st);
  constexpr int target = 1024;
  constexpr int mink = 4096;
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  int ksplit = (target + tiles - 1) / tiles;
  const int maxsplit = (K + mink - 1) / mink;
  if (ksplit > maxsplit) ksplit = maxsplit;
  if (ksplit >= 8) ksplit = (ksplit + 7) / 8 * 8;
  return gemm_wide<T>(M, N, K, ksplit, la, lb, ep, st);
}

// ---------------- row-streaming 3x3 conv, 64 -> 64 channels (layer1) ----------------
// The implicit GEMM re-fetches every input pixel once per filter tap (9x) and
// its 9 K-steps per 256-row tile leave the prologue and epilogue exposed; at
// 64 output channels that made the layer-1 convolutions the slowest GEMMs.
// Here a workgroup owns whole images: all 9 taps of the weights are loaded
// once (LDS, then registers) and the input streams through a 5-row ring (130 pixels x 128 B per
// row, zero halo columns); output row i reads input rows i-1..i+1 as shifted
// windows of the ring, so each input byte is fetched once and a row's 9 taps
// run without barriers.  Input row i+3 is fetched while row i is computed.
//   waves: 8, each 32 output pixels x 32 channels (MFMA 16x16x32, B = weights)
// Requirements: C = Co = 64, 3x3, stride 1, pad 1, W = 128, bf16.
constexpr int kRcW = 128;                        // image width handled
// Ring row layout: pixel-major, 16-B chunk c of pixel p at c ^ ((p >> 1) & 7)
// (conflict-free at tap column 0 only; r5 PMC: 44 % of the data-gradient kernels'
// LDS cycles are conflicts, but a conflict-free planar layout measured a wash --
// profiles/r5r2_rows_planar_ab.txt -- and was removed).
constexpr int kRcSlot = (kRcW + 2) * 128;        // one ring row (bytes)
constexpr int kRcWeights = 9 * 64 * 128;         // 73728
constexpr int kRcRing = 5;
constexpr int kRcRingOff = kRcWeights;
constexpr int kRcAux = 0;                        // staging 16 KB | statistics 32 KB | y row 16 KB (filter area)
constexpr int kRcTail = kRcWeights + kRcRing * kRcSlot;   // direct-mode stats / coefficients
constexpr int kRcXtab = kRcTail + 2048;          // input-transform table: (scale, shift) or (k, b, c)
constexpr int kRcLds = kRcXtab + 768;
static_assert(kRcLds <= 160 * 1024, "rows kernel LDS map");

#ifndef VLP_ACT_NT
#define VLP_ACT_NT 0   // non-temporal stores of the transformed input rows
#endif
// Input transforms (XF), applied once per input row, in place in the ring right
// after the row lands (padding rows stay zero), the result also written to
// xin.out (the operand the weight gradient reads):
//   XF = 1 (forward): the input is the raw output of the previous conv, turned
//     into relu(sc[c]*x + sh[c]) -- BN-apply + ReLU without a separate pass;
//   XF = 2 (data gradient): the ring streams the BN output gradient g and the
//     transform is that BN's folded backward dy = k[c]*g + b[c]*y + c[c]
//     (coefficients from vlp_bn_bwd_coef; y = the BN input, LDS-DMA'd one row
//     ahead) -- the bn_bwd_apply pass without a separate launch.
struct RowsXIn {
  const float* t0; const float* t1;   // XF 1: scale, shift; XF 2: t0 = [k | b | c] (3 x 64)
  const bf16* y;                      // XF 2: the BN input
  bf16* out;                          // the transformed input rows
};
template <class EP, int XF = 0>
__global__ void __launch_bounds__(512)
conv3x3_c64_rows_kernel(int N, int H, const bf16* __restrict__ x, const bf16* __restrict__ w, int flip,
                        EP ep, int M, RowsXIn xin) {
  // 8 waves: wave w computes pixels 32*(w&3) .. +31 and channels 32*(w>>2) .. +31
  // of each output row; its 9 taps x 2 k-substeps x 2 column blocks of filter
  // fragments (144 VGPRs) stay in registers, so the row loop reads only the
  // input ring (4 ds_read_b128 per tap) and two waves share each SIMD.
  constexpr int S = RowTrait<EP>::value ? 2 : 4;  // global stores per lane per output row
  static_assert(XF != 1 || !RowTrait<EP>::value, "forward input transform with the direct epilogue only");
  static_assert(XF != 2 || RowTrait<EP>::value, "backward input transform with a row-chunk epilogue only");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wlds = smem;
  char* ring = smem + kRcRingOff;
  char* aux = smem + kRcAux;   // row-chunk epilogue: staging tile, statistics, y row
  // stats scratch: 2 KB after the ring (direct mode) or the aux area past
  // the 16 KB staging tile (row-chunk mode, 32 KB, used after the last row)
  float* red = reinterpret_cast<float*>(RowTrait<EP>::value ? aux + 16384 : smem + kRcTail);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
  const int pq = wv & 3, ch = wv >> 2;
  const rsrc_t rx = buf_rsrc(x, (unsigned)((size_t)N * H * kRcW * 64 * 2));
  const rsrc_t rw = buf_rsrc(w, 64 * 576 * 2);
  const rsrc_t rz = null_rsrc(zero_page());

  // weights: tap block t (or 8 - t: the flipped filter of a data gradient),
  // [64 rows][8 chunks] XOR-swizzled like a K-contig GEMM image
  for (int j = wv; j < 72; j += 8) {
    const int b = j >> 3, q = (j & 7) * 64 + lane;
    const int r = q >> 3, c = (q & 7) ^ ((r >> 1) & 7);
    const int tb = flip ? 8 - b : b;
    dma16(rw, (unsigned)((r * 576 + tb * 64 + c * 8) * 2), wlds + j * 1024);
  }
  // zero halo columns (ring pixels 0 and 129 of every slot)
  auto zero_halo = [&]() {
    for (int q = tid; q < kRcRing * 2 * 8; q += 512) {
      const int sl = q >> 4, side = (q >> 3) & 1, c = q & 7;
      *reinterpret_cast<uint4*>(ring + sl * kRcSlot + (side ? (kRcW + 1) * 128 : 0) + c * 16) = zero4();
    }
  };
  zero_halo();
  // the ring (or y-row) position of piece jj of this wave: pixels 8j .. 8j + 7
  auto piece_src = [&](int j, int ln, int& px, int& c) __attribute__((always_inline)) {
    const int q = j * 64 + ln;
    px = q >> 3;
    c = (q & 7) ^ (((px + 1) >> 1) & 7);
  };
  auto piece_lds = [&](char* rowbase, int j) __attribute__((always_inline)) -> char* {
    return rowbase + 128 + j * 1024;
  };
  // input row i of image n -> ring slot (i + 1) % 5, pixels at ring positions 1..128
  auto fetch = [&](int n, int i) {
    char* slot = ring + ((i + 1) % kRcRing) * kRcSlot;
    const bool live = (unsigned)i < (unsigned)H;
    const rsrc_t r = live ? rx : rz;
    const unsigned base = live ? (unsigned)(((size_t)n * H + i) * kRcW * 128) : 0u;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wv * 2 + jj;
      int px, c;
      piece_src(j, lane, px, c);
      dma16(r, base + (unsigned)(px * 128 + c * 16), piece_lds(slot, j));
    }
  };
  v4f s1[2], s2[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) s1[b] = s2[b] = v4f{0.f, 0.f, 0.f, 0.f};
  const int li = lane & 15, lg = lane >> 4;
  wait_vmcnt<0>();
  __syncthreads();
  v8bf wf[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int b = 0; b < 2; ++b) wf[t][s][b] = frag_bf16<true, 128, true>(wlds + t * 8192, ch * 32 + b * 16, s);
  if constexpr (RowTrait<EP>::value && EP::kStats) {
    __syncthreads();   // every wave holds its filter fragments before the area is reused
    v4f* rp = reinterpret_cast<v4f*>(red + tid * 16);
    rp[0] = rp[1] = rp[2] = rp[3] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  // the epilogue's per-channel coefficients (64 floats each) staged in LDS: read
  // per row with ds_read instead of held in (or reloaded into) VGPRs
  constexpr int NCF = CoefTrait<EP>::value;
  float* cfl = reinterpret_cast<float*>(smem + kRcTail);
  if constexpr (NCF > 0) {
    for (int q = tid; q < NCF * 64; q += 512) cfl[q] = ep.coef(q >> 6)[q & 63];
    __syncthreads();
  }
  float* xtab = reinterpret_cast<float*>(smem + kRcXtab);
  if constexpr (XF == 1) {
    if (tid < 128) xtab[tid] = tid < 64 ? xin.t0[tid] : xin.t1[tid - 64];
    __syncthreads();
  }
  if constexpr (XF == 2) {
    if (tid < 192) xtab[tid] = xin.t0[tid];
    __syncthreads();
  }
  // XF 2: the BN input y of a row, one row ahead, LDS-DMA'd into a one-row
  // buffer in the filter area's free part (past the 16 KB epilogue staging tile
  // and the 32 KB statistics scratch) at the same chunk positions as the ring
  // row: each thread reads back exactly the chunks its own DMA wrote
  char* ybuf = aux + 16384 + 32768;
  static_assert(16384 + 32768 + kRcW * 128 <= kRcWeights, "y row buffer fits the filter area");
  const rsrc_t ry = XF == 2 ? buf_rsrc(xin.y, (unsigned)((size_t)N * H * kRcW * 64 * 2)) : rz;
  auto yload = [&](int n, int r) __attribute__((always_inline)) {
    const bool live = (unsigned)r < (unsigned)H;   // past the last row: a null fetch keeps the vmcnt pattern
    const rsrc_t rr = live ? ry : rz;
    const unsigned base = live ? (unsigned)(((size_t)n * H + r) * kRcW * 128) : 0u;
    // the lane offsets are recomputed per call from an opaque seed (hoisted out of
    // the row loop they are loop-invariant VGPRs beside the epilogue operands)
    int sd = lane;
    asm volatile("" : "+v"(sd));
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wv * 2 + jj;
      int px, c;
      piece_src(j, sd, px, c);
      dma16(rr, base + (unsigned)(px * 128 + c * 16), ybuf + j * 1024);
    }
  };
  // ring row r (0 <= r < H) of image n -> relu(sc*x + sh), in place and to xout;
  // each thread transforms the two 16-B chunks its own ring fetch wrote, so
  // its vmcnt wait alone makes them readable (no barrier before the transform)
  auto xrow = [&](int n, int r) __attribute__((always_inline)) {
    char* slot = ring + ((r + 1) % kRcRing) * kRcSlot;
    int sd = lane;
    if constexpr (XF == 2) asm volatile("" : "+v"(sd));
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int j = wv * 2 + jj, q = j * 64 + sd;
      int px, cc;
      piece_src(j, sd, px, cc);
      uint4* p = reinterpret_cast<uint4*>(piece_lds(slot, j) + sd * 16);
      float f[8];
      Chunk<bf16>::unpack(*p, f);
      if constexpr (XF == 2) {
        float yy[8];
        Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(ybuf + q * 16), yy);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          f[j] = bn_bwd_dy(xtab[cc * 8 + j], xtab[64 + cc * 8 + j], xtab[128 + cc * 8 + j], f[j], yy[j]);
      } else {
        const v4f s0 = *reinterpret_cast<const v4f*>(xtab + cc * 8), s1 = *reinterpret_cast<const v4f*>(xtab + cc * 8 + 4);
        const v4f h0 = *reinterpret_cast<const v4f*>(xtab + 64 + cc * 8), h1 = *reinterpret_cast<const v4f*>(xtab + 68 + cc * 8);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f[j] = fmaxf(fmaf(f[j], s0[j], h0[j]), 0.f);
          f[4 + j] = fmaxf(fmaf(f[4 + j], s1[j], h1[j]), 0.f);
        }
      }
      const uint4 v = Chunk<bf16>::pack(f);
      *p = v;
#if VLP_ACT_NT
      typedef unsigned v4u_nt __attribute__((ext_vector_type(4)));
      __builtin_nontemporal_store(v4u_nt{v.x, v.y, v.z, v.w},
                                  reinterpret_cast<v4u_nt*>(xin.out + (((size_t)n * H + r) * kRcW + px) * 64 + cc * 8));
#else
      stg16(xin.out + (((size_t)n * H + r) * kRcW + px) * 64 + cc * 8, v);
#endif
    }
  };

  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    wait_vmcnt<0>();
    __syncthreads();
    if constexpr (XF == 2) {
      fetch(n, -1); fetch(n, 0); yload(n, 0);
    } else {
      fetch(n, -1); fetch(n, 0); fetch(n, 1); fetch(n, 2);
    }
    for (int i = 0; i < H; ++i) {
      if constexpr (XF == 2) {
        // per row i: [dy stores of row i+1] [epilogue operands of row i] [y of row
        // i+2] [ring fetch of row i+3] MFMAs [epilogue stores of row i]; row i+1's
        // ring data and y are older than the last fetch and epilogue stores
        if (i == 0) {
          // prologue order: fetch -1, fetch 0, y 0, then y 1, fetch 1, fetch 2 here
          wait_vmcnt<0>();
          xrow(n, 0);
          yload(n, 1);
          fetch(n, 1);
          fetch(n, 2);
          wait_vmcnt<2>();                                   // y 1 and ring row 1 landed (row 2 in flight)
          xrow(n, 1);
        } else {
          wait_vmcnt<2 + S>();                               // y / ring row i+1 landed (fetch i+2, row i-1 stores in flight)
          if (i + 1 < H) xrow(n, i + 1);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else {
        // XF adds the xout stores (2 per row, rows 0 and 1 both in row 0) before
        // each row's ring fetch
        if (i == 0) wait_vmcnt<2>();                           // rows -1..1 landed (row 2 in flight)
        else if (i == 1) wait_vmcnt<2 + S + (XF ? 4 : 0)>();   // row 2 (row 3, row-0 stores in flight)
        else wait_vmcnt<2 + 2 * S + (XF ? 2 : 0)>();           // row i+1 (rows i+2, stores of i-2, i-1)
        if constexpr (XF == 1) {
          if (i == 0) { xrow(n, 0); xrow(n, 1); }
          else if (i + 1 < H) xrow(n, i + 1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
      raw_barrier();                            // all waves: ring rows landed (and transformed), row i-1 done
      // epilogue operands of this row (row-chunk epilogues): issued now, consumed
      // after the MFMAs, and BEFORE the ring fetch of row i+3 -- vmcnt retires in
      // issue order, so the epilogue's wait for them leaves that fetch in flight
      // (issued after the fetch, the wait drained it within the row: layer-1
      // data gradient with the ReLU epilogue 641 -> 561 us, tools/conv_bench.py)
      constexpr bool kRowEpi = RowTrait<EP>::value;
      if constexpr (!kRowEpi) fetch(n, i + 3);
      RowPre pre[2];
      if constexpr (kRowEpi) {
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) ep.pre8((n * H + i) * kRcW + (tid >> 3) + 64 * h2, (tid & 7) * 8, pre[h2]);
        __builtin_amdgcn_sched_barrier(0);      // keep the issue order
        if constexpr (XF == 2) {
          yload(n, i + 2);
          __builtin_amdgcn_sched_barrier(0);
        }
        fetch(n, i + 3);
      }
      v4f acc[2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};
      // row-chunk epilogues: the lane's ring offsets of its (kw, s) fragments
      // (kc_off of ring row 32pq + kw + li, chunk 4s + lg; the a = 1 fragment is
      // +16 rows = +2 KiB, same swizzle) are recomputed per row from an opaque
      // seed -- hoisted out of the row loop they were ~35 loop-invariant VGPRs
      // that spilled beside the epilogue operands, and every scratch reload's
      // vmcnt(0) drained the ring prefetch.  (The forward, with no epilogue
      // operands, keeps the hoisted form: 362 vs 383 us.)
      int seed = pq * 32 + li;
      if constexpr (kRowEpi) asm volatile("" : "+v"(seed));
      int foff[3][2];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int r = seed + kw;
          foff[kw][s] = r * 128 + (((4 * s + lg) ^ ((r >> 1) & 7)) << 4);
        }
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* sl = ring + ((i + kh) % kRcRing) * kRcSlot;   // input row i - 1 + kh
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          v8bf fa[2][2];
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a) {
              if constexpr (kRowEpi) fa[s][a] = *reinterpret_cast<const v8bf*>(sl + foff[kw][s] + a * 2048);
              else fa[s][a] = frag_bf16<true, 128, true>(sl, pq * 32 + a * 16 + kw, s);
            }
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int b = 0; b < 2; ++b)
                acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kh * 3 + kw][s][b], fa[s][a], acc[a][b], 0, 0, 0);
        }
      }
      if constexpr (RowTrait<EP>::value) {
        // row-chunk epilogue through the (now free) filter staging area: the
        // output row is staged as bf16, then thread t handles pixels t/8 and
        // t/8 + 64 at the FIXED 8-channel group t%8, so its operand loads and
        // stores are row-contiguous 16-B chunks
        bf16* stg = reinterpret_cast<bf16*>(wlds);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const int px = pq * 32 + a * 16 + li, co = ch * 32 + b * 16 + 4 * lg;
            v4bf ob;
            ob[0] = (bf16)acc[a][b][0]; ob[1] = (bf16)acc[a][b][1];
            ob[2] = (bf16)acc[a][b][2]; ob[3] = (bf16)acc[a][b][3];
            *reinterpret_cast<v4bf*>(stg + px * 64 + (((co >> 3) ^ (px & 7)) << 3) + (co & 4)) = ob;
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        raw_barrier();
        const int rowbase = (n * H + i) * kRcW;
        float r1[8], r2[8];   // this row's sums of the thread's 8 channels
#pragma unroll
        for (int j = 0; j < 8; ++j) r1[j] = r2[j] = 0.f;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          const int px = (tid >> 3) + 64 * h2, c = tid & 7;
          float v[8];
          Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(stg + px * 64 + ((c ^ (px & 7)) << 3)), v);
          if constexpr (NCF > 0) ep.row8(rowbase + px, c * 8, v, pre[h2], r1, r2, (lds_fp)cfl);
          else ep.row8(rowbase + px, c * 8, v, pre[h2], r1, r2);
        }
        if constexpr (EP::kStats) {   // running sums live in LDS (thread-private slots), not VGPRs
          v4f* rp = reinterpret_cast<v4f*>(red + tid * 16);
          v4f q0 = rp[0], q1 = rp[1], q2 = rp[2], q3 = rp[3];
#pragma unroll
          for (int j = 0; j < 4; ++j) { q0[j] += r1[j]; q1[j] += r1[4 + j]; q2[j] += r2[j]; q3[j] += r2[4 + j]; }
          rp[0] = q0; rp[1] = q1; rp[2] = q2; rp[3] = q3;
        }
      } else {
        // direct epilogue: lane (li, lg) owns pixel 32pq + 16a + li, channels 32ch + 16b + 4lg .. +3
        const int rowbase = (n * H + i) * kRcW + pq * 32;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            v4f c1 = v4f{0.f, 0.f, 0.f, 0.f}, c2 = c1;
            ep(rowbase + a * 16 + li, ch * 32 + b * 16 + 4 * lg, acc[a][b], c1, c2);
            if constexpr (EP::kStats) { s1[b] += c1; s2[b] += c2; }
          }
      }
    }
  }
  if constexpr (EP::kStats && RowTrait<EP>::value) {
    // per-column sums: thread t holds columns 8*(t%8) .. +7 -> 64 threads per group
    __syncthreads();
    if (tid < 128) {
      const int co = tid >> 1, stt = tid & 1;
      float xs = 0.f;
      for (int k = co >> 3; k < 512; k += 8) xs += red[k * 16 + stt * 8 + (co & 7)];
      const int rep = ep.stat_rep > 1 ? (int)(blockIdx.x % ep.stat_rep) : 0;
      atomicAdd((stt ? ep.stat2 : ep.stat1) + (size_t)rep * 64 + co, (double)xs);
    }
  } else if constexpr (EP::kStats) {
    // per-column sums: rows of each 16-lane group, then the 4 pixel-quarter
    // waves, then one fp64 atomic per column into replica blockIdx % stat_rep
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xs = row16_sum(s1[b][j]), ys = row16_sum(s2[b][j]);
        if (li == 15) {
          const int co = ch * 32 + b * 16 + 4 * lg + j;
          red[(pq * 64 + co) * 2 + 0] = xs;
          red[(pq * 64 + co) * 2 + 1] = ys;
        }
      }
    __syncthreads();
    if (tid < 64) {
      float xs = 0.f, ys = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) { xs += red[(q * 64 + tid) * 2]; ys += red[(q * 64 + tid) * 2 + 1]; }
      const int rep = ep.stat_rep > 1 ? (int)(blockIdx.x % ep.stat_rep) : 0;
      atomicAdd(ep.stat1 + (size_t)rep * 64 + tid, (double)xs);
      atomicAdd(ep.stat2 + (size_t)rep * 64 + tid, (double)ys);
    }
  }
  (void)M;
}

static bool rows_c64_ok(const ConvGeom& g) {
  constexpr int off = 0;
  return !off && g.C == 64 && g.Co == 64 && g.KH == 3 && g.KW == 3 && g.S == 1 && g.P == 1 && g.W == kRcW &&
         g.H >= 3 && (size_t)g.N * g.H * kRcW * 128 < (1ull << 31);
}
template <class EP, int XF = 0>
static int launch_rows_c64(const ConvGeom& g, const void* x, const void* w, int flip, const EP& ep,
                           hipStream_t st, const RowsXIn& xin = RowsXIn{}) {
  // per device and cheap: set on every launch (a process-wide flag would miss a second GPU)
  const hipError_t ae = hipFuncSetAttribute((const void*)&conv3x3_c64_rows_kernel<EP, XF>,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, kRcLds);
  if (ae != hipSuccess) return (int)ae;
  int grid = device_cus();
  if (grid > g.N) grid = g.N;
  hipLaunchKernelGGL((conv3x3_c64_rows_kernel<EP, XF>), dim3(grid), dim3(512), kRcLds, st, g.N, g.H,
                     (const bf16*)x, (const bf16*)w, flip, ep, g.N * g.H * g.W, xin);
  return (int)hipGetLastError();
}

// ---------------- row-streaming 3x3 weight gradient, 64 -> 64 channels (layer1) ----------------
//   dW[co][(kh,kw,ci)] = sum_(n,i,j) dy[n][i][j][co] * x[n][i+kh-1][j+kw-1][ci]
// The im2col weight-gradient GEMM (64 x 192 tiles) pulled every input pixel
// through the LDS-DMA path once per filter tap (9x the input and 3x dy per
// launch) and ran at 40 % of HBM and 33 % of the MFMA rate.  Here a workgroup
// owns whole images and streams them row by row: dy row i and input rows
// i-1..i+1 sit in two LDS rings, pixel-major as they arrive, and both MFMA
// operands are ds_read_b64_tr_b16 transposing reads -- the reduction index of
// both is the pixel, so a tap's column shift is only the first ring position
// a lane addresses.  Each byte of dy and x is fetched from HBM once.  The
// workgroup's 64 x 576 fp32 partial stays in registers across its images and
// is written once, as split slab blockIdx.x; vlp_conv_wgrad_fold sums the
// slabs in a fixed order (deterministic).
//   waves: 8; wave w owns output channels 32(w&1) .. +31 x columns 144(w>>1) .. +143
//   (2 x 9 blocks of 16 x 16: 72 fp32 accumulators per lane)
//   rings: input rows in 5 slots (rows i-1 .. i+3), dy rows in 3 (i .. i+2), so
//   two rows of each are in flight while row i is reduced
// Measured at bs 256 (profiles/r6_wgrad_rows_ab.txt): 337 us per launch, 3.2 TB/s
// and 0.92 PF; timing builds without the MFMAs ~215 us (5 TB/s) and without the
// ring fetches ~200 us, at an effective clock of ~1.6 GHz (GRBM_GUI_ACTIVE / 8 /
// wall): the two halves overlap only partly under the chip's power limit.
#ifndef VLP_WGRAD_ROWS
#define VLP_WGRAD_ROWS 1   // 0: layer-1 weight gradients on the im2col GEMM (gemm_short)
#endif
constexpr int kRwXSlot = (kRcW + 2) * 128;   // 130 ring positions: zero halo at 0 and 129
constexpr int kRwDSlot = kRcW * 128;
constexpr int kRwXSlots = 5, kRwDSlots = 3;
constexpr int kRwDOff = kRwXSlots * kRwXSlot;
constexpr int kRwLds = kRwDOff + kRwDSlots * kRwDSlot;
static_assert(kRwLds <= 160 * 1024, "weight-gradient rows kernel LDS map");
static_assert(kRwXSlot % 256 == 0 && kRwDOff % 256 == 0, "ring slots start on bank 0");
// 16-B chunk c of ring position `pos` is stored at chunk c ^ mn8_h(pos).  A
// transposing read's 32-lane half touches positions r0 + {0..3} and r0 + {8..11}
// (8 B each of one 32-B channel block); XOR-ing bits 1 and 3 of the position
// into the chunk puts them on 64 distinct banks for every r0 mod 8 (a Python
// bank model over the r0 the reads use: 0..2 and 4..6 mod 8, all conflict-free).

// two transposing reads (k-rows +0..3 from `lo`, +4..7 from `hi`) at immediate OFF
template <int OFF>
__device__ __forceinline__ v8bf tr_pair(unsigned lo_addr, unsigned hi_addr) {
  v4bf lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(lo_addr), "n"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(hi_addr), "n"(OFF));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
conv3x3_c64_wgrad_rows_kernel(int N, int H, const bf16* __restrict__ dy, const bf16* __restrict__ x,
                              float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(tid >> 6));
  const int ch = wv & 1, cq = wv >> 1;
  const unsigned bytes = (unsigned)((size_t)N * H * kRcW * 128);
  const rsrc_t rx = buf_rsrc(x, bytes), rd = buf_rsrc(dy, bytes);

  // zero halo positions (never DMA targets): all 8 chunks of positions 0 and 129
  for (int q = tid; q < kRwXSlots * 16; q += 512) {
    const int sl = q >> 4, side = (q >> 3) & 1, c = q & 7;
    *reinterpret_cast<uint4*>(smem + sl * kRwXSlot + (side ? (kRcW + 1) * 128 : 0) + c * 16) = zero4();
  }
  // DMA pieces: piece j = 2 wv + jj of a row fills LDS chunks j*64 + lane (pixel
  // (j*64 + lane) >> 3, stored chunk lane & 7) from the logical chunk the swizzle
  // puts there; input rows sit one position right of their pixel (the halo)
  unsigned xo[2], dof[2];
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int u = (wv * 2 + jj) * 64 + lane, px = u >> 3, cs = u & 7;
    dof[jj] = (unsigned)(px * 128 + ((cs ^ mn8_h(px)) << 4));
    xo[jj] = (unsigned)(px * 128 + ((cs ^ mn8_h(px + 1)) << 4));
  }
  auto fetch_x = [&](int n, int r) __attribute__((always_inline)) {
    char* sl = smem + ((r + 1) % kRwXSlots) * kRwXSlot + 128;
    const unsigned base = (unsigned)r < (unsigned)H ? (unsigned)(((size_t)n * H + r) * (kRcW * 128)) : kOOB;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) dma16(rx, base + xo[jj], sl + (wv * 2 + jj) * 1024);
  };
  auto fetch_d = [&](int n, int r) __attribute__((always_inline)) {
    char* sl = smem + kRwDOff + (r % kRwDSlots) * kRwDSlot;
    const unsigned base = r < H ? (unsigned)(((size_t)n * H + r) * (kRcW * 128)) : kOOB;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) dma16(rd, base + dof[jj], sl + (wv * 2 + jj) * 1024);
  };

  // lane read addresses (slot 0, k-step 0): lane 16g + 4q + p reads k-rows
  // (pixels) 8g + q (+4 for the upper half) at channels 4p .. 4p+3 of its block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const unsigned l0 = lds_addr(smem);
  unsigned abase[2][2], bbase[9][2];
  int bkh[9];   // input-row offset (kh) of column block jb: wave-uniform
#pragma unroll
  for (int hl = 0; hl < 2; ++hl) {
    const int pos = 8 * g + q + 4 * hl;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int c = 2 * (2 * ch + a) + (p >> 1);
      abase[a][hl] = l0 + kRwDOff + pos * 128 + ((c ^ mn8_h(pos)) << 4) + 8 * (p & 1);
    }
#pragma unroll
    for (int jb = 0; jb < 9; ++jb) {
      const int b = 9 * cq + jb, t = b >> 2, kw = t % 3, c = 2 * (b & 3) + (p >> 1);
      bkh[jb] = t / 3;
      const int ps = pos + kw;
      bbase[jb][hl] = l0 + ps * 128 + ((c ^ mn8_h(ps)) << 4) + 8 * (p & 1);
    }
  }

  v4f acc[2][9];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int jb = 0; jb < 9; ++jb) acc[a][jb] = v4f{0.f, 0.f, 0.f, 0.f};

  // Read units: k-step s = u / 3 (pixels 32s .. 32s+31) and column blocks
  // 3 (u % 3) .. +2, plus the k-step's two dy fragments in its first unit.  Unit
  // u+1's reads are issued in front of unit u's 6 MFMAs (about 100 cycles per
  // wave, two waves per SIMD, cover their latency) with 40 fragment VGPRs live;
  // whole k-steps double-buffered (88) spilled once the pipeline crossed rows.
  v8bf fa[2][2], fb[2][3];
  auto issue_unit = [&](auto U, unsigned dso, const unsigned (&xso)[9]) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value, s = u / 3, gq = u % 3, OFF = s * 32 * 128;
    if constexpr (gq == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[s & 1][a] = tr_pair<OFF>(abase[a][0] + dso, abase[a][1] + dso);
    }
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int jb = 3 * gq + jj;
      fb[u & 1][jj] = tr_pair<OFF>(bbase[jb][0] + xso[jb], bbase[jb][1] + xso[jb]);
    }
  };
  // the asm reads are invisible to the compiler's LDS tracking: wait by hand and
  // tie the wait to the fragment registers so no MFMA is scheduled above it
  auto land_unit = [&](auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value, s = u / 3, gq = u % 3;
    v8bf(&ta)[2] = fa[s & 1];
    v8bf(&tb)[3] = fb[u & 1];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (gq == 0) {
#pragma unroll
      for (int a = 0; a < 2; ++a) asm volatile("" : "+v"(ta[a]));
    }
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) asm volatile("" : "+v"(tb[jj]));
  };
  auto mfma_unit = [&](auto U) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value, s = u / 3, gq = u % 3;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
        acc[a][3 * gq + jj] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[u & 1][jj], fa[s & 1][a], acc[a][3 * gq + jj], 0, 0, 0);
  };
  auto slots = [&](int i, unsigned& dso, unsigned (&xso)[9]) __attribute__((always_inline)) {
    dso = (unsigned)((i % kRwDSlots) * kRwDSlot);
#pragma unroll
    for (int jb = 0; jb < 9; ++jb) xso[jb] = (unsigned)(((i + bkh[jb]) % kRwXSlots) * kRwXSlot);
  };

  // Per row i: read units 0..10, then the row's one barrier, then unit 11.  The
  // barrier sits in front of the LAST unit so that the next row's first reads
  // (and the ring fetches of input row i+4 / dy row i+3) are issued before it and
  // overlap its MFMAs: no wave idles on an LDS round trip at a row start.  Fetch
  // group of row i (issued at its barrier): input row i+4 into the slot of row
  // i-1 and dy row i+3 into the slot of dy row i -- every wave has LANDED all of
  // row i's fragment reads before the barrier (lgkmcnt(0)), so both slots are
  // free.  vmcnt (in-order retirement): at row i's barrier the groups of rows i-1
  // (input i+3, dy i+2) and i-2 are outstanding; waiting down to 4 lands the
  // older one, i.e. input row i+2 and dy row i+1, the last rows row i+1 needs.
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    wait_vmcnt<0>();
    __syncthreads();   // the previous image's ring reads are done (and the halo is zero)
    fetch_x(n, -1); fetch_x(n, 0); fetch_x(n, 1); fetch_d(n, 0);
    fetch_x(n, 2); fetch_d(n, 1);
    wait_vmcnt<4>();     // input rows -1..1 and dy row 0 (input 2 and dy 1 in flight)
    raw_barrier();
    fetch_x(n, 3); fetch_d(n, 2);   // the "row -1" group
    unsigned dso, xso[9];
    slots(0, dso, xso);
    issue_unit(std::integral_constant<int, 0>{}, dso, xso);
    for (int i = 0; i < H; ++i) {
      // sched_barrier: the scheduler otherwise sinks each unit's reads below the
      // MFMAs of the unit before (fewer live VGPRs), so every unit waited out a
      // full LDS round trip in front of its MFMAs
      static_for<0, 11>([&](auto U) {
        land_unit(U);
        issue_unit(std::integral_constant<int, decltype(U)::value + 1>{}, dso, xso);
        __builtin_amdgcn_sched_barrier(0);
        mfma_unit(U);
        __builtin_amdgcn_sched_barrier(0);
      });
      land_unit(std::integral_constant<int, 11>{});   // this wave reads nothing more of row i
      wait_vmcnt<4>();     // input row i+2 and dy row i+1 landed
      raw_barrier();
      fetch_x(n, i + 4);
      fetch_d(n, i + 3);
      // unconditional (a branch here made the compiler copy the in-flight
      // fragment registers at the merge); past the last row it reads stale slots
      slots(i + 1, dso, xso);
      issue_unit(std::integral_constant<int, 0>{}, dso, xso);
      __builtin_amdgcn_sched_barrier(0);
      mfma_unit(std::integral_constant<int, 11>{});
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // no read in flight past the image
  }
  wait_vmcnt<0>();
  // lane (g, i) holds columns 16 b + 4g .. +3 of output channel 16 (2ch + a) + i
  float* out = ws + (size_t)blockIdx.x * (64 * 576);
  const int i16 = lane & 15;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int jb = 0; jb < 9; ++jb)
      *reinterpret_cast<v4f*>(out + (size_t)(16 * (2 * ch + a) + i16) * 576 + 16 * (9 * cq + jb) + 4 * g) = acc[a][jb];
}

// smallest batch (images) for the row-streaming form: one workgroup per image, so
// a batch well below the CU count leaves most of the chip idle (the per-image
// time is fixed) where the im2col GEMM spreads the pixels over every CU
static int g_wgrad_rows_min = -1;   // -1: 3/4 of the device's CUs
static bool wgrad_rows_ok(const ConvGeom& g) {
  const int mn = g_wgrad_rows_min >= 0 ? g_wgrad_rows_min : device_cus() * 3 / 4;
  return VLP_WGRAD_ROWS && g.C == 64 && g.Co == 64 && g.KH == 3 && g.KW == 3 && g.S == 1 && g.P == 1 &&
         g.W == kRcW && g.H >= 1 && g.N >= mn && (size_t)g.N * g.H * kRcW * 128 < (1ull << 31);
}
// one slab per workgroup: grid <= the slabs the workspace holds
static int launch_wgrad_rows(const ConvGeom& g, const void* dy, const void* x, float* ws, int max_ks, int* ks_out,
                             hipStream_t st) {
  const hipError_t ae = hipFuncSetAttribute((const void*)&conv3x3_c64_wgrad_rows_kernel,
                                            hipFuncAttributeMaxDynamicSharedMemorySize, kRwLds);
  if (ae != hipSuccess) return (int)ae;
  int grid = device_cus();
  if (grid > g.N) grid = g.N;
  if (grid > max_ks) grid = max_ks;
  hipLaunchKernelGGL(conv3x3_c64_wgrad_rows_kernel, dim3(grid), dim3(512), kRwLds, st, g.N, g.H,
                     (const bf16*)dy, (const bf16*)x, ws);
  *ks_out = grid;
  return (int)hipGetLastError();
}

// ---------------- LDS-window implicit GEMM: 3x3, stride 1, 64-channel chunks ----------------
// The im2col GEMMs fetch every input pixel once per filter tap: 9 copies of the
// A operand per 64-channel chunk pass through the LDS-DMA path, whose intake
// bounds those kernels (no-DMA timing experiment 299 -> 185 us on
// layer 3).  Here a workgroup owns 256 output pixels = TH full image rows of
// width TW; per 64-channel chunk it stages the tile's input WINDOW -- (TH+2) x
// (TW+2) pixels with the halo, zero outside the image -- once, and all 9 taps
// read their A fragments from it at a compile-time pixel offset (tap (kh, kw):
// +(kh * (TW+2) + kw); the data gradient, FLIP, reads the flipped tap).  Only
// the B operand (the filter slice of the tap) streams per K-step, through a
// 4-slot ring of 32-deep half-tiles (HStager, as the ping-pong kernel).  A
// bytes per chunk: ~1.5 tiles instead of 9.
// Window layout: 160 B per pixel (128 B of channels + 32 B of padding).  A
// ds_read_b128 is serviced in 4 lane groups of 16 that mix the fragment's
// pixels li in {0-3, 12-15} of one 16-B chunk with li in {4-11} of the next
// chunk: at a stride of 10 16-B units the first set lands on the even and the
// second on the odd bank slots, all distinct, for ANY first pixel -- every tap
// offset reads conflict-free (a 128-B stride with an XOR swizzle cannot be
// conflict-free for all 3 column offsets).  The LDS-DMA pieces (1 KiB per wave
// instruction, lane -> 16 B) fill the padding from past the buffer resource
// (zeros), as they do pixels outside the image.  Two window buffers: chunk
// c+1's pieces are issued over the first half-steps of chunk c, so the in-order
// vmcnt wait for each B half-tile never waits on a whole window.  Workgroup
// geometry: 8 waves, 4 (M) x 2 (N), 64 x BN/2 per wave (MFMA 16x16x32), in two
// ping-pong groups (below); the epilogue is the multi-stage kernels'
// ms_epilogue<256, BN, 4, 2>.  (r5: a lock-step 8-wave form, a persistent forward
// and timing-experiment builds were measured against this one and removed; their
// records are profiles/r5q3_window_pingpong_ab.txt, r5p3_window_persistent_ab.txt,
// r5x_window_experiments.txt, r5ds_window_desync_ab.json.)
template <int TW, int NW = 8, int MINP = 0>
struct WinGeom {
  static constexpr int TH = 256 / TW;                  // image rows per tile
  static constexpr int WR = TH + 2, WC = TW + 2;       // window rows / columns
  static constexpr int PS = 160;                       // LDS bytes per window pixel
  static constexpr int BYTES = WR * WC * PS;
  static constexpr int PPW0 = ((BYTES + 1023) / 1024 + NW - 1) / NW;
  // 1-KiB pieces per wave (MINP: at least that many pieces per buffer -- 64 when the
  // epilogue's operand tile [256][128] bf16 is staged in the spare buffer)
  static constexpr int PPW = PPW0 * NW >= MINP ? PPW0 : (MINP + NW - 1) / NW;
  static constexpr int SLOT = PPW * NW * 1024;         // one window buffer
};
// 64 pieces per buffer when the row epilogue's operand tile [256][128] bf16 is staged in the spare buffer
template <class EP> constexpr int win_minp() { return LdsSlotTrait<EP>::value >= 0 ? 64 : 0; }

// Ping-pong window kernel (conv3x3_winpp_kernel).  The two wave groups (rows
// 0-127: waves 0-3, rows 128-255: waves 4-7; one wave of each per SIMD) run one
// barrier interval apart, as in gemm_pp_kernel: every half-step is [wait, barrier,
// fetch + fragment reads, barrier, MFMAs], so in each interval one group's MFMAs
// run while the other group issues its LDS-DMA pieces and fragment reads, and the
// SIMD's MFMA pipe does not drain at every barrier.  Group 0 fetches the windows
// (chunk c+1's pieces one per half-step over the first PPW half-steps of chunk
// c), group 1 the B half-tiles (B(u+3) at half-step u, ring slot (u+3) & 3).
// Barrier k of group 0 pairs with barrier k of group 1: group 1 runs one extra
// barrier before its first half-step, group 0 one after its last.  Hazards (u =
// half-step, #k = barrier k; group 0 reads in (#2u+1, #2u+2), group 1 in (#2u+2,
// #2u+3)): B(u+3) is written after #2u+2, its slot last read before #2u+1; B(v) is
// waited for by group 1 before #2v and read after #2v+1; window c+1's pieces go
// out at half-steps 18c+1 .. 18c+PPW (PPW <= 16), the last waited for by group 0
// before #36c+37, the first read of chunk c+1.  Window buffer reuse: chunk c+1's
// first piece is written after #36c+3; the last reads of that buffer (chunk c-1)
// are group 1's at half-step 18c-1, issued before #36c+1 and retired by its
// lgkmcnt(0) before it reaches #36c+2 (one barrier of margin, as the B ring).
//
// (r6: BN-apply + ReLU of the input applied in the window, XF = 1, was built here
// -- bit-identical to the pass + conv -- and measured slower than the separate
// pass at every width: profiles/r6_window_act_ab.txt; removed.)
template <int TW, int BN, bool FLIP, class EP>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
conv3x3_winpp_kernel(GemmShape sh, int H, int C, const bf16* __restrict__ x, unsigned xbytes, KMat<bf16> lb, EP ep) {
  // LS >= 0: group 0's last-chunk pieces fetch the row epilogue's operand tile (as
  // conv3x3_win_kernel) into the spare window buffer
  constexpr int LS = LdsSlotTrait<EP>::value;
  using WG = WinGeom<TW, 4, win_minp<EP>()>;   // window pieces over group 0's four waves
  constexpr int BM = 256, WGN = 2, WGM = 4, NTG = 256;
  constexpr int WTN = BN / WGN, MB = 4, NB = WTN / 16;
  constexpr int BSLOT = BN * 64;
  constexpr int PPW = WG::PPW;
  using SB = HStager<BN, KMat<bf16>, NTG>;
  static_assert(PPW <= 16, "group 0's last window piece lands before the next chunk's first read");
  static_assert(2 * WG::SLOT + 4 * BSLOT <= 160 * 1024 && BM * BN * 2 + 4096 <= 2 * WG::SLOT + 4 * BSLOT, "LDS budget");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const win = smem;
  char* const ring = smem + 2 * WG::SLOT;

  const int nwg = sh.tiles_m * sh.tiles_n;
  const int bid = blockIdx.x;
  int g = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = nwg >> 3, rr = nwg & 7;
    g = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int tm = g / sh.tiles_n, tn = g - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int n = row0 / (H * TW), h0 = (row0 - n * H * TW) / TW;
  const int NC = C / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / WGN, wn = wv - wm * WGN;
  const int grp = wv >> 2, wg = wv & 3;
  const int li = lane & 15, lg = lane >> 4;
  const rsrc_t rx = buf_rsrc(x, xbytes);
  const rsrc_t rb = lb.rsrc();
  const rsrc_t rz = null_rsrc(zero_page());
  rsrc_t rop = rz;
  if constexpr (LS >= 0) rop = buf_rsrc(ep.lds_operand(), (unsigned)((size_t)sh.M * sh.N * 2));

  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};
  const int aoff = li * WG::PS + lg * 16;
  const int wpx = wm * 64;
  const char* const bbase = ring + li * 64 + (pp_chunk(li, lg) << 4) + wn * WTN * 64;
  // fragments of half-step (tap t, half hh) of window buffer wb, ring slot sl
  auto mma = [&](auto sc_, const char* wb, int sl) __attribute__((always_inline)) {
    constexpr int S = decltype(sc_)::value;
    constexpr int T = S >> 1, HH = S & 1;
    constexpr int KH = FLIP ? 2 - T / 3 : T / 3, KW = FLIP ? 2 - T % 3 : T % 3;
    v8bf fa[MB], fb[NB];
#pragma unroll
    for (int a = 0; a < MB; ++a) {
      const int px = wpx + a * 16;
      const int wrow = px / TW + KH, wcol = px % TW;
      fa[a] = *reinterpret_cast<const v8bf*>(wb + aoff + (wrow * WG::WC + wcol + KW) * WG::PS + HH * 64);
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) fb[b] = *reinterpret_cast<const v8bf*>(bbase + sl * BSLOT + b * 16 * 64);
    __builtin_amdgcn_sched_barrier(0);
    raw_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#if VLP_PP_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
#if VLP_PP_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    __builtin_amdgcn_sched_barrier(0);
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;

  auto run = [&](auto gc) __attribute__((always_inline)) {
    constexpr int G = decltype(gc)::value;
    // group 0: window pieces; group 1: B half-tiles (each holds only its own loader state)
    unsigned woff[G == 0 ? PPW : 1];
    SB sb;
    if constexpr (G == 0) {
#pragma unroll
      for (int i = 0; i < PPW; ++i) {
        const int off = (wg * PPW + i) * 1024 + lane * 16;
        const int p = off / WG::PS, c = (off - p * WG::PS) >> 4;
        const int wr = p / WG::WC, wc = p - wr * WG::WC;
        const int hh = h0 - 1 + wr, ww = wc - 1;
        const bool ok = c < 8 && p < WG::WR * WG::WC && hh >= 0 && hh < H && ww >= 0 && ww < TW;
        woff[i] = ok ? (unsigned)((((n * H + hh) * TW + ww) * C) * 2 + c * 16) : kOOB;
      }
#pragma unroll
      for (int i = 0; i < PPW; ++i) dma16(rx, woff[i], win + (wg * PPW + i) * 1024);
      wait_vmcnt<0>();
    } else {
      sb.init(lb, col0, 0, wg);
      sb.template issue<0>(lb, rb, 0, ring, wg);
      sb.template issue<1>(lb, rb, 0, ring + BSLOT, wg);
      sb.template issue<0>(lb, rb, C, ring + 2 * BSLOT, wg);
      wait_vmcnt<2 * SB::P>();
    }
    raw_barrier();
    if constexpr (G == 1) raw_barrier();   // the stagger
    __builtin_amdgcn_sched_barrier(0);
    auto chunk = [&](auto pc, int cc) __attribute__((always_inline)) {
      constexpr int PC = decltype(pc)::value;
      const char* const wbuf = win + PC * WG::SLOT;
      char* const wnext = win + (1 - PC) * WG::SLOT;
      static_for<0, 18>([&](auto sc_) {
        constexpr int S = decltype(sc_)::value;
        constexpr int SL = (S + 2 * PC) & 3;
        if constexpr (G == 0) {
          wait_vmcnt<(S >= 2 && S <= PPW + 1) ? 1 : 0>();   // pieces of half-step S-2 landed
        } else {
          wait_vmcnt<SB::P>();                           // B(u+1) landed
        }
        __builtin_amdgcn_sched_barrier(0);
        raw_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (G == 0) {
          if constexpr (S >= 1 && S <= PPW) {
            // piece I = S-1 at half-steps 1..PPW: the first write into wnext follows
            // barrier #36c+3, after group 1's lgkmcnt(0) on its last reads of that
            // buffer (chunk c-1, half-step 17, completed before its barrier #36c+2)
            constexpr int I = S >= 1 && S <= PPW ? S - 1 : 0;
            if (LS >= 0 && cc + 1 == NC) {
              const int j = wg * PPW + I, row = j * 4 + (lane >> 4);
              const unsigned o = row < BM ? (unsigned)(((row0 + row) * sh.N + col0) * 2 + (lane & 15) * 16) : kOOB;
              dma16(rop, o, wnext + j * 1024);
            } else {
              dma16(cc + 1 < NC ? rx : rz, woff[I] + (unsigned)(cc + 1) * 128u, wnext + (wg * PPW + I) * 1024);
            }
          }
        } else {
          constexpr int S3 = S + 3 < 18 ? S + 3 : S + 3 - 18;
          const int c3 = S + 3 < 18 ? cc : cc + 1;
          sb.template issue<S3 & 1>(lb, c3 < NC ? rb : rz, (S3 >> 1) * C + c3 * 64, ring + ((SL + 3) & 3) * BSLOT, wg);
        }
        mma(sc_, wbuf, SL);
      });
    };
    for (int cc = 0; cc < NC; cc += 2) {
      chunk(std::integral_constant<int, 0>{}, cc);
      chunk(std::integral_constant<int, 1>{}, cc + 1);
    }
    if constexpr (G == 0) raw_barrier();   // matches group 1's stagger barrier
  };
  if (grp == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 1>{});
  wait_vmcnt<0>();
  __syncthreads();
  if constexpr (LS >= 0) {
    ms_epilogue<BM, BN, WGM, WGN, EP, true>(sh, ep, acc, row0, col0, g, wm, wn, smem + WG::SLOT, smem);
  } else {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep, acc, row0, col0, g, wm, wn, smem);
  }
}
template <int TW, bool FLIP, class EP>
static int launch_winpp_t(const ConvGeom& g, int cin, int nout, const void* x, const void* w, const EP& ep,
                          hipStream_t st) {
  constexpr int BN = 128;
  constexpr int lds = 2 * WinGeom<TW, 4, win_minp<EP>()>::SLOT + 4 * BN * 64;
  static KernelDevState kst;
  const int e = prepare_kernel(kst, (const void*)&conv3x3_winpp_kernel<TW, BN, FLIP, EP>, lds, 0, nullptr);
  if (e) return e;
  GemmShape sh;
  sh.M = g.N * g.H * g.W;
  sh.N = nout;
  sh.K = 9 * cin;
  sh.kchunk = sh.K;
  sh.tiles_m = sh.M / 256;
  sh.tiles_n = nout / BN;
  sh.xsplit = 0;
  sh.dbg = 0;
  sh.nsplit = 1;
  KMat<bf16> lb{(const bf16*)w, sh.K, nout, sh.K};
  hipLaunchKernelGGL((conv3x3_winpp_kernel<TW, BN, FLIP, EP>), dim3(sh.tiles_m * sh.tiles_n), dim3(512), lds, st,
                     sh, g.H, cin, (const bf16*)x, (unsigned)((size_t)g.N * g.H * g.W * cin * 2), lb, ep);
  return (int)hipGetLastError();
}

// 3x3 / stride 1 / pad 1 with C and the GEMM N both multiples of 128, 256-pixel
// tiles of whole rows, widths 16 / 32 / 64 (ResNet34 layers 2-4 at 512 x 512)
// image widths routed to the window kernel (bit W / 16): r5 A/B at the bench
// shapes (profiles/r5w_window_ab.txt) -- layer 2 (W 64) -8..-16 %, layer 4 (W 16)
// -1..-3 %, layer 3 (W 32) +1..+7 % against the 256 x 256 ping-pong tiles
#ifndef VLP_WIN_WIDTHS
#define VLP_WIN_WIDTHS ((1 << 1) | (1 << 4))
#endif
static bool win_ok(const ConvGeom& g, int cin, int nout, int widths = VLP_WIN_WIDTHS) {
  return g.KH == 3 && g.KW == 3 && g.S == 1 && g.P == 1 && (g.W == 16 || g.W == 32 || g.W == 64) &&
         ((widths >> (g.W / 16)) & 1) &&
         g.H % (256 / g.W) == 0 && cin % 128 == 0 && nout % 128 == 0 &&
         // 32-bit offsets into the input AND the [M][nout] epilogue operands / outputs
         (size_t)g.N * g.H * g.W * (cin > nout ? cin : nout) * 2 < (1ull << 31);
}
#ifndef VLP_WIN
#define VLP_WIN 1   // the LDS-window kernel for the 3x3 stride-1 GEMMs of layers 2-4 (0: im2col GEMMs)
#endif
template <bool FLIP, class EP>
static int launch_win(const ConvGeom& g, int cin, int nout, const void* x, const void* w, const EP& ep,
                      hipStream_t st) {
  if (g.W == 64) return launch_winpp_t<64, FLIP>(g, cin, nout, x, w, ep, st);
  if (g.W == 32) return launch_winpp_t<32, FLIP>(g, cin, nout, x, w, ep, st);
  return launch_winpp_t<16, FLIP>(g, cin, nout, x, w, ep, st);
}

#ifndef VLP_FWD_BN_PP
#define VLP_FWD_BN_PP 1   // bf16 BN-on-load forward on the ping-pong kernel (fragment transform)
#endif
template <typename T>
static int conv_fwd_t(const void* x, const void* wp, void* y, ConvGeom g, const float* sc,
                      const float* sh, double* s1, double* s2, int rep, hipStream_t st) {
  g.M = g.N * g.Ho * g.Wo;
  g.K = g.KH * g.KW * g.C;
  KMat<T> lb{(const T*)wp, g.K, g.Co, g.K};
  EpiConvFwd<T> ep{s1, s2, rep, (T*)y, g.Co};
  if (sc) {
#if VLP_FWD_BN_PP
    if constexpr (std::is_same<T, bf16>::value) {
      if (g.C % 64 == 0 && g.C <= 512 && g.M >= 256 && g.Co >= 256) {
        ConvFwdABn la{{g, (const bf16*)x, sc, sh}};
        return launch_gemm_pp<256, 256, 2, 4>(g.M, g.Co, g.K, 1, la, lb, ep, st);
      }
    }
#endif
    ConvFwdA<T, true> la{g, (const T*)x, sc, sh};
    return gemm_auto<T>(g.M, g.Co, g.K, 1, la, lb, ep, st);
  }
  ConvFwdA<T, false> la{g, (const T*)x, nullptr, nullptr};
  if constexpr (std::is_same<T, bf16>::value) {
    if (rows_c64_ok(g)) return launch_rows_c64(g, x, wp, 0, ep, st);
    if (VLP_WIN && win_ok(g, g.C, g.Co)) return launch_win<false>(g, g.C, g.Co, x, wp, ep, st);
    // the LDS-DMA loaders take ONE filter tap per 64-deep K-step; a channel
    // count that is not a multiple of 64 (NesT's 96-channel ConvPool input)
    // takes the register-staged engine, which resolves the tap per 16-B chunk
    if (g.C % 64) {
      ConvFwdAReg<T> lr{la};
      return launch_gemm<T, 128, 128, 2>(g.M, g.Co, g.K, 1, lr, lb, ep, st);
    }
  }
  return gemm_auto<T>(g.M, g.Co, g.K, 1, la, lb, ep, st);
}

template <typename T>
static int conv_dgrad_t(const void* dy, const void* wt, void* dx, ConvGeom g, const void* addend,
                        const void* ybn, const float* sc, const float* sh, const float* mean,
                        const float* invstd, double* s1, double* s2, int rep, hipStream_t st) {
  g.M = g.N * g.H * g.W;
  g.K = g.KH * g.KW * g.Co;
  if (std::is_same<T, bf16>::value && g.Co % 64) return (int)hipErrorInvalidValue;   // one tap per K-step
  if (g.S == 2) {
    // four parity classes, each a dense GEMM over its valid taps only
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        S2Class c = make_s2class(g, ph, pw);
        const int Mc = g.N * c.Hc * c.Wc, Kc = c.nth * c.ntw * g.Co;
        if (Mc <= 0) continue;
        ConvDgradS2A<T> la{g, c, (const T*)dy, Mc, Kc};
        WtS2B<T> lb{(const T*)wt, g, c, Kc};
        int r;
        if (ybn) {
          EpiDgradBN<T> in{s1, s2, rep, (T*)dx, g.C, (const T*)ybn, sc, sh, mean, invstd};
          EpiS2Remap<EpiDgradBN<T>> ep{s1, s2, rep, in, c, g.H, g.W};
          r = gemm_s2<T>(Mc, g.C, Kc, la, lb, ep, st);
        } else {
          EpiDgradAdd<T> in{nullptr, nullptr, (T*)dx, (const T*)addend, g.C};
          EpiS2Remap<EpiDgradAdd<T>> ep{nullptr, nullptr, 1, in, c, g.H, g.W};
          r = gemm_s2<T>(Mc, g.C, Kc, la, lb, ep, st);
        }
        if (r) return r;
      }
    return 0;
  }
  ConvDgradA<T> la{g, (const T*)dy};
  KMat<T> lb{(const T*)wt, g.K, g.C, g.K};
  // stride-1 dgrad = forward conv of dy with the flipped, transposed filter
  const bool rows = std::is_same<T, bf16>::value && rows_c64_ok(g);
  const bool win = std::is_same<T, bf16>::value && VLP_WIN && win_ok(g, g.Co, g.C);
  if (ybn) {
    EpiDgradBN<T> ep{s1, s2, rep, (T*)dx, g.C, (const T*)ybn, sc, sh, mean, invstd};
    if constexpr (std::is_same<T, bf16>::value) {
      if (rows) return launch_rows_c64(g, dy, wt, 1, ep, st);
      if (win) return launch_win<true>(g, g.Co, g.C, dy, wt, ep, st);
    }
    return gemm_auto<T>(g.M, g.C, g.K, 1, la, lb, ep, st);
  }
  EpiDgradAdd<T> ep{nullptr, nullptr, (T*)dx, (const T*)addend, g.C};
  if constexpr (std::is_same<T, bf16>::value) {
    if (rows) return launch_rows_c64(g, dy, wt, 1, ep, st);
    if (win) return launch_win<true>(g, g.Co, g.C, dy, wt, ep, st);
  }
  return gemm_auto<T>(g.M, g.C, g.K, 1, la, lb, ep, st);
}

// dgrad whose output is masked by a ReLU output and reduced for a BN backward
template <typename T, bool BITS>
static int conv_dgrad_relu_impl(const void* dy, const void* wt, void* gout, ConvGeom g0, const void* addend,
                                const void* relu_out, const uint8_t* relu_mask, const void* y, const float* mean,
                                const float* invstd, double* s1, double* s2, int rep, hipStream_t st,
                                long long dd_off = 0, long long wd_off = 0) {
  ConvGeom g = g0;
  g.M = g.N * g.H * g.W;
  g.K = g.KH * g.KW * g.Co;
  EpiDgradRelu<T, BITS> in{s1, s2, rep, (T*)gout, (const T*)addend, g.C, (const T*)relu_out, (const T*)y, mean,
                           invstd, relu_mask};
  if (g.S == 2) {
    for (int ph = 0; ph < 2; ++ph)
      for (int pw = 0; pw < 2; ++pw) {
        S2Class c = make_s2class(g, ph, pw);
        const int Mc = g.N * c.Hc * c.Wc, Kc1 = c.nth * c.ntw * g.Co;
        if (Mc <= 0) continue;
        // the downsample's 1x1/2 data gradient lands on the (0, 0) pixels only
        const bool fold = dd_off && ph == 0 && pw == 0;
        const int Kc = Kc1 + (fold ? g.Co : 0);
        ConvDgradS2A<T> la{g, c, (const T*)dy, Mc, Kc};
        WtS2B<T> lb{(const T*)wt, g, c, Kc};
        if (fold) {
          la.Kc1 = Kc1; la.dd_off = dd_off;
          lb.Kc1 = Kc1; lb.wd_off = wd_off;
        }
        EpiS2Remap<EpiDgradRelu<T, BITS>> ep{s1, s2, rep, in, c, g.H, g.W};
        const int r = gemm_s2<T>(Mc, g.C, Kc, la, lb, ep, st);
        if (r) return r;
      }
    return 0;
  }
  if constexpr (std::is_same<T, bf16>::value) {
    if (rows_c64_ok(g)) return launch_rows_c64(g, dy, wt, 1, in, st);
    if (VLP_WIN && win_ok(g, g.Co, g.C)) return launch_win<true>(g, g.Co, g.C, dy, wt, in, st);
  }
  ConvDgradA<T> la{g, (const T*)dy};
  KMat<T> lb{(const T*)wt, g.K, g.C, g.K};
  return gemm_auto<T>(g.M, g.C, g.K, 1, la, lb, in, st);
}
template <typename T>
static int conv_dgrad_relu_t(const void* dy, const void* wt, void* gout, ConvGeom g0, const void* addend,
                             const void* relu_out, const uint8_t* relu_mask, const void* y, const float* mean,
                             const float* invstd, double* s1, double* s2, int rep, hipStream_t st) {
  if (relu_mask)
    return conv_dgrad_relu_impl<T, true>(dy, wt, gout, g0, addend, relu_out, relu_mask, y, mean, invstd, s1, s2,
                                         rep, st);
  return conv_dgrad_relu_impl<T, false>(dy, wt, gout, g0, addend, relu_out, relu_mask, y, mean, invstd, s1, s2,
                                        rep, st);
}

template <typename T>
static int conv_wgrad_t(const void* dy, const void* x, float* dw, ConvGeom g, const float* sc,
                        const float* sh, hipStream_t st) {
  g.M = g.N * g.Ho * g.Wo;        // pixels (reduction)
  g.K = g.KH * g.KW * g.C;        // columns
  MNMat<T> la{(const T*)dy, g.Co, g.Co, g.M};
  EpiAtomic ep{nullptr, nullptr, dw, g.K, 1.0f};
  if (sc) {
    ConvWgradB<T, true> lb{g, (const T*)x, sc, sh, g.K, make_pixstep(g, Elem<T>::BK)};
    return gemm_wgrad<T>(g.Co, g.K, g.M, la, lb, ep, st);
  }
  ConvWgradB<T, false> lb{g, (const T*)x, nullptr, nullptr, g.K, make_pixstep(g, Elem<T>::BK)};
  return gemm_wgrad<T>(g.Co, g.K, g.M, la, lb, ep, st);
}

// Weight gradient straight into the parameter's [Co][C][KH][KW] layout: the
// GEMM's K-splits write fp32 slabs ws[s][Co][KH*KW*C] (EpiSplitStore) and one
// fold pass sums them and transposes.  Thread per slab element: reads are
// coalesced over c with 4 independent slab streams in flight per thread; the
// transposing writes (stride KH*KW) merge in L2.
__global__ void wgrad_fold_kernel(int Co, int C, int T, int ks, size_t slab, const float* __restrict__ ws,
                                  float* __restrict__ g) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= slab) return;
  const float* p = ws + i;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int s = 0;
  for (; s + 4 <= ks; s += 4) {
    a0 += p[(size_t)s * slab];
    a1 += p[(size_t)(s + 1) * slab];
    a2 += p[(size_t)(s + 2) * slab];
    a3 += p[(size_t)(s + 3) * slab];
  }
  for (; s < ks; ++s) a0 += p[(size_t)s * slab];
  const int c = (int)(i % C);
  const size_t r = i / C;
  const int t = (int)(r % T), co = (int)(r / T);
  g[((size_t)co * C + c) * T + t] = (a0 + a1) + (a2 + a3);
}

// r6: one workgroup per output channel row (T * C floats): every split slab read
// as 16-B vectors (the per-element kernel above issued 4-B loads), the same
// per-element summation order (s mod 4 partials, (a0 + a1) + (a2 + a3)), and the
// [t][c] -> [c][t] transpose staged in LDS so the gradient row is written
// contiguously.  Rows up to kFoldRowMax floats (layer 4: 9 * 512).
constexpr int kFoldRowMax = 9 * 512;
#ifndef VLP_FOLD_ROW
#define VLP_FOLD_ROW 1   // 0: the per-element fold (wgrad_fold_kernel) for every conv
#endif
__global__ void __launch_bounds__(256) wgrad_fold_row_kernel(int C, int T, int ks, size_t slab,
                                                              const float* __restrict__ ws, float* __restrict__ g) {
  __shared__ float row[kFoldRowMax];
  const int L = C * T;
  const size_t base = (size_t)blockIdx.x * L;
  for (int e = threadIdx.x * 4; e < L; e += 1024) {
    const float* p = ws + base + e;
    v4f a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    int s = 0;
    // 16 slabs' loads in flight per thread (the layer-1 folds reduce ~85 slabs with
    // 64 workgroups: latency-bound), added in the same per-element order
    for (; s + 16 <= ks; s += 16) {
      v4f t[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) t[j] = *reinterpret_cast<const v4f*>(p + (size_t)(s + j) * slab);
#pragma unroll
      for (int j = 0; j < 16; j += 4) {
        a0 += t[j];
        a1 += t[j + 1];
        a2 += t[j + 2];
        a3 += t[j + 3];
      }
    }
    for (; s + 4 <= ks; s += 4) {
      a0 += *reinterpret_cast<const v4f*>(p + (size_t)s * slab);
      a1 += *reinterpret_cast<const v4f*>(p + (size_t)(s + 1) * slab);
      a2 += *reinterpret_cast<const v4f*>(p + (size_t)(s + 2) * slab);
      a3 += *reinterpret_cast<const v4f*>(p + (size_t)(s + 3) * slab);
    }
    for (; s < ks; ++s) a0 += *reinterpret_cast<const v4f*>(p + (size_t)s * slab);
    const v4f v = (a0 + a1) + (a2 + a3);
#pragma unroll
    for (int j = 0; j < 4; ++j) row[e + j] = v[j];   // slab order: e = t * C + c
  }
  __syncthreads();
  for (int o = threadIdx.x; o < L; o += 256) {       // gradient order: o = c * T + t
    const int c = o / T, t = o - c * T;
    g[base + o] = row[t * C + c];
  }
}

#ifndef VLP_WGRAD_SLOT_DIV
#define VLP_WGRAD_SLOT_DIV 1   // weight-gradient split count sized for 1/DIV of the chip's slots
#endif
template <typename T>
static int conv_wgrad_ws_t(const void* dy, const void* x, float* ws, long long ws_floats, int* ks_out, ConvGeom g,
                           hipStream_t st) {
  g.M = g.N * g.Ho * g.Wo;
  g.K = g.KH * g.KW * g.C;
  const size_t slab = (size_t)g.Co * g.K;
  const long long fit = ws_floats > 0 ? ws_floats / (long long)slab : 0;
  const int max_ks = (int)(fit < 4096 ? fit : 4096);
  if (max_ks < 1) return (int)hipErrorInvalidValue;
  int ks = 1;
  bool split_store = false;
  if constexpr (std::is_same<T, bf16>::value) {
    // layer 1: the row-streaming kernel, one slab per workgroup
    if (wgrad_rows_ok(g)) return launch_wgrad_rows(g, dy, x, ws, max_ks, ks_out, st);
    // tile engines whose epilogue honours per-split output slabs
    if (gemm_variant() >= 5 && g.K % 4 == 0) {
      constexpr int mink5 = 2048;
      int mink = g.Co <= 64 ? 2048 : mink5;
      const int need = (g.M + max_ks - 1) / max_ks;
      if (mink < need) mink = need;
      static_assert(use_bk<bf16, MNMat<bf16>, ConvWgradB<bf16, false>>(),
                    "split slabs need the bk / big engines");
      MNMat<bf16> la{(const bf16*)dy, g.Co, g.Co, g.M};
      ConvWgradB<bf16, false> lb{g, (const bf16*)x, nullptr, nullptr, g.K, make_pixstep(g, Elem<bf16>::BK)};
      EpiSplitStore ep{nullptr, nullptr, ws, g.K, slab};
      ksplit_slot_div() = VLP_WGRAD_SLOT_DIV;
      const int r = g.Co <= 64 ? gemm_short<bf16>(g.Co, g.K, g.M, -mink, la, lb, ep, st)
                               : gemm_conv_wide<bf16>(g.Co, g.K, g.M, -mink, la, lb, ep, st);
      ksplit_slot_div() = 1;
      if (r) return r;
      ks = last_ksplit();
      if (ks > max_ks) return (int)hipErrorInvalidValue;   // would have overrun the workspace
      split_store = true;
    }
  }
  if (!split_store) {   // other engines: atomics into slab 0
    if (hipMemsetAsync(ws, 0, slab * sizeof(float), st) != hipSuccess) return (int)hipGetLastError();
    const int r = conv_wgrad_t<T>(dy, x, ws, g, nullptr, nullptr, st);
    if (r) return r;
  }
  *ks_out = ks;
  return 0;
}

static StemGeom make_stem(int N, int H, int W) {
  StemGeom g;
  g.N = N;
  g.Ho = (H + 6 - 7) / 2 + 1;
  g.Wo = (W + 6 - 7) / 2 + 1;
  g.Hp = 2 * g.Ho + 6;
  g.Wp = 2 * g.Wo + 6;
  g.M = N * g.Ho * g.Wo;
  g.fd_howo = make_fastdiv(g.Ho * g.Wo);
  g.fd_wo = make_fastdiv(g.Wo);
  return g;
}

// NCHW (3 ch, fp32) -> padded NHWC4 image of type T (interior only; the
// caller zeroes the buffer once so the padding stays zero).
template <typename T>
__global__ void stem_prep_kernel(const float* __restrict__ x, T* __restrict__ xp, int N, int H, int W,
                                 int Hp, int Wp) {
  size_t total = (size_t)N * H * W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    int w = (int)(i % W);
    size_t t = i / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    const float* src = x + (size_t)n * 3 * H * W + (size_t)h * W + w;
    T* dst = xp + (((size_t)n * Hp + h + 3) * Wp + w + 3) * 4;
    dst[0] = from_f<T>(src[0]);
    dst[1] = from_f<T>(src[(size_t)H * W]);
    dst[2] = from_f<T>(src[(size_t)2 * H * W]);
    dst[3] = from_f<T>(0.f);
  }
}
// 1-channel uint8 radiograph -> normalised, replicated padded NHWC4 image
// (the on-device half of the pinned-uint8 collation path).
template <typename T>
__global__ void stem_prep_u8_kernel(const uint8_t* __restrict__ x, T* __restrict__ xp, int N, int H,
                                    int W, int Hp, int Wp, float mean, float inv_std) {
  size_t total = (size_t)N * H * W;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    int w = (int)(i % W);
    size_t t = i / W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float v = ((float)x[i] - mean) * inv_std;
    T* dst = xp + (((size_t)n * Hp + h + 3) * Wp + w + 3) * 4;
    T tv = from_f<T>(v);
    dst[0] = tv; dst[1] = tv; dst[2] = tv; dst[3] = from_f<T>(0.f);
  }
}

// uint8 [N][1][H][W] -> normalised single-channel padded image in 4 shifted copies
// (Xs[s][n][h][j] = Xpad[n][h][j + 2s], Xpad = the image at (3, 3), zeros around);
// one thread per 8 output elements, every element written (no pre-zeroing)
template <typename T>
__global__ void stem1_prep_u8_kernel(const uint8_t* __restrict__ x, T* __restrict__ xs, Stem1Geom g, int H, int W,
                                     float mean, float inv_std) {
  // 32-bit index math (the host bounds 4 * copy elements below 2^31): the 64-bit
  // divisions of a size_t grid-stride loop dominated this copy-rate kernel
  const unsigned rows = 4u * (unsigned)g.N * (unsigned)g.Hp;
  const unsigned cpr = (unsigned)g.Wp1 / 8u;
  const unsigned total = rows * cpr;
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const unsigned row = i / cpr;
    const int c = (int)(i - row * cpr);
    const unsigned t = row / (unsigned)g.Hp;
    const int hp = (int)(row - t * (unsigned)g.Hp);
    const unsigned sh = t / (unsigned)g.N;
    const int n = (int)(t - sh * (unsigned)g.N);
    const int h = hp - 3;
    const bool hin = h >= 0 && h < H;
    const uint8_t* xr = x + ((size_t)n * H + (hin ? h : 0)) * W;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int w = c * 8 + j + 2 * (int)sh - 3;
      v[j] = (hin && w >= 0 && w < W) ? ((float)xr[w] - mean) * inv_std : 0.f;
    }
    T* dst = xs + (size_t)row * g.Wp1 + c * 8;
    if constexpr (sizeof(T) == 2) {
      stg16(dst, Chunk<bf16>::pack(v));
    } else {
      stg16(dst, Chunk<float>::pack(v));
      stg16(dst + 4, Chunk<float>::pack(v + 4));
    }
  }
}
// stem [64][3][7][7] -> W1[64][kh:8][kw:8] = sum over the 3 channels (zeros outside)
template <typename T>
__global__ void pack_stem1_kernel(const float* __restrict__ w, T* __restrict__ wp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 64) return;
  const int co = i >> 6, kh = (i >> 3) & 7, kw = i & 7;
  float v = 0.f;
  if (kh < 7 && kw < 7)
    v = w[((co * 3 + 0) * 7 + kh) * 7 + kw] + w[((co * 3 + 1) * 7 + kh) * 7 + kw] + w[((co * 3 + 2) * 7 + kh) * 7 + kw];
  wp[i] = from_f<T>(v);
}
// slabs [ks][64][64] of d/dW1 -> the parameter's [64][3][7][7] gradient: the three
// channels carry identical images, so each receives the same gradient
__global__ void __launch_bounds__(256) stem1_wgrad_fold_kernel(int ks, const float* __restrict__ ws,
                                                               float* __restrict__ g) {
  __shared__ float part[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;   // e < 64 * 64
  const float* p = ws + e;
  float a0 = 0.f, a1 = 0.f;
  int s = grp;
  for (; s + 4 < ks; s += 8) { a0 += p[(size_t)s * 64 * 64]; a1 += p[(size_t)(s + 4) * 64 * 64]; }
  if (s < ks) a0 += p[(size_t)s * 64 * 64];
  part[grp][threadIdx.x & 63] = a0 + a1;
  __syncthreads();
  if (grp == 0) {
    const int co = e >> 6, kh = (e >> 3) & 7, kw = e & 7;
    if (kh < 7 && kw < 7) {
      const int l = threadIdx.x & 63;
      const float v = (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
#pragma unroll
      for (int c = 0; c < 3; ++c) g[((co * 3 + c) * 7 + kh) * 7 + kw] = v;
    }
  }
}

}  // namespace vlp

using namespace vlp;

VLP_EXPORT int vlp_conv_fwd(int dtype, const void* x, const void* wp, void* y, int N, int H, int W,
                            int C, int Co, int KH, int KW, int S, int P, const float* in_scale,
                            const float* in_shift, double* stat_sum, double* stat_sumsq,
                            int stat_rep, void* stream) {
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    return conv_fwd_t<bf16>(x, wp, y, g, in_scale, in_shift, stat_sum, stat_sumsq, stat_rep, st);
  return conv_fwd_t<float>(x, wp, y, g, in_scale, in_shift, stat_sum, stat_sumsq, stat_rep, st);
}

VLP_EXPORT int vlp_conv_fwd_act_ok(int dtype, int N, int H, int W, int C, int Co, int KH, int KW, int S,
                                  int P) {
  if (dtype != VLP_BF16 || N < 1) return 0;
  const ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  return rows_c64_ok(g) ? 1 : 0;
}

VLP_EXPORT int vlp_conv_fwd_act(int dtype, const void* x, const void* wp, void* y, void* x_act, int N,
                                int H, int W, int C, int Co, int KH, int KW, int S, int P,
                                const float* in_scale, const float* in_shift, double* stat_sum,
                                double* stat_sumsq, int stat_rep, void* stream) {
  if (!vlp_conv_fwd_act_ok(dtype, N, H, W, C, Co, KH, KW, S, P) || !in_scale || !in_shift || !x_act ||
      !stat_sum || !stat_sumsq)
    return (int)hipErrorInvalidValue;
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  g.M = g.N * g.Ho * g.Wo;
  g.K = g.KH * g.KW * g.C;
  EpiConvFwd<bf16> ep{stat_sum, stat_sumsq, stat_rep, (bf16*)y, g.Co};
  RowsXIn xin{};
  xin.t0 = in_scale;
  xin.t1 = in_shift;
  xin.out = (bf16*)x_act;
  return launch_rows_c64<EpiConvFwd<bf16>, 1>(g, x, wp, 0, ep, (hipStream_t)stream, xin);
}

// Layer-1 data gradients with the BN backward of their input folded into the
// rows kernel's ring (XF = 2): g_in is the BN output gradient, y_in the BN
// input; dy_out receives dy = k*g + b*y + c (the weight gradient's operand).
static RowsXIn rows_bwd_xin(const void* y_in, const float* in_coef, void* dy_out) {
  RowsXIn xin{};
  xin.t0 = in_coef;
  xin.y = (const bf16*)y_in;
  xin.out = (bf16*)dy_out;
  return xin;
}

VLP_EXPORT int vlp_conv_dgrad_act_ok(int dtype, int N, int H, int W, int C, int Co, int KH, int KW, int S,
                                    int P) {
  return dtype == VLP_BF16 && N >= 1 && rows_c64_ok(make_geom(N, H, W, C, Co, KH, KW, S, P)) ? 1 : 0;
}

VLP_EXPORT int vlp_conv_dgrad_bn_act(int dtype, const void* g_in, const void* y_in, const float* in_coef,
                                     void* dy_out, const void* wt, void* dx, int N, int H,
                                     int W, int C, int Co, int KH, int KW, int S, int P, const void* y_bn,
                                     const float* bn_scale, const float* bn_shift, const float* bn_mean,
                                     const float* bn_invstd, double* stat1, double* stat2, int stat_rep,
                                     void* stream) {
  if (!vlp_conv_dgrad_act_ok(dtype, N, H, W, C, Co, KH, KW, S, P) || !g_in || !y_in || !dy_out || !in_coef ||
      !y_bn || !bn_scale || !bn_shift || !bn_mean || !bn_invstd || !stat1 || !stat2)
    return (int)hipErrorInvalidValue;
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  g.M = g.N * g.H * g.W;
  g.K = g.KH * g.KW * g.Co;
  EpiDgradBN<bf16> ep{stat1, stat2, stat_rep, (bf16*)dx, g.C, (const bf16*)y_bn, bn_scale, bn_shift, bn_mean,
                      bn_invstd};
  return launch_rows_c64<EpiDgradBN<bf16>, 2>(g, g_in, wt, 1, ep, (hipStream_t)stream,
                                              rows_bwd_xin(y_in, in_coef, dy_out));
}

VLP_EXPORT int vlp_conv_dgrad_relu_act(int dtype, const void* g_in, const void* y_in, const float* in_coef,
                                       void* dy_out, const void* wt, void* gout, int N,
                                       int H, int W, int C, int Co, int KH, int KW, int S, int P,
                                       const void* addend, const void* relu_out, const uint8_t* relu_mask,
                                       const void* y, const float* mean, const float* invstd, double* stat1,
                                       double* stat2, int stat_rep, void* stream) {
  if (!vlp_conv_dgrad_act_ok(dtype, N, H, W, C, Co, KH, KW, S, P) || !g_in || !y_in || !dy_out || !in_coef ||
      (relu_out == nullptr) == (relu_mask == nullptr) || !y ||
      !mean || !invstd || !stat1 || !stat2)
    return (int)hipErrorInvalidValue;
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  g.M = g.N * g.H * g.W;
  g.K = g.KH * g.KW * g.Co;
  const RowsXIn xin = rows_bwd_xin(y_in, in_coef, dy_out);
  hipStream_t st = (hipStream_t)stream;
  if (relu_mask) {
    EpiDgradRelu<bf16, true> ep{stat1, stat2, stat_rep, (bf16*)gout, (const bf16*)addend, g.C,
                                (const bf16*)relu_out, (const bf16*)y, mean, invstd, relu_mask};
    return launch_rows_c64<EpiDgradRelu<bf16, true>, 2>(g, g_in, wt, 1, ep, st, xin);
  }
  EpiDgradRelu<bf16, false> ep{stat1, stat2, stat_rep, (bf16*)gout, (const bf16*)addend, g.C,
                               (const bf16*)relu_out, (const bf16*)y, mean, invstd, relu_mask};
  return launch_rows_c64<EpiDgradRelu<bf16, false>, 2>(g, g_in, wt, 1, ep, st, xin);
}

VLP_EXPORT int vlp_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int N, int H,
                              int W, int C, int Co, int KH, int KW, int S, int P,
                              const void* addend, const void* y_bn, const float* bn_scale,
                              const float* bn_shift, const float* bn_mean,
                              const float* bn_invstd, double* stat1, double* stat2,
                              int stat_rep, void* stream) {
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    return conv_dgrad_t<bf16>(dy, wt, dx, g, addend, y_bn, bn_scale, bn_shift, bn_mean, bn_invstd,
                              stat1, stat2, stat_rep, st);
  return conv_dgrad_t<float>(dy, wt, dx, g, addend, y_bn, bn_scale, bn_shift, bn_mean, bn_invstd,
                             stat1, stat2, stat_rep, st);
}

VLP_EXPORT int vlp_conv_dgrad_relu(int dtype, const void* dy, const void* wt, void* g, int N, int H,
                                   int W, int C, int Co, int KH, int KW, int S, int P,
                                   const void* addend, const void* relu_out, const uint8_t* relu_mask,
                                   const void* y, const float* mean, const float* invstd, double* stat1,
                                   double* stat2, int stat_rep, void* stream) {
  ConvGeom geo = make_geom(N, H, W, C, Co, KH, KW, S, P);
  hipStream_t st = (hipStream_t)stream;
  if ((relu_out == nullptr) == (relu_mask == nullptr) || C % 8) return (int)hipErrorInvalidValue;
  if (dtype == VLP_BF16)
    return conv_dgrad_relu_t<bf16>(dy, wt, g, geo, addend, relu_out, relu_mask, y, mean, invstd, stat1, stat2,
                                   stat_rep, st);
  return conv_dgrad_relu_t<float>(dy, wt, g, geo, addend, relu_out, relu_mask, y, mean, invstd, stat1, stat2,
                                  stat_rep, st);
}

// The second block of layers 2-4: conv1's data gradient (+ the identity
// gradient) through the previous block's output ReLU (sign bits) with that
// block's bn2 AND downsample-BN backward sums in the epilogue (EpiDgradRelu2).
VLP_EXPORT int vlp_conv_dgrad_relu2(int dtype, const void* dy, const void* wt, void* g, int N, int H, int W, int C,
                                    int Co, int KH, int KW, int S, int P, const void* addend,
                                    const uint8_t* relu_mask, const void* y, const float* mean, const float* invstd,
                                    const void* yd, const float* meand, const float* invstdd, double* stat1,
                                    double* stat2, double* stat3, int stat_rep, void* stream) {
  ConvGeom g0 = make_geom(N, H, W, C, Co, KH, KW, S, P);
  // row-chunk epilogue kernels only: bf16 LDS-DMA engine, stride 1, N = C >= 128, K a multiple of 64
  if (dtype != VLP_BF16 || gemm_variant() < 5 || S != 1 || C < 128 || C % 64 || Co % 64 || !relu_mask || !y ||
      !yd || !mean || !invstd || !meand || !invstdd || !stat1 || !stat2 || !stat3)
    return (int)hipErrorInvalidValue;
  ConvGeom g1 = g0;
  g1.M = g1.N * g1.H * g1.W;
  g1.K = g1.KH * g1.KW * g1.Co;
  EpiDgradRelu2<bf16> ep{stat1, stat2, stat_rep, stat3, (bf16*)g, (const bf16*)addend, g1.C, relu_mask,
                         (const bf16*)y, (const bf16*)yd, mean, invstd, meand, invstdd};
  if (VLP_WIN && win_ok(g1, g1.Co, g1.C)) return launch_win<true>(g1, g1.Co, g1.C, dy, wt, ep, (hipStream_t)stream);
  ConvDgradA<bf16> la{g1, (const bf16*)dy};
  KMat<bf16> lb{(const bf16*)wt, g1.K, g1.C, g1.K};
  return gemm_auto<bf16>(g1.M, g1.C, g1.K, 1, la, lb, ep, (hipStream_t)stream);
}

// Stride-2 block entry (layers 2-4, block 0): conv1's 3x3/2 data gradient with the
// 1x1/2 downsample's data gradient folded into parity class (0, 0) as extra K-steps
// (replaces vlp_conv_dgrad of the downsample + the addend of vlp_conv_dgrad_relu).
// dyd must follow dy in one allocation (dyd = dy + N*Ho*Wo*Co) and wtd must follow
// wt (wtd = wt + C*KH*KW*Co); bf16 only.
VLP_EXPORT int vlp_conv_dgrad_relu_ds(int dtype, const void* dy, const void* dyd, const void* wt, const void* wtd,
                                      void* g, int N, int H, int W, int C, int Co, int KH, int KW, int S, int P,
                                      const void* relu_out, const uint8_t* relu_mask, const void* y,
                                      const float* mean, const float* invstd, double* stat1, double* stat2,
                                      int stat_rep, void* stream) {
  ConvGeom geo = make_geom(N, H, W, C, Co, KH, KW, S, P);
  const long long dd = (long long)geo.N * geo.Ho * geo.Wo * geo.Co, wd = (long long)C * KH * KW * Co;
  if (dtype != VLP_BF16 || S != 2 || KH != 3 || KW != 3 || P != 1 || C % 8 || Co % 64 ||
      (relu_out == nullptr) == (relu_mask == nullptr) || (const bf16*)dyd != (const bf16*)dy + dd ||
      (const bf16*)wtd != (const bf16*)wt + wd || (size_t)2 * dd * 2 >= (1ull << 32))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (relu_mask)
    return conv_dgrad_relu_impl<bf16, true>(dy, wt, g, geo, nullptr, relu_out, relu_mask, y, mean, invstd, stat1,
                                            stat2, stat_rep, st, dd, wd);
  return conv_dgrad_relu_impl<bf16, false>(dy, wt, g, geo, nullptr, relu_out, relu_mask, y, mean, invstd, stat1,
                                           stat2, stat_rep, st, dd, wd);
}

VLP_EXPORT int vlp_conv_wgrad(int dtype, const void* dy, const void* x, float* dw_ws, int N, int H,
                              int W, int C, int Co, int KH, int KW, int S, int P,
                              const float* in_scale, const float* in_shift, void* stream) {
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  hipStream_t st = (hipStream_t)stream;
  if ((long long)N * H * W * C >= (1ll << 31)) return (int)hipErrorInvalidValue;   // 32-bit pixel walk
  if (dtype == VLP_BF16) return conv_wgrad_t<bf16>(dy, x, dw_ws, g, in_scale, in_shift, st);
  return conv_wgrad_t<float>(dy, x, dw_ws, g, in_scale, in_shift, st);
}

VLP_EXPORT int vlp_conv_wgrad_ws(int dtype, const void* dy, const void* x, float* split_ws, long long ws_floats,
                                 int* nsplit, int N, int H, int W, int C, int Co, int KH, int KW, int S, int P,
                                 void* stream) {
  ConvGeom g = make_geom(N, H, W, C, Co, KH, KW, S, P);
  hipStream_t st = (hipStream_t)stream;
  if (!nsplit || (long long)N * H * W * C >= (1ll << 31)) return (int)hipErrorInvalidValue;
  if (dtype == VLP_BF16) return conv_wgrad_ws_t<bf16>(dy, x, split_ws, ws_floats, nsplit, g, st);
  return conv_wgrad_ws_t<float>(dy, x, split_ws, ws_floats, nsplit, g, st);
}

VLP_EXPORT int vlp_set_wgrad_rows_min_images(int n, int* prev) {
  if (prev) *prev = g_wgrad_rows_min;
  g_wgrad_rows_min = n < 0 ? -1 : n;
  return 0;
}

VLP_EXPORT int vlp_conv_wgrad_fold(int Co, int C, int KH, int KW, int nsplit, const float* split_ws, float* grad,
                                   void* stream) {
  if (nsplit < 1) return (int)hipErrorInvalidValue;
  const size_t n = (size_t)Co * KH * KW * C;
  if (VLP_FOLD_ROW && C % 4 == 0 && KH * KW * C <= kFoldRowMax && ((uintptr_t)split_ws & 15) == 0) {
    hipLaunchKernelGGL(wgrad_fold_row_kernel, dim3((unsigned)Co), dim3(256), 0, (hipStream_t)stream, C, KH * KW,
                       nsplit, n, split_ws, grad);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(wgrad_fold_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, Co,
                     C, KH * KW, nsplit, n, split_ws, grad);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_stem_prep(int dtype, const float* x, void* xp, int N, int H, int W, void* stream) {
  StemGeom g = make_stem(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  size_t total = (size_t)N * H * W;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(stem_prep_kernel<bf16>, dim3(blocks), dim3(256), 0, st, x, (bf16*)xp, N, H, W, g.Hp, g.Wp);
  else
    hipLaunchKernelGGL(stem_prep_kernel<float>, dim3(blocks), dim3(256), 0, st, x, (float*)xp, N, H, W, g.Hp, g.Wp);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_stem_prep_u8(int dtype, const uint8_t* x, void* xp, int N, int H, int W,
                                float mean, float std, void* stream) {
  StemGeom g = make_stem(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  size_t total = (size_t)N * H * W;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(stem_prep_u8_kernel<bf16>, dim3(blocks), dim3(256), 0, st, x, (bf16*)xp, N, H, W, g.Hp, g.Wp, mean, 1.f / std);
  else
    hipLaunchKernelGGL(stem_prep_u8_kernel<float>, dim3(blocks), dim3(256), 0, st, x, (float*)xp, N, H, W, g.Hp, g.Wp, mean, 1.f / std);
  return (int)hipGetLastError();
}

// Padded-image geometry for the host (so Python allocates the right buffer).
VLP_EXPORT void vlp_stem_geom(int H, int W, int* Ho, int* Wo, int* Hp, int* Wp) {
  StemGeom g = make_stem(1, H, W);
  *Ho = g.Ho; *Wo = g.Wo; *Hp = g.Hp; *Wp = g.Wp;
}

VLP_EXPORT int vlp_stem_fwd(int dtype, const void* xp, const void* wp, void* y, int N, int H, int W,
                            double* stat_sum, double* stat_sumsq, int stat_rep, void* stream) {
  StemGeom g = make_stem(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16) {
    StemA<bf16> la{g, (const bf16*)xp};
    KMat<bf16> lb{(const bf16*)wp, 256, 64, 256};
    EpiConvFwd<bf16> ep{stat_sum, stat_sumsq, stat_rep, (bf16*)y, 64};
    return gemm_narrow<bf16>(g.M, 64, 256, 1, la, lb, ep, st);
  }
  StemA<float> la{g, (const float*)xp};
  KMat<float> lb{(const float*)wp, 256, 64, 256};
  EpiConvFwd<float> ep{stat_sum, stat_sumsq, stat_rep, (float*)y, 64};
  return launch_gemm<float, 256, 64, 4>(g.M, 64, 256, 1, la, lb, ep, st);
}

// dW_ws[64][256] (kh:8, kw:8, c:4 layout), fp32, accumulated atomically.
VLP_EXPORT int vlp_stem_wgrad(int dtype, const void* dy, const void* xp, float* dw_ws, int N, int H, int W,
                              void* stream);
// stem weight gradient through per-split fp32 slabs [ks][64][256] (no atomics),
// folded straight into the parameter's [64][3][7][7] gradient:
// 64 slab elements x 4 slab groups per block: every wave reads 256 contiguous
// bytes of one slab per step; the 4 group partials meet in LDS (deterministic)
__global__ void __launch_bounds__(256) stem_wgrad_fold_kernel(int ks, const float* __restrict__ ws,
                                                              float* __restrict__ g) {
  __shared__ float part[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), grp = threadIdx.x >> 6;   // e < 64 * 256
  const float* p = ws + e;
  float a0 = 0.f, a1 = 0.f;
  int s = grp;
  for (; s + 4 < ks; s += 8) { a0 += p[(size_t)s * 64 * 256]; a1 += p[(size_t)(s + 4) * 64 * 256]; }
  if (s < ks) a0 += p[(size_t)s * 64 * 256];
  part[grp][threadIdx.x & 63] = a0 + a1;
  __syncthreads();
  if (grp == 0) {
    const int co = e >> 8, k = e & 255, kh = k >> 5, kw = (k >> 2) & 7, c = k & 3;
    if (kh < 7 && kw < 7 && c < 3) {
      const int l = threadIdx.x & 63;
      g[((co * 3 + c) * 7 + kh) * 7 + kw] = (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
    }
  }
}

VLP_EXPORT int vlp_stem_wgrad_ws(int dtype, const void* dy, const void* xp, float* split_ws, long long ws_floats,
                                 int* nsplit, int N, int H, int W, void* stream) {
  StemGeom g = make_stem(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  if (!nsplit || (long long)N * g.Hp * g.Wp * 4 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  const long long slab = 64 * 256;
  const long long fit = ws_floats / slab;
  const int max_ks = (int)(fit < 4096 ? fit : 4096);
  if (max_ks < 1) return (int)hipErrorInvalidValue;
  if (dtype != VLP_BF16 || gemm_variant() < 4) {   // other engines: atomics into slab 0
    if (hipMemsetAsync(split_ws, 0, slab * sizeof(float), st) != hipSuccess) return (int)hipGetLastError();
    *nsplit = 1;
    return vlp_stem_wgrad(dtype, dy, xp, split_ws, N, H, W, stream);
  }
  // <= 512 splits: the fold then reads <= 32 MB of slabs
  int mink = 2048;
  const int need = (g.M + (max_ks < 512 ? max_ks : 512) - 1) / (max_ks < 512 ? max_ks : 512);
  if (mink < need) mink = need;
  StemWgradB<bf16> lb{g, (const bf16*)xp, make_stem_pixstep(g, Elem<bf16>::BK)};
  MNMat<bf16> la{(const bf16*)dy, 64, 64, g.M};
  EpiSplitStore ep{nullptr, nullptr, split_ws, 256, (size_t)slab};
  const int r = launch_gemm_bk<64, 128, 1, 4>(64, 224, g.M, -mink, la, lb, ep, st);
  if (r) return r;
  *nsplit = last_ksplit();
  return *nsplit > max_ks ? (int)hipErrorInvalidValue : 0;
}

VLP_EXPORT int vlp_stem_wgrad_fold(int nsplit, const float* split_ws, float* grad, void* stream) {
  if (nsplit < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stem_wgrad_fold_kernel, dim3(64 * 256 / 64), dim3(256), 0, (hipStream_t)stream, nsplit, split_ws,
                     grad);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_stem_wgrad(int dtype, const void* dy, const void* xp, float* dw_ws, int N, int H,
                              int W, void* stream) {
  StemGeom g = make_stem(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  if ((long long)N * g.Hp * g.Wp * 4 >= (1ll << 31)) return (int)hipErrorInvalidValue;
  EpiAtomic ep{nullptr, nullptr, dw_ws, 256, 1.0f};
  if (dtype == VLP_BF16) {
    StemWgradB<bf16> lb{g, (const bf16*)xp, make_stem_pixstep(g, Elem<bf16>::BK)};
    MNMat<bf16> la{(const bf16*)dy, 64, 64, g.M};
    return gemm_wgrad<bf16>(64, 224, g.M, la, lb, ep, st);
  }
  MNMat<float> la{(const float*)dy, 64, 64, g.M};
  StemWgradB<float> lb{g, (const float*)xp, make_stem_pixstep(g, Elem<float>::BK)};
  return gemm_wgrad<float>(64, 224, g.M, la, lb, ep, st);
}

// ---------------- single-channel stem (Stem1*) ----------------
VLP_EXPORT int vlp_stem1_geom(int H, int W, int* Ho, int* Wo, int* Hp, int* Wp1) {
  Stem1Geom g = make_stem1(1, H, W);
  *Ho = g.Ho; *Wo = g.Wo; *Hp = g.Hp; *Wp1 = g.Wp1;
  return g.Wo % 4 == 0 ? 0 : (int)hipErrorInvalidValue;   // the shifted-copy walk needs Wo % 4 == 0
}

VLP_EXPORT int vlp_stem1_prep_u8(int dtype, const uint8_t* x, void* xs, int N, int H, int W, float mean, float std,
                                 void* stream) {
  Stem1Geom g = make_stem1(N, H, W);
  if (g.Wo % 4 || 4 * g.copy * (dtype == VLP_BF16 ? 2 : 4) >= (1ull << 31)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const size_t total = 4 * g.copy / 8;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(stem1_prep_u8_kernel<bf16>, dim3(blocks), dim3(256), 0, st, x, (bf16*)xs, g, H, W, mean,
                       1.f / std);
  else
    hipLaunchKernelGGL(stem1_prep_u8_kernel<float>, dim3(blocks), dim3(256), 0, st, x, (float*)xs, g, H, W, mean,
                       1.f / std);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_pack_stem1(int dtype, const float* w, void* wp, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(pack_stem1_kernel<bf16>, dim3(16), dim3(256), 0, st, w, (bf16*)wp);
  else
    hipLaunchKernelGGL(pack_stem1_kernel<float>, dim3(16), dim3(256), 0, st, w, (float*)wp);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_stem1_fwd(int dtype, const void* xs, const void* wp, void* y, int N, int H, int W,
                             double* stat_sum, double* stat_sumsq, int stat_rep, void* stream) {
  Stem1Geom g = make_stem1(N, H, W);
  if (g.Wo % 4) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16) {
    Stem1A<bf16> la{g, (const bf16*)xs};
    KMat<bf16> lb{(const bf16*)wp, 64, 64, 64};
    EpiConvFwd<bf16> ep{stat_sum, stat_sumsq, stat_rep, (bf16*)y, 64};
    return launch_gemm_bk<256, 64, 4, 1>(g.M, 64, 64, 1, la, lb, ep, st);
  }
  Stem1A<float> la{g, (const float*)xs};
  KMat<float> lb{(const float*)wp, 64, 64, 64};
  EpiConvFwd<float> ep{stat_sum, stat_sumsq, stat_rep, (float*)y, 64};
  return launch_gemm<float, 256, 64, 4>(g.M, 64, 64, 1, la, lb, ep, st);
}

// d/dW1 through per-split fp32 slabs [ks][64][64] (no atomics) -> vlp_stem1_wgrad_fold
VLP_EXPORT int vlp_stem1_wgrad_ws(int dtype, const void* dy, const void* xs, float* split_ws, long long ws_floats,
                                  int* nsplit, int N, int H, int W, void* stream) {
  Stem1Geom g = make_stem1(N, H, W);
  hipStream_t st = (hipStream_t)stream;
  if (!nsplit || g.Wo % 4) return (int)hipErrorInvalidValue;
  const long long slab = 64 * 64;
  const long long fit = ws_floats / slab;
  const int max_ks = (int)(fit < 4096 ? fit : 4096);
  if (max_ks < 1) return (int)hipErrorInvalidValue;
  EpiSplitStore ep{nullptr, nullptr, split_ws, 64, (size_t)slab};
  if (dtype != VLP_BF16) {   // fp32 parity mode: split-K with fp32 atomics into slab 0
    if (hipMemsetAsync(split_ws, 0, slab * sizeof(float), st) != hipSuccess) return (int)hipGetLastError();
    *nsplit = 1;
    MNMat<float> la{(const float*)dy, 64, 64, g.M};
    Stem1WgradB<float> lb{g, (const float*)xs, make_stem1_pixstep(g, Elem<float>::BK)};
    EpiAtomic epa{nullptr, nullptr, split_ws, 64, 1.0f};
    return gemm_wgrad<float>(64, 56, g.M, la, lb, epa, st);
  }
  int mink = 2048;
  const int need = (g.M + (max_ks < 512 ? max_ks : 512) - 1) / (max_ks < 512 ? max_ks : 512);
  if (mink < need) mink = need;
  Stem1WgradB<bf16> lb{g, (const bf16*)xs, make_stem1_pixstep(g, Elem<bf16>::BK)};
  MNMat<bf16> la{(const bf16*)dy, 64, 64, g.M};
  const int r = launch_gemm_bk<64, 64, 1, 4>(64, 56, g.M, -mink, la, lb, ep, st);
  if (r) return r;
  *nsplit = last_ksplit();
  return *nsplit > max_ks ? (int)hipErrorInvalidValue : 0;
}

VLP_EXPORT int vlp_stem1_wgrad_fold(int nsplit, const float* split_ws, float* grad, void* stream) {
  if (nsplit < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stem1_wgrad_fold_kernel, dim3(64 * 64 / 64), dim3(256), 0, (hipStream_t)stream, nsplit,
                     split_ws, grad);
  return (int)hipGetLastError();
}
