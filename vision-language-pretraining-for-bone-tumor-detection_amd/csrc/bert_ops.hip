// TinyBERT-4L-312D text tower operators (HF `BertModel`, called from the
// reference at src/models/pretrain/VisionLanguageModule.py:38-60): embeddings +
// LayerNorm(eps 1e-12) + 4 x [fused QKV projection, 12-head softmax attention
// (head dim 26), output projection + dropout + residual + LN, FFN 312->1200
// GELU(erf) ->312 + dropout + residual + LN].
//
// Rows are tokens (M = B*T); hidden vectors are row-major [M][312].  All
// projections run on the shared MFMA GEMM engine with fused epilogues
// (bias, GELU, dropout+residual); the attention runs one workgroup per
// (sequence, head) with the 40x40 score tile resident in LDS.
#include "gemm.h"

namespace vlp {

// NesT short-K / short-side token GEMMs on gemm_big_kernel (tools/build_variant.sh A/B knobs)
#ifndef VLP_LIN_SHORTK
#define VLP_LIN_SHORTK 1
#endif
#ifndef VLP_LINW_BIG
#define VLP_LINW_BIG 1
#endif

// GELU(erf) = x * Phi(x), Phi(x) = (1 + erf(x / sqrt 2)) / 2, with erf from
// Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7, branch-free: one reciprocal and
// one exp): 1 - erf(z) = P(t) exp(-z^2), t = 1 / (1 + p z), z = |x| / sqrt 2 >= 0.
// The tail 1 - erf is formed directly (no cancellation for x < 0); the result is
// within 3.3e-7 absolute of the exact GELU over [-12, 12], as close as
// 0.5 * x * (1 + erff(.)) in fp32 (4.5e-7), at a third of its VALU cost (the
// library erff is two branchy polynomials; the NesT fc1 epilogue spent more time
// in it than in the GEMM).  exp(-z^2) = exp(-x^2 / 2) is also the Gaussian
// density's exponential, shared by the gradient.
__device__ __forceinline__ float gelu_tail(float x, float& e) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.2316418883f, ax, 1.f));   // p / sqrt 2 = 0.3275911 / 1.41421356
  float P = fmaf(t, 1.061405429f, -1.453152027f);
  P = fmaf(t, P, 1.421413741f);
  P = fmaf(t, P, -0.284496736f);
  P = fmaf(t, P, 0.254829592f);
  P *= t;
  e = __expf(-0.5f * x * x);
  return P * e;
}
__device__ __forceinline__ float gelu_erf(float x) {
  float e;
  const float q = 0.5f * x * gelu_tail(x, e);   // x * (1 - Phi(|x|))
  return x >= 0.f ? x - q : q;
}
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float e;
  const float h = 0.5f * gelu_tail(x, e);       // 1 - Phi(|x|)
  const float cdf = x >= 0.f ? 1.f - h : h;
  return fmaf(x * 0.3989422804014327f, e, cdf);   // Phi(x) + x phi(x)
}
__device__ __forceinline__ float drop_scale(uint64_t seed, uint64_t idx, float p) {
  return hash_uniform(seed, idx) >= p ? 1.f / (1.f - p) : 0.f;
}

// linear forward epilogue: v = acc + bias; modes
//   0: out = v
//   1: aux = v (pre-activation), out = gelu(v)
//   2: out = dropout(v) + res                (pre-LayerNorm residual sum)
template <typename T>
struct EpiLinear {
  static constexpr bool kStats = false;
  double* stat1 = nullptr; double* stat2 = nullptr;
  T* out; int ldo; const float* bias; int mode;
  T* aux; const T* res; int ldr; float p; uint64_t seed; int N;
  const float* rscale = nullptr; int rps = 1;   // mode 2: out = rscale[row / rps] * v + res (DropPath)
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    if (bias) v += *reinterpret_cast<const v4f*>(bias + col);
    if (mode == 1) {
      store4(aux + (size_t)row * ldo + col, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_erf(v[j]);
    } else if (mode == 2) {
      if (p > 0.f) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] *= drop_scale(seed, (uint64_t)row * N + col + j, p);
      }
      if (rscale) v *= rscale[row / rps];
      v += load4(res + (size_t)row * ldr + col);
    }
    store4(out + (size_t)row * ldo + col, v);
  }
  // bf16 GEMMs: the row-chunk epilogue (gemm.h ms_epilogue).  acc + bias is staged
  // once as bf16 (what torch autocast's bf16 linear output holds), then every
  // thread streams 16-B row chunks of one fixed 8-column group: contiguous 16-B
  // stores of out / aux and 16-B loads of res instead of 8-B pieces of 16 rows.
  static constexpr bool kRow = true;
  static constexpr bool kStageBias = true;
  static constexpr int kPreDepth = 16;
  __device__ void pre8(int row, int col, RowPre& pr) const {
    if (mode == 2) pr.u[0] = ldg16(res + (size_t)row * ldr + col);
  }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& pr, float (&)[8], float (&)[8]) const {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j];
    if (mode == 1) {
      stg16(aux + (size_t)row * ldo + col, Chunk<T>::pack(o));
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = gelu_erf(o[j]);
    } else if (mode == 2) {
      if (p > 0.f) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= drop_scale(seed, (uint64_t)row * N + col + j, p);
      }
      if (rscale) {
        const float rs = rscale[row / rps];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= rs;
      }
      float r[8];
      Chunk<T>::unpack(pr.u[0], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] += r[j];
    }
    stg16(out + (size_t)row * ldo + col, Chunk<T>::pack(o));
  }
};

// linear data-gradient epilogue: modes
//   0: out = v (+ addend)
//   1: out = v * gelu'(u)            (u = saved pre-activation)
template <typename T>
struct EpiLinearBwd {
  static constexpr bool kStats = false;
  double* stat1 = nullptr; double* stat2 = nullptr;
  T* out; int ldo; int mode; const T* aux; int lda; const T* addend; int ldad;
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    if (mode == 1) {
      v4f u = load4(aux + (size_t)row * lda + col);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= gelu_erf_grad(u[j]);
    } else if (addend) {
      v += load4(addend + (size_t)row * ldad + col);
    }
    store4(out + (size_t)row * ldo + col, v);
  }
  // bf16 GEMMs: row-chunk epilogue (see EpiLinear)
  static constexpr bool kRow = true;
  static constexpr int kPreDepth = 16;
  __device__ void pre8(int row, int col, RowPre& p) const {
    if (mode == 1) p.u[0] = ldg16(aux + (size_t)row * lda + col);
    else if (addend) p.u[0] = ldg16(addend + (size_t)row * ldad + col);
  }
  __device__ void row8(int row, int col, const float (&v)[8], const RowPre& p, float (&)[8], float (&)[8]) const {
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = v[j];
    if (mode == 1 || addend) {
      float u[8];
      Chunk<T>::unpack(p.u[0], u);
      if (mode == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] *= gelu_erf_grad(u[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] += u[j];
      }
    }
    stg16(out + (size_t)row * ldo + col, Chunk<T>::pack(o));
  }
};

// split-K weight gradients: EpiSplitStore (gemm.h) writes slab s of
// ws[ks][Nout][Kin] with plain stores; linw_reduce_kernel folds the slabs
__global__ void linw_reduce_kernel(size_t n4, int ks, const float4* __restrict__ ws, float4* __restrict__ dw) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    float4 a = dw[i];
    for (int s = 0; s < ks; ++s) {
      const float4 b = ws[(size_t)s * n4 + i];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    dw[i] = a;
  }
}

template <typename T, class LA, class LB, class EP>
static int gemm_lin(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                    hipStream_t st) {
  if (N <= 64) return gemm_narrow<T>(M, N, K, ksplit, la, lb, ep, st);
  if (M <= 1024) return launch_gemm<T, 64, 256, 1>(M, N, K, ksplit, la, lb, ep, st);
  // large same-layout GEMMs (NesT level-2 projections: M = 131 k tokens, K = 384 / 1536)
  // take the 256x256 ping-pong kernel the convolutions use
  if constexpr (use_bk<T, LA, LB>()) {
    // VLP_LIN_PP: 0 off, 1 same-layout GEMMs only, 2 (default) also the data gradients
    // (NesT step +2.6 % and +0.7 %)
    constexpr int lin_pp = 2;   // linear GEMMs on the ping-pong kernel: same-layout and data gradients (measured)
    if (lin_pp && gemm_variant() >= 5 && M >= 256 && N >= 256 && K >= 256 && K % 64 == 0) {
      if constexpr (LA::kKContig == LB::kKContig) return gemm_big_auto(M, N, K, ksplit, la, lb, ep, st);
      // data gradients (K-contig dy x MN-contig W)
      else if (lin_pp >= 2) return launch_gemm_pp<256, 256, 2, 4>(M, N, K, ksplit, la, lb, ep, st);
    }
    // short-K token GEMMs (NesT levels 0 / 1: K = 96 / 192 over 0.5-2 M token rows)
    // are HBM-bound: the LDS-DMA kernel with two K-tiles in flight instead of the
    // one-tile ring (the loaders zero-fill the K tail)
    // (r6, tools/nest_gemm_bench.py, profiles/r6_lin_shortk_ab.txt: wins at K >= 192 --
    // level 1 fc1 674 -> 550 us, fc2 410 -> 349, qkv 345 -> 318, level-0 fc2 618 -> 548 --
    // and for N <= 128; loses on the K = 96, N >= 288 level-0 qkv / fc1: 674 -> 780,
    // 1123 -> 1324, which keep the one-tile ring)
    if constexpr (LA::kKContig && LB::kKContig) {
      if (VLP_LIN_SHORTK && gemm_variant() >= 5 && M >= 65536 && N >= 96 && (K >= 192 || N <= 128))
        return gemm_big_auto(M, N, K, ksplit, la, lb, ep, st);
    }
  }
  return gemm_wide<T>(M, N, K, ksplit, la, lb, ep, st);
}

// ---------------- LayerNorm over rows of D ----------------
// 16 lanes per row, 16-B chunks: lane j of a row owns chunks j, j+16, ...
// (NCH of them, D = 8 * chunks for bf16 / 4 * chunks for fp32, D <= 512), so
// a row is read once into registers and reduced with four 16-lane shuffles.
// fp32 statistics; mean / rstd saved per row.
// sum over a 16-lane row, result in every lane (DPP row_ror 8 / 4, then two
// quad permutations: VALU only)
__device__ __forceinline__ float row16_allsum(float x) {
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x128, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x124, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0xB1, 0xf, 0xf, false));
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), 0x4E, 0xf, 0xf, false));
  return x;
}

template <typename T, int NCH>
__global__ void __launch_bounds__(256)
layernorm_fwd_kernel(int M, int D, const T* __restrict__ x, const float* __restrict__ gamma,
                     const float* __restrict__ beta, float eps, T* __restrict__ y,
                     float* __restrict__ mean_out, float* __restrict__ rstd_out, float p, uint64_t seed) {
  constexpr int E = Chunk<T>::N;
  const int row = blockIdx.x * 16 + (threadIdx.x >> 4), j = threadIdx.x & 15;
  if (row >= M) return;
  const int nch = D / E;
  const T* xr = x + (size_t)row * D;
  float v[NCH][E];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = j + 16 * k;
    if (c < nch) {
      Chunk<T>::unpack(ldg16(xr + c * E), v[k]);
#pragma unroll
      for (int e = 0; e < E; ++e) s += v[k][e];
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) v[k][e] = 0.f;
    }
  }
  const float mean = row16_allsum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < NCH; ++k)
    if (j + 16 * k < nch)
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float d = v[k][e] - mean;
        q += d * d;
      }
  const float rstd = rsqrtf(row16_allsum(q) / D + eps);
  T* yr = y + (size_t)row * D;
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = j + 16 * k;
    if (c < nch) {
      const v4f* g4 = reinterpret_cast<const v4f*>(gamma + c * E);
      const v4f* b4 = reinterpret_cast<const v4f*>(beta + c * E);
      float o[E];
#pragma unroll
      for (int h = 0; h < E / 4; ++h) {
        const v4f g = g4[h], b = b4[h];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[4 * h + e] = (v[k][4 * h + e] - mean) * rstd * g[e] + b[e];
      }
      if (p > 0.f) {
#pragma unroll
        for (int e = 0; e < E; ++e) o[e] *= drop_scale(seed, (uint64_t)row * D + c * E + e, p);
      }
      stg16(yr + c * E, Chunk<T>::pack(o));
    }
  }
  if (j == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// LN backward.  dy is the gradient of the LN output (before the output dropout
// when p_out > 0: the dropout mask is re-generated from the seed).  Writes
//   dx  = LN input gradient (+ addend, e.g. a pre-norm residual's gradient)
//   dxd = optional second output: with rscale, rscale[row / rps] * dx (the
//         DropPath-scaled gradient of the residual branch that produced the
//         LN input, NesT); otherwise the LN part times the input dropout mask
// and accumulates dgamma/dbeta.  Same lane layout as the forward; rows are
// strided over a capped grid so the gamma/beta partials stay in registers,
// meet across the wave's four rows by shuffles and across the block in LDS,
// then one atomic per column and block.
template <typename T, int NCH, int NW = 4>
__global__ void __launch_bounds__(NW * 64)
layernorm_bwd_kernel(int M, int D, const T* __restrict__ dy, float p_out, uint64_t seed_out,
                     const T* __restrict__ x, const float* __restrict__ mean,
                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                     T* __restrict__ dx, T* __restrict__ dxd, float p_in, uint64_t seed_in,
                     float* dgamma, float* dbeta, const T* __restrict__ addend,
                     const float* __restrict__ rscale, int rps) {
  constexpr int E = Chunk<T>::N;
  __shared__ float part[NW][2][512];
  const int j = threadIdx.x & 15, w = threadIdx.x >> 6;
  const int nch = D / E;
  float pg[NCH][E], pb[NCH][E], gm[NCH][E];
#pragma unroll
  for (int k = 0; k < NCH; ++k) {
    const int c = j + 16 * k;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      pg[k][e] = pb[k][e] = 0.f;
      gm[k][e] = c < nch ? gamma[c * E + e] : 0.f;
    }
  }
  for (int row = blockIdx.x * (NW * 4) + (threadIdx.x >> 4); row < M; row += gridDim.x * (NW * 4)) {
    const T* xr = x + (size_t)row * D;
    const T* dyr = dy + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float g[NCH][E], xh[NCH][E];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = j + 16 * k;
      if (c < nch) {
        Chunk<T>::unpack(ldg16(dyr + c * E), g[k]);
        Chunk<T>::unpack(ldg16(xr + c * E), xh[k]);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) g[k][e] = xh[k][e] = 0.f;
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        if (p_out > 0.f && c < nch) g[k][e] *= drop_scale(seed_out, (uint64_t)row * D + c * E + e, p_out);
        xh[k][e] = c < nch ? (xh[k][e] - mu) * rs : 0.f;
        const float gg = g[k][e] * gm[k][e];
        a += gg;
        b += gg * xh[k][e];
        pg[k][e] += g[k][e] * xh[k][e];
        pb[k][e] += g[k][e];
      }
    }
    a = row16_allsum(a) / D;
    b = row16_allsum(b) / D;
    const float rsc = rscale ? rscale[row / rps] : 0.f;
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int c = j + 16 * k;
      if (c < nch) {
        float d[E], ad[E];
        if (addend) Chunk<T>::unpack(ldg16(addend + (size_t)row * D + c * E), ad);
#pragma unroll
        for (int e = 0; e < E; ++e) {
          d[e] = rs * (g[k][e] * gm[k][e] - a - xh[k][e] * b);
          if (addend) ad[e] += d[e];   // (the addend joins dx; without rscale dxd stays the LN part)
        }
        stg16(dx + (size_t)row * D + c * E, Chunk<T>::pack(addend ? ad : d));
        if (dxd) {
          float dd[E];
#pragma unroll
          for (int e = 0; e < E; ++e)
            dd[e] = rscale ? rsc * (addend ? ad[e] : d[e])
                           : (p_in > 0.f ? d[e] * drop_scale(seed_in, (uint64_t)row * D + c * E + e, p_in) : d[e]);
          stg16(dxd + (size_t)row * D + c * E, Chunk<T>::pack(dd));
        }
      }
    }
  }
  // the wave's four rows hold the same columns: fold lanes 16 apart, then waves in LDS
#pragma unroll
  for (int k = 0; k < NCH; ++k)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float u = pg[k][e], t = pb[k][e];
      u += __shfl_xor(u, 16, 64); u += __shfl_xor(u, 32, 64);
      t += __shfl_xor(t, 16, 64); t += __shfl_xor(t, 32, 64);
      const int c = j + 16 * k;
      if ((threadIdx.x & 63) < 16 && c < nch) {
        part[w][0][c * E + e] = u;
        part[w][1][c * E + e] = t;
      }
    }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int q = 0; q < NW; ++q) { sg += part[q][0][c]; sb += part[q][1][c]; }
    atomicAdd(dgamma + c, sg);
    atomicAdd(dbeta + c, sb);
  }
}

// out[n] (+)= sum_m x[m*ld + n]  (bias gradients)
template <typename T>
__global__ void colsum_kernel(int M, int N, const T* __restrict__ x, int ld, float* __restrict__ out) {
  int n = blockIdx.x * 64 + (threadIdx.x & 63);
  int part = threadIdx.x >> 6;  // 4 row-partitions per block
  if (n >= N) return;
  float s = 0.f;
  for (int m = blockIdx.y * 4 + part; m < M; m += gridDim.y * 4) s += to_f(x[(size_t)m * ld + n]);
  atomicAdd(out + n, s);
}

// 16-B column chunks: 32 chunks (256 bf16 columns) x 8 row partitions per
// block, 4 independent row loads in flight per thread
__global__ void __launch_bounds__(256)
colsum_vec_kernel(int M, int N, const bf16* __restrict__ x, int ld, float* __restrict__ out) {
  const int cg = threadIdx.x & 31, part = threadIdx.x >> 5;
  const int n0 = blockIdx.x * 256 + cg * 8;
  __shared__ float red[8][256 + 8];
  float s[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = 0.f;
  if (n0 < N) {
    const int step = gridDim.y * 8;
    int m = blockIdx.y * 8 + part;
    for (; m + 3 * step < M; m += 4 * step) {
      uint4 u[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) u[q] = ldg16(x + (size_t)(m + q * step) * ld + n0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float f[8];
        Chunk<bf16>::unpack(u[q], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += f[j];
      }
    }
    for (; m < M; m += step) {
      float f[8];
      Chunk<bf16>::unpack(ldg16(x + (size_t)m * ld + n0), f);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += f[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[part][cg * 8 + j] = s[j];
  __syncthreads();
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n < N) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x];
    atomicAdd(out + n, t);
  }
}

// ---------------- attention ----------------
// BertSelfAttention (transformers, called through VisionLanguageModule.py:45,
// 57-60): S = Q K^T * scale + ext_mask, P = softmax(S), P' = dropout(P),
// ctx = P' V.  ONE WAVE per (sequence b, head h): the token dimension is padded
// to TB*16 (T <= 64) and the head dimension (26 for TinyBERT) to 32, and every
// product is a chain of 16x16 MFMA tiles on LDS-staged operands:
//   bf16: v_mfma_f32_16x16x32_bf16 (one K-step of 32),
//   fp32 (parity mode): v_mfma_f32_16x16x4f32 x 4 per K-step of 16 (exact fp32 fma).
// Convention (mma()): D[m][n] = sum_k X[m][k] * Y[n][k] over row-major LDS
// images X, Y (k contiguous); lane l = 16g + i ends up holding D[4g + r][i],
// r = 0..3.  So with Y = the query rows, each lane owns ONE query i and four
// consecutive keys / head channels, and the softmax row reductions are two
// cross-lane xor-shuffles (lanes i, i+16, i+32, i+48) -- a wavefront-reduced
// softmax with no LDS traffic.
// The masked-key bias is HF's: scores + finfo(fp32).min where attention_mask == 0
// (modeling_bert get_extended_attention_mask); padded key slots (j >= T) are -inf.
// P (fp32, pre-dropout, [B][H][T][T]) is saved for the backward.
constexpr int kMaxT = 64;
constexpr int kMaxDh = 32;

template <typename T> struct AttnMma;
template <> struct AttnMma<bf16> {
  static constexpr int KS = 32;   // k per MFMA step
  __device__ static __forceinline__ void mma(v4f& acc, const bf16* X, int ldx, int xr, const bf16* Y, int ldy,
                                             int yr, int k0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const v8bf a = *reinterpret_cast<const v8bf*>(X + (xr + i) * ldx + k0 + 8 * g);
    const v8bf b = *reinterpret_cast<const v8bf*>(Y + (yr + i) * ldy + k0 + 8 * g);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
};
template <> struct AttnMma<float> {
  static constexpr int KS = 16;
  __device__ static __forceinline__ void mma(v4f& acc, const float* X, int ldx, int xr, const float* Y, int ldy,
                                             int yr, int k0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    const v4f a = *reinterpret_cast<const v4f*>(X + (xr + i) * ldx + k0 + 4 * g);
    const v4f b = *reinterpret_cast<const v4f*>(Y + (yr + i) * ldy + k0 + 4 * g);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[j], acc, 0, 0, 0);
  }
};

// row reductions over the 4 lanes (i, i+16, i+32, i+48) holding one query
__device__ __forceinline__ float q4_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float q4_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// LDS image geometry (elements): rows of a "k = head channel" image hold DP = 32
// values (+ pad), rows of a "k = token" image TPK = TB*16 values, rounded up to
// the MFMA K-step (+ pad); pads keep 16-B row alignment and spread LDS banks.
template <typename T, int TB>
struct AttnGeom {
  static constexpr int TP = TB * 16;                                   // padded tokens
  static constexpr int KS = AttnMma<T>::KS;
  static constexpr int TK = (TP + KS - 1) / KS * KS;                   // token-k extent
  static constexpr int PADE = 16 / (int)sizeof(T);                     // one 16-B pad
  static constexpr int LD = 32 + PADE;                                 // k = channel
  static constexpr int LT = TK + PADE;                                 // k = token
};

template <typename T>
__device__ __forceinline__ void zero_lds(T* p, int n) {
  for (int e = threadIdx.x; e < n; e += blockDim.x) p[e] = from_f<T>(0.f);
}

// rows t < Tn, channels d < dh of one head slice -> LDS image (row-major or transposed)
template <typename T>
__device__ __forceinline__ void load_head(T* dst, int ld, bool transpose, const T* src, size_t src_ld, int Tn,
                                          int dh) {
  for (int e = threadIdx.x; e < Tn * dh; e += blockDim.x) {
    const int t = e / dh, d = e - t * dh;
    const T v = src[(size_t)t * src_ld + d];
    if (transpose) dst[d * ld + t] = v;
    else dst[t * ld + d] = v;
  }
}

// VLP_ATTN_MW: one wave per 16-query block of the (b, h) (TB waves per
// workgroup: loads, the score/softmax rows and the output rows split across
// them); 0 = the whole (b, h) on one wave
#ifndef VLP_ATTN_MW
#define VLP_ATTN_MW 1
#endif
template <int TB>
constexpr int attn_waves() { return VLP_ATTN_MW ? TB : 1; }

template <typename T, int TB>
__global__ void __launch_bounds__(256)
attn_fwd_kernel(int B, int Tn, int H, int dh, const T* __restrict__ qkv, const int64_t* __restrict__ amask,
                T* __restrict__ ctx, float* __restrict__ P, float scale, float p, uint64_t seed) {
  using G = AttnGeom<T, TB>;
  using M = AttnMma<T>;
  __shared__ __attribute__((aligned(16))) T sQ[G::TP * G::LD];
  __shared__ __attribute__((aligned(16))) T sK[G::TP * G::LD];
  __shared__ __attribute__((aligned(16))) T sVt[32 * G::LT];   // V^T: [d][j]
  __shared__ __attribute__((aligned(16))) T sP[G::TP * G::LT];  // P': [i][j]
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int Dm = H * dh;
  const size_t ld = 3 * (size_t)Dm;
  const int l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  zero_lds(sQ, G::TP * G::LD);
  zero_lds(sK, G::TP * G::LD);
  zero_lds(sVt, 32 * G::LT);
  zero_lds(sP, G::TP * G::LT);
  __syncthreads();
  const T* base = qkv + (size_t)b * Tn * ld + h * dh;
  load_head(sQ, G::LD, false, base, ld, Tn, dh);
  load_head(sK, G::LD, false, base + Dm, ld, Tn, dh);
  load_head(sVt, G::LT, true, base + 2 * Dm, ld, Tn, dh);
  __syncthreads();
  // key bias per lane: keys j = jb*16 + 4*lg + r
  float kb[TB][4];
#pragma unroll
  for (int jb = 0; jb < TB; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jb * 16 + 4 * lg + r;
      kb[jb][r] = j >= Tn ? -INFINITY : (amask && amask[(size_t)b * Tn + j] == 0 ? -3.402823466e38f : 0.f);
    }
  constexpr int NW = attn_waves<TB>();
  const int wv = NW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  for (int ib = wv; ib < TB; ib += NW) {
    // S[i][j] for the 16 queries of block ib: lane holds query ib*16 + li, keys 4lg+r of each key block
    v4f s[TB];
#pragma unroll
    for (int jb = 0; jb < TB; ++jb) {
      s[jb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < 32; k0 += M::KS) M::mma(s[jb], sK, G::LD, jb * 16, sQ, G::LD, ib * 16, k0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int jb = 0; jb < TB; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[jb][r] = s[jb][r] * scale + kb[jb][r];
        mx = fmaxf(mx, s[jb][r]);
      }
    mx = q4_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int jb = 0; jb < TB; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[jb][r] = __expf(s[jb][r] - mx);
        sum += s[jb][r];
      }
    const float inv = 1.f / q4_sum(sum);
    const int i = ib * 16 + li;
#pragma unroll
    for (int jb = 0; jb < TB; ++jb) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb * 16 + 4 * lg + r;
        float pr = s[jb][r] * inv;
        if (i < Tn && j < Tn) {
          P[(((size_t)b * H + h) * Tn + i) * Tn + j] = pr;
          if (p > 0.f) pr *= drop_scale(seed, (((uint64_t)b * H + h) * Tn + i) * Tn + j, p);
        } else {
          pr = 0.f;
        }
        sP[i * G::LT + j] = from_f<T>(pr);
      }
    }
  }
  __syncthreads();
  // ctx[i][d] = sum_j P'[i][j] V[j][d]: X = V^T (rows d), Y = P' (rows i)
  for (int ib = wv; ib < TB; ib += NW) {
    const int i = ib * 16 + li;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      v4f o = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < G::TK; k0 += M::KS) M::mma(o, sVt, G::LT, db * 16, sP, G::LT, ib * 16, k0);
      if (i < Tn) {
        T* dst = ctx + ((size_t)b * Tn + i) * Dm + h * dh;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = db * 16 + 4 * lg + r;
          if (d < dh) dst[d] = from_f<T>(o[r]);
        }
      }
    }
  }
}

// Backward of attn_fwd_kernel, one wave per (b, h):
//   dP' = dctx V^T ; dP = dP' * dropout mask ; dS = P (dP - rowsum(P dP))
//   dq = scale * dS K ;  dk = scale * dS^T Q ;  dv = P'^T dctx
template <typename T, int TB>
__global__ void __launch_bounds__(256)
attn_bwd_kernel(int B, int Tn, int H, int dh, const T* __restrict__ qkv, const float* __restrict__ P,
                const T* __restrict__ dctx, T* __restrict__ dqkv, float scale, float p, uint64_t seed) {
  using G = AttnGeom<T, TB>;
  using M = AttnMma<T>;
  __shared__ __attribute__((aligned(16))) T sV[G::TP * G::LD];     // V: [j][d]
  __shared__ __attribute__((aligned(16))) T sdO[G::TP * G::LD];    // dctx: [i][d]
  __shared__ __attribute__((aligned(16))) T sKt[32 * G::LT];       // K^T: [d][j]
  __shared__ __attribute__((aligned(16))) T sQt[32 * G::LT];       // Q^T: [d][i]
  __shared__ __attribute__((aligned(16))) T sdOt[32 * G::LT];      // dctx^T: [d][i]
  __shared__ __attribute__((aligned(16))) T sdS[G::TP * G::LT];    // dS: [i][j]
  __shared__ __attribute__((aligned(16))) T sdSt[G::TP * G::LT];   // dS^T: [j][i]
  __shared__ __attribute__((aligned(16))) T sPdt[G::TP * G::LT];   // P'^T: [j][i]
  const int b = blockIdx.x / H, h = blockIdx.x - (blockIdx.x / H) * H;
  const int Dm = H * dh;
  const size_t ld = 3 * (size_t)Dm;
  const int l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  zero_lds(sV, G::TP * G::LD);
  zero_lds(sdO, G::TP * G::LD);
  zero_lds(sKt, 32 * G::LT);
  zero_lds(sQt, 32 * G::LT);
  zero_lds(sdOt, 32 * G::LT);
  zero_lds(sdS, G::TP * G::LT);
  zero_lds(sdSt, G::TP * G::LT);
  zero_lds(sPdt, G::TP * G::LT);
  __syncthreads();
  const T* base = qkv + (size_t)b * Tn * ld + h * dh;
  const T* dbase = dctx + (size_t)b * Tn * Dm + h * dh;
  load_head(sQt, G::LT, true, base, ld, Tn, dh);
  load_head(sKt, G::LT, true, base + Dm, ld, Tn, dh);
  load_head(sV, G::LD, false, base + 2 * Dm, ld, Tn, dh);
  load_head(sdO, G::LD, false, dbase, Dm, Tn, dh);
  load_head(sdOt, G::LT, true, dbase, Dm, Tn, dh);
  __syncthreads();
  const float* Pb = P + ((size_t)b * H + h) * Tn * Tn;
  constexpr int NW = attn_waves<TB>();
  const int wv = NW > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
  for (int ib = wv; ib < TB; ib += NW) {
    const int i = ib * 16 + li;
    // dP'[i][j] = sum_d dO[i][d] V[j][d]: X = V (rows j), Y = dO (rows i)
    v4f dp[TB];
#pragma unroll
    for (int jb = 0; jb < TB; ++jb) {
      dp[jb] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k0 = 0; k0 < 32; k0 += M::KS) M::mma(dp[jb], sV, G::LD, jb * 16, sdO, G::LD, ib * 16, k0);
    }
    float pr[TB][4], pd[TB][4];
    float dot = 0.f;
#pragma unroll
    for (int jb = 0; jb < TB; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb * 16 + 4 * lg + r;
        const bool ok = i < Tn && j < Tn;
        const float m = (ok && p > 0.f) ? drop_scale(seed, (((uint64_t)b * H + h) * Tn + i) * Tn + j, p) : 1.f;
        pr[jb][r] = ok ? Pb[(size_t)i * Tn + j] : 0.f;
        pd[jb][r] = pr[jb][r] * m;        // P' (what multiplied V)
        dp[jb][r] *= m;                   // dP
        dot += pr[jb][r] * dp[jb][r];
      }
    dot = q4_sum(dot);
#pragma unroll
    for (int jb = 0; jb < TB; ++jb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb * 16 + 4 * lg + r;
        const float ds = pr[jb][r] * (dp[jb][r] - dot);
        sdS[i * G::LT + j] = from_f<T>(ds);
        sdSt[j * G::LT + i] = from_f<T>(ds);
        sPdt[j * G::LT + i] = from_f<T>(pd[jb][r]);
      }
  }
  __syncthreads();
  for (int nb = wv; nb < TB; nb += NW) {
    const int t = nb * 16 + li;
#pragma unroll
    for (int db = 0; db < 2; ++db) {
      v4f dq = v4f{0.f, 0.f, 0.f, 0.f}, dk = dq, dv = dq;
#pragma unroll
      for (int k0 = 0; k0 < G::TK; k0 += M::KS) {
        M::mma(dq, sKt, G::LT, db * 16, sdS, G::LT, nb * 16, k0);     // dq[t=i][d]
        M::mma(dk, sQt, G::LT, db * 16, sdSt, G::LT, nb * 16, k0);    // dk[t=j][d]
        M::mma(dv, sdOt, G::LT, db * 16, sPdt, G::LT, nb * 16, k0);   // dv[t=j][d]
      }
      if (t < Tn) {
        T* r0 = dqkv + ((size_t)b * Tn + t) * ld + h * dh;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int d = db * 16 + 4 * lg + r;
          if (d < dh) {
            r0[d] = from_f<T>(dq[r] * scale);
            r0[Dm + d] = from_f<T>(dk[r] * scale);
            r0[2 * Dm + d] = from_f<T>(dv[r]);
          }
        }
      }
    }
  }
}

// ---------------- embeddings ----------------
// e = word[ids] + pos[t] + type[tt]; h = dropout(LN(e)); saves e (T) for backward.
template <typename T>
__global__ void embed_fwd_kernel(int M, int Tn, int D, const int64_t* __restrict__ ids,
                                 const int64_t* __restrict__ tt, const float* __restrict__ wemb,
                                 const float* __restrict__ pemb, const float* __restrict__ temb,
                                 T* __restrict__ e_out) {
  int row = blockIdx.x;
  int t = row % Tn;
  int64_t id = ids[row];
  int64_t ty = tt ? tt[row] : 0;
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    float s = wemb[(size_t)id * D + c] + pemb[(size_t)t * D + c] + temb[(size_t)ty * D + c];
    e_out[(size_t)row * D + c] = from_f<T>(s);
  }
}
// word-embedding rows: scatter-add (ids are mostly distinct, low contention)
template <typename T>
__global__ void embed_bwd_kernel(int M, int Tn, int D, const int64_t* __restrict__ ids,
                                 const T* __restrict__ de, float* dwemb) {
  const int row = blockIdx.x;
  const int64_t id = ids[row];
  // nn.Embedding(vocab, hidden, padding_idx=pad_token_id = 0) (BertEmbeddings): the
  // padding row never receives a gradient
  if (id == 0) return;
  for (int c = threadIdx.x; c < D; c += blockDim.x)
    atomicAdd(dwemb + (size_t)id * D + c, to_f(de[(size_t)row * D + c]));
}
// position rows (sum over the batch of each position) and token-type rows
// (sum over all rows of each type): reductions, not 10^4-way atomic
// contention on the same few addresses.  Block = (position t, 64 columns).
template <typename T>
__global__ void __launch_bounds__(256)
embed_pt_bwd_kernel(int B, int Tn, int D, const int64_t* __restrict__ tt, const T* __restrict__ de,
                    float* dpemb, float* dtemb) {
  __shared__ float part[4][3][64];
  const int t = blockIdx.x, l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + l;
  float sp = 0.f, s0 = 0.f, s1 = 0.f;
  if (c < D) {
    for (int b = w; b < B; b += 4) {
      const size_t row = (size_t)b * Tn + t;
      const float g = to_f(de[row * D + c]);
      sp += g;
      const int64_t ty = tt ? tt[row] : 0;
      s0 += ty == 0 ? g : 0.f;
      s1 += ty == 1 ? g : 0.f;
    }
  }
  part[w][0][l] = sp; part[w][1][l] = s0; part[w][2][l] = s1;
  __syncthreads();
  if (w == 0 && c < D) {
    float a = 0.f, b0 = 0.f, b1 = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) { a += part[q][0][l]; b0 += part[q][1][l]; b1 += part[q][2][l]; }
    atomicAdd(dpemb + (size_t)t * D + c, a);
    atomicAdd(dtemb + c, b0);
    if (b1 != 0.f) atomicAdd(dtemb + D + c, b1);
  }
}

// scatter rows: out[r*ldo + c] = in[r*ldi + c]  (CLS row gradients into [B*T][D])
template <typename T>
__global__ void scatter_rows_kernel(int R, int D, const T* __restrict__ in, int ldi, T* __restrict__ out,
                                    int ldo) {
  int r = blockIdx.x;
  for (int c = threadIdx.x; c < D; c += blockDim.x) out[(size_t)r * ldo + c] = in[(size_t)r * ldi + c];
}

}  // namespace vlp

using namespace vlp;

// y[M][N] = x[M][K] W[N][K]^T (+bias) with epilogue mode (see EpiLinear).
VLP_EXPORT int vlp_linear_fwd(int dtype, int M, int N, int K, const void* x, int ldx, const void* w,
                              const float* bias, void* y, int ldy, int mode, void* aux,
                              const void* res, int ldr, float p, unsigned long long seed,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16) {
    // the bf16 row-chunk epilogue moves 8-column groups with 16-B accesses
    if (N % 8 || ldy % 8 || (res && ldr % 8)) return (int)hipErrorInvalidValue;
    KMat<bf16> la{(const bf16*)x, ldx, M, K};
    KMat<bf16> lb{(const bf16*)w, K, N, K};
    EpiLinear<bf16> ep{nullptr, nullptr, (bf16*)y, ldy, bias, mode, (bf16*)aux, (const bf16*)res, ldr, p, seed, N};
    return gemm_lin<bf16>(M, N, K, 1, la, lb, ep, st);
  }
  KMat<float> la{(const float*)x, ldx, M, K};
  KMat<float> lb{(const float*)w, K, N, K};
  EpiLinear<float> ep{nullptr, nullptr, (float*)y, ldy, bias, mode, (float*)aux, (const float*)res, ldr, p, seed, N};
  return gemm_lin<float>(M, N, K, 1, la, lb, ep, st);
}

// residual + DropPath: y = res + rscale[row / rps] * (x W^T + bias)  (NesT
// TransformerLayer: x + drop_path(branch), one per-sample scale 0 or 1/(1-p))
VLP_EXPORT int vlp_linear_fwd_rs(int dtype, int M, int N, int K, const void* x, int ldx, const void* w,
                                 const float* bias, void* y, int ldy, const void* res, int ldr,
                                 const float* rscale, int rps, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (!rscale || rps < 1) return (int)hipErrorInvalidValue;
  if (dtype == VLP_BF16) {
    if (N % 8 || ldy % 8 || ldr % 8) return (int)hipErrorInvalidValue;
    KMat<bf16> la{(const bf16*)x, ldx, M, K};
    KMat<bf16> lb{(const bf16*)w, K, N, K};
    EpiLinear<bf16> ep{nullptr, nullptr, (bf16*)y, ldy, bias, 2, nullptr, (const bf16*)res, ldr, 0.f, 0, N, rscale, rps};
    return gemm_lin<bf16>(M, N, K, 1, la, lb, ep, st);
  }
  KMat<float> la{(const float*)x, ldx, M, K};
  KMat<float> lb{(const float*)w, K, N, K};
  EpiLinear<float> ep{nullptr, nullptr, (float*)y, ldy, bias, 2, nullptr, (const float*)res, ldr, 0.f, 0, N, rscale, rps};
  return gemm_lin<float>(M, N, K, 1, la, lb, ep, st);
}

// dx[M][Kin] = dy[M][Nout] W[Nout][Kin]   (mode 1: * gelu'(aux))
VLP_EXPORT int vlp_linear_dgrad(int dtype, int M, int Kin, int Nout, const void* dy, int lddy,
                                const void* w, void* dx, int lddx, int mode, const void* aux,
                                int ldaux, const void* addend, int ldad, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16) {
    if (Kin % 8 || lddx % 8 || (aux && ldaux % 8) || (addend && ldad % 8)) return (int)hipErrorInvalidValue;
    KMat<bf16> la{(const bf16*)dy, lddy, M, Nout};
    MNMat<bf16> lb{(const bf16*)w, Kin, Kin, Nout};
    EpiLinearBwd<bf16> ep{nullptr, nullptr, (bf16*)dx, lddx, mode, (const bf16*)aux, ldaux, (const bf16*)addend, ldad};
    return gemm_lin<bf16>(M, Kin, Nout, 1, la, lb, ep, st);
  }
  KMat<float> la{(const float*)dy, lddy, M, Nout};
  MNMat<float> lb{(const float*)w, Kin, Kin, Nout};
  EpiLinearBwd<float> ep{nullptr, nullptr, (float*)dx, lddx, mode, (const float*)aux, ldaux, (const float*)addend, ldad};
  return gemm_lin<float>(M, Kin, Nout, 1, la, lb, ep, st);
}

// dW[Nout][Kin] += sum_m dy[m][n] x[m][k]  (fp32 atomics; caller zeroes dW)
VLP_EXPORT int vlp_linear_wgrad(int dtype, int M, int Nout, int Kin, const void* dy, int lddy,
                                const void* x, int ldx, float* dw, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  // each split reduces >= 1024 token rows (short splits were prologue/atomic bound)
  constexpr int rows_per_split = 1024;
  int tiles = ((Nout + 127) / 128) * ((Kin + 127) / 128);
  int ksplit = (512 + tiles - 1) / tiles;
  int maxsplit = (M + rows_per_split - 1) / rows_per_split;
  if (ksplit > maxsplit) ksplit = maxsplit;
  EpiAtomic ep{nullptr, nullptr, dw, Kin, 1.0f};
  if (dtype == VLP_BF16) {
    MNMat<bf16> la{(const bf16*)dy, lddy, Nout, M};
    MNMat<bf16> lb{(const bf16*)x, ldx, Kin, M};
    return gemm_wide<bf16>(Nout, Kin, M, ksplit, la, lb, ep, st);
  }
  MNMat<float> la{(const float*)dy, lddy, Nout, M};
  MNMat<float> lb{(const float*)x, ldx, Kin, M};
  return launch_gemm<float, 128, 128, 2>(Nout, Kin, M, ksplit, la, lb, ep, st);
}

// split counts of vlp_linear_wgrad_ws before the workspace cap: the one-tile ring /
// gemm_big_kernel paths (128 x 128 tiles, >= 256 token rows per split, ~512
// workgroups) and the 256 x 256 ping-pong path (one round of 256, >= 2048 rows)
static int linw_splits(int M, int Nout, int Kin) {
  const int tiles = ((Nout + 127) / 128) * ((Kin + 127) / 128);
  int ks = (512 + tiles - 1) / tiles;
  const int maxsplit = (M + 255) / 256;
  if (ks > maxsplit) ks = maxsplit;
  return ks;
}
static int linw_splits_pp(int M, int Nout, int Kin) {
  const int t256 = ((Nout + 255) / 256) * ((Kin + 255) / 256);
  int k2 = (256 + t256 - 1) / t256;
  if (k2 > M / 2048) k2 = M / 2048 > 0 ? M / 2048 : 1;
  return k2;
}
static bool linw_use_pp(int M, int Nout, int Kin) {
  return gemm_variant() >= 5 && Nout >= 256 && Kin >= 256 && M >= 16384 && M % 64 == 0;
}
// fp32 elements of the split-K workspace vlp_linear_wgrad_ws uses at its full split
// count for this shape (a smaller workspace trims the splits)
VLP_EXPORT int vlp_linear_wgrad_ws_floats(int M, int Nout, int Kin, long long* n) {
  if (M < 1 || Nout < 1 || Kin < 1 || !n) return (int)hipErrorInvalidValue;
  const int ks = linw_use_pp(M, Nout, Kin) ? linw_splits_pp(M, Nout, Kin) : linw_splits(M, Nout, Kin);
  *n = (long long)(ks > 1 ? ks : 1) * Nout * Kin;
  return 0;
}

// dW[Nout][Kin] += sum_m dy[m][n] x[m][k] through a split-K workspace
// ws[ks][Nout][Kin] fp32 (ws_elems >= ks * Nout * Kin; Kin % 4 == 0)
VLP_EXPORT int vlp_linear_wgrad_ws(int dtype, int M, int Nout, int Kin, const void* dy, int lddy,
                                   const void* x, int ldx, float* dw, float* ws, long long ws_elems,
                                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype != VLP_BF16 || Kin % 4 || !ws) return (int)hipErrorInvalidValue;
  // each split reduces >= VLP_LINW_WS_ROWS token rows: the text tower runs on a
  // side stream beside the image tower, where CU time per FLOP (prologue,
  // epilogue, slab traffic), not latency, is what the step pays for
  int ks = linw_splits(M, Nout, Kin);   // >= 256 token rows per split
  while (ks > 1 && (long long)ks * Nout * Kin > ws_elems) --ks;
  int kc = (M + ks - 1) / ks;
  kc = (kc + 63) / 64 * 64;
  ks = (M + kc - 1) / kc;
  MNMat<bf16> la{(const bf16*)dy, lddy, Nout, M};
  MNMat<bf16> lb{(const bf16*)x, ldx, Kin, M};
  EpiSplitStore ep{nullptr, nullptr, ws, Kin, (size_t)Nout * Kin};
  int r;
  if (linw_use_pp(M, Nout, Kin)) {
    // deep token reductions (NesT level 2) on the 256x256 ping-pong kernel: one
    // round of 256 workgroups, >= 2048 tokens per split, within the workspace
    int k2 = linw_splits_pp(M, Nout, Kin);
    while (k2 > 1 && (long long)k2 * Nout * Kin > ws_elems) --k2;
    r = launch_gemm_pp<256, 256, 2, 4>(Nout, Kin, M, k2, la, lb, ep, st);
    ks = last_ksplit();
  } else if (VLP_LINW_BIG && M >= 65536) {
    // deep token reductions with a short side (NesT levels 0 / 1: Nout or Kin = 96 / 192):
    // two K-tiles in flight (gemm_big_kernel) instead of the one-tile ring
    r = VLP_LINW_BIG == 2 && Kin >= 256 ? launch_gemm_big<128, 256, 2, 4>(Nout, Kin, M, ks, la, lb, ep, st)
                                        : launch_gemm_big<128, 128, 2, 2>(Nout, Kin, M, ks, la, lb, ep, st);
    ks = last_ksplit();
  } else {
    r = launch_gemm_bk<128, 128, 2, 2>(Nout, Kin, M, ks, la, lb, ep, st);
  }
  if (r) return r;
  const size_t n4 = (size_t)Nout * Kin / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(linw_reduce_kernel, dim3(blocks), dim3(256), 0, st, n4, ks, (const float4*)ws, (float4*)dw);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_colsum(int dtype, int M, int N, const void* x, int ld, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16 && N % 8 == 0 && ld % 8 == 0 && ((uintptr_t)x & 15) == 0) {
    const int gx = (N + 255) / 256;
    int gy = 512 / gx;
    if (gy > (M + 63) / 64) gy = (M + 63) / 64;
    if (gy < 1) gy = 1;
    hipLaunchKernelGGL(colsum_vec_kernel, dim3(gx, gy), dim3(256), 0, st, M, N, (const bf16*)x, ld, out);
    return (int)hipGetLastError();
  }
  int gy = (M + 255) / 256;
  if (gy > 64) gy = 64;
  dim3 grid((N + 63) / 64, gy);
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, st, M, N, (const bf16*)x, ld, out);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, M, N, (const float*)x, ld, out);
  return (int)hipGetLastError();
}

template <typename T, int NCH>
static void ln_fwd_t(int M, int D, const void* x, const float* gamma, const float* beta, float eps, void* y,
                     float* mean, float* rstd, float p, unsigned long long seed, hipStream_t st) {
  hipLaunchKernelGGL((layernorm_fwd_kernel<T, NCH>), dim3((M + 15) / 16), dim3(256), 0, st, M, D, (const T*)x, gamma,
                     beta, eps, (T*)y, mean, rstd, p, (uint64_t)seed);
}
// chunks per lane: ceil(D / (16 elements-per-chunk... x 16 lanes))
static int ln_nch(int dtype, int D) {
  const int e = dtype == VLP_BF16 ? 8 : 4;
  if (D < 1 || D > 512 || D % e) return -1;
  return (D / e + 15) / 16;
}
#define LN_DISPATCH(F, dtype, nch, ...)                                                          \
  do {                                                                                         \
    if ((dtype) == VLP_BF16) {                                                                 \
      switch (nch) {                                                                           \
        case 1: F<bf16, 1>(__VA_ARGS__); break;                                                \
        case 2: F<bf16, 2>(__VA_ARGS__); break;                                                \
        case 3: F<bf16, 3>(__VA_ARGS__); break;                                                \
        default: F<bf16, 4>(__VA_ARGS__); break;                                               \
      }                                                                                        \
    } else {                                                                                   \
      switch (nch) {                                                                           \
        case 1: F<float, 1>(__VA_ARGS__); break;                                               \
        case 2: F<float, 2>(__VA_ARGS__); break;                                               \
        case 3: F<float, 3>(__VA_ARGS__); break;                                               \
        case 4: F<float, 4>(__VA_ARGS__); break;                                               \
        case 5: case 6: F<float, 6>(__VA_ARGS__); break;                                       \
        default: F<float, 8>(__VA_ARGS__); break;                                              \
      }                                                                                        \
    }                                                                                          \
  } while (0)

VLP_EXPORT int vlp_layernorm_fwd(int dtype, int M, int D, const void* x, const float* gamma,
                                 const float* beta, float eps, void* y, float* mean, float* rstd,
                                 float p, unsigned long long seed, void* stream) {
  const int nch = ln_nch(dtype, D);
  if (nch < 0) return (int)hipErrorInvalidValue;
  if (M < 1) return 0;
  LN_DISPATCH(ln_fwd_t, dtype, nch, M, D, x, gamma, beta, eps, y, mean, rstd, p, seed, (hipStream_t)stream);
  return (int)hipGetLastError();
}

#ifndef VLP_LNB_TEXT_WAVES
#define VLP_LNB_TEXT_WAVES 8   // waves per LayerNorm-backward block at text-sized M (4 = the NesT block)
#endif
template <typename T, int NCH>
static void ln_bwd_t(int M, int D, const void* dy, float p_out, unsigned long long seed_out, const void* x,
                     const float* mean, const float* rstd, const float* gamma, void* dx, void* dxd, float p_in,
                     unsigned long long seed_in, float* dgamma, float* dbeta, const void* addend,
                     const float* rscale, int rps, hipStream_t st) {
  // rows are strided over a capped grid: every block ends in one dgamma / dbeta
  // atomic per column, so the grid size is the atomic fan-in per address
  // (640 blocks at M = 10240 serialised on 624 addresses: 36 us per launch);
  // the cap applies to text-sized M only: NesT's 0.1-2 M token rows need the
  // wide grid for bandwidth (a 160 or M/2048 cap there: -3 % per NesT step)
  constexpr int cap = 160;   // LayerNorm-backward grid cap for text-sized M (atomic fan-in)
  if (M <= 65536 && VLP_LNB_TEXT_WAVES > 4) {
    // text-sized M: the capped grid with 8-wave blocks (32 rows per pass, twice the
    // loads in flight per CU at the same atomic fan-in)
    constexpr int NW = VLP_LNB_TEXT_WAVES;
    int blocks = (M + NW * 4 - 1) / (NW * 4);
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL((layernorm_bwd_kernel<T, NCH, NW>), dim3(blocks), dim3(NW * 64), 0, st, M, D, (const T*)dy,
                       p_out, (uint64_t)seed_out, (const T*)x, mean, rstd, gamma, (T*)dx, (T*)dxd, p_in,
                       (uint64_t)seed_in, dgamma, dbeta, (const T*)addend, rscale, rps);
    return;
  }
  int blocks = (M + 15) / 16;
  const int lim = M <= 65536 ? cap : 4096;
  if (blocks > lim) blocks = lim;
  hipLaunchKernelGGL((layernorm_bwd_kernel<T, NCH>), dim3(blocks), dim3(256), 0, st, M, D, (const T*)dy, p_out,
                     (uint64_t)seed_out, (const T*)x, mean, rstd, gamma, (T*)dx, (T*)dxd, p_in, (uint64_t)seed_in,
                     dgamma, dbeta, (const T*)addend, rscale, rps);
}
static int layernorm_bwd_launch(int dtype, int M, int D, const void* dy, float p_out,
                                unsigned long long seed_out, const void* x, const float* mean,
                                const float* rstd, const float* gamma, void* dx, void* dxd,
                                float p_in, unsigned long long seed_in, float* dgamma, float* dbeta,
                                const void* addend, const float* rscale, int rps, void* stream) {
  const int nch = ln_nch(dtype, D);
  if (nch < 0 || (rscale && rps < 1)) return (int)hipErrorInvalidValue;
  if (M < 1) return 0;
  LN_DISPATCH(ln_bwd_t, dtype, nch, M, D, dy, p_out, seed_out, x, mean, rstd, gamma, dx, dxd, p_in, seed_in, dgamma,
              dbeta, addend, rscale, rps, (hipStream_t)stream);
  return (int)hipGetLastError();
}
VLP_EXPORT int vlp_layernorm_bwd(int dtype, int M, int D, const void* dy, float p_out,
                                 unsigned long long seed_out, const void* x, const float* mean,
                                 const float* rstd, const float* gamma, void* dx, void* dxd,
                                 float p_in, unsigned long long seed_in, float* dgamma, float* dbeta,
                                 void* stream) {
  return layernorm_bwd_launch(dtype, M, D, dy, p_out, seed_out, x, mean, rstd, gamma, dx, dxd, p_in, seed_in,
                              dgamma, dbeta, nullptr, nullptr, 1, stream);
}
// pre-norm residual form: dx = LN backward + addend (NesT: x + attn(norm1(x)));
// dxs (optional) = rscale[row / rps] * dx, the DropPath-scaled gradient of the
// residual branch that produced x (nullptr rscale: dxs unused)
VLP_EXPORT int vlp_layernorm_bwd_add(int dtype, int M, int D, const void* dy, const void* x, const float* mean,
                                     const float* rstd, const float* gamma, const void* addend, void* dx,
                                     float* dgamma, float* dbeta, void* stream) {
  return layernorm_bwd_launch(dtype, M, D, dy, 0.f, 0, x, mean, rstd, gamma, dx, nullptr, 0.f, 0, dgamma, dbeta,
                              addend, nullptr, 1, stream);
}
VLP_EXPORT int vlp_layernorm_bwd_add_rs(int dtype, int M, int D, const void* dy, const void* x, const float* mean,
                                        const float* rstd, const float* gamma, const void* addend, void* dx,
                                        void* dxs, const float* rscale, int rps, float* dgamma, float* dbeta,
                                        void* stream) {
  if (!rscale || !dxs) return (int)hipErrorInvalidValue;
  return layernorm_bwd_launch(dtype, M, D, dy, 0.f, 0, x, mean, rstd, gamma, dx, dxs, 0.f, 0, dgamma, dbeta,
                              addend, rscale, rps, stream);
}

template <typename T, int TB>
static void launch_attn_fwd(int B, int Tn, int H, int dh, const void* qkv, const long long* amask, void* ctx,
                            float* P, float scale, float p, unsigned long long seed, hipStream_t st) {
  hipLaunchKernelGGL((attn_fwd_kernel<T, TB>), dim3(B * H), dim3(64 * attn_waves<TB>()), 0, st, B, Tn, H, dh, (const T*)qkv,
                     (const int64_t*)amask, (T*)ctx, P, scale, p, (uint64_t)seed);
}
template <typename T, int TB>
static void launch_attn_bwd(int B, int Tn, int H, int dh, const void* qkv, const float* P, const void* dctx,
                            void* dqkv, float scale, float p, unsigned long long seed, hipStream_t st) {
  hipLaunchKernelGGL((attn_bwd_kernel<T, TB>), dim3(B * H), dim3(64 * attn_waves<TB>()), 0, st, B, Tn, H, dh, (const T*)qkv, P,
                     (const T*)dctx, (T*)dqkv, scale, p, (uint64_t)seed);
}

VLP_EXPORT int vlp_attn_fwd(int dtype, int B, int Tn, int H, int dh, const void* qkv,
                            const long long* amask, void* ctx, float* P, float scale, float p,
                            unsigned long long seed, void* stream) {
  if (Tn < 1 || Tn > kMaxT || dh < 1 || dh > kMaxDh || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const bool small = Tn <= 48;
  if (dtype == VLP_BF16) {
    if (small) launch_attn_fwd<bf16, 3>(B, Tn, H, dh, qkv, amask, ctx, P, scale, p, seed, st);
    else launch_attn_fwd<bf16, 4>(B, Tn, H, dh, qkv, amask, ctx, P, scale, p, seed, st);
  } else {
    if (small) launch_attn_fwd<float, 3>(B, Tn, H, dh, qkv, amask, ctx, P, scale, p, seed, st);
    else launch_attn_fwd<float, 4>(B, Tn, H, dh, qkv, amask, ctx, P, scale, p, seed, st);
  }
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_attn_bwd(int dtype, int B, int Tn, int H, int dh, const void* qkv, const float* P,
                            const void* dctx, void* dqkv, float scale, float p,
                            unsigned long long seed, void* stream) {
  if (Tn < 1 || Tn > kMaxT || dh < 1 || dh > kMaxDh || B < 1 || H < 1) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const bool small = Tn <= 48;
  if (dtype == VLP_BF16) {
    if (small) launch_attn_bwd<bf16, 3>(B, Tn, H, dh, qkv, P, dctx, dqkv, scale, p, seed, st);
    else launch_attn_bwd<bf16, 4>(B, Tn, H, dh, qkv, P, dctx, dqkv, scale, p, seed, st);
  } else {
    if (small) launch_attn_bwd<float, 3>(B, Tn, H, dh, qkv, P, dctx, dqkv, scale, p, seed, st);
    else launch_attn_bwd<float, 4>(B, Tn, H, dh, qkv, P, dctx, dqkv, scale, p, seed, st);
  }
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_embed_fwd(int dtype, int M, int Tn, int D, const long long* ids,
                             const long long* tt, const float* wemb, const float* pemb,
                             const float* temb, void* e_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(embed_fwd_kernel<bf16>, dim3(M), dim3(128), 0, st, M, Tn, D,
                       (const int64_t*)ids, (const int64_t*)tt, wemb, pemb, temb, (bf16*)e_out);
  else
    hipLaunchKernelGGL(embed_fwd_kernel<float>, dim3(M), dim3(128), 0, st, M, Tn, D,
                       (const int64_t*)ids, (const int64_t*)tt, wemb, pemb, temb, (float*)e_out);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_embed_bwd(int dtype, int M, int Tn, int D, const long long* ids,
                             const long long* tt, const void* de, float* dwemb, float* dpemb,
                             float* dtemb, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (M % Tn) return (int)hipErrorInvalidValue;
  const dim3 gpt(Tn, (D + 63) / 64);
  if (dtype == VLP_BF16) {
    hipLaunchKernelGGL(embed_bwd_kernel<bf16>, dim3(M), dim3(128), 0, st, M, Tn, D,
                       (const int64_t*)ids, (const bf16*)de, dwemb);
    hipLaunchKernelGGL(embed_pt_bwd_kernel<bf16>, gpt, dim3(256), 0, st, M / Tn, Tn, D,
                       (const int64_t*)tt, (const bf16*)de, dpemb, dtemb);
  } else {
    hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3(M), dim3(128), 0, st, M, Tn, D,
                       (const int64_t*)ids, (const float*)de, dwemb);
    hipLaunchKernelGGL(embed_pt_bwd_kernel<float>, gpt, dim3(256), 0, st, M / Tn, Tn, D,
                       (const int64_t*)tt, (const float*)de, dpemb, dtemb);
  }
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_scatter_rows(int dtype, int R, int D, const void* in, int ldi, void* out, int ldo,
                                void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(scatter_rows_kernel<bf16>, dim3(R), dim3(128), 0, st, R, D, (const bf16*)in,
                       ldi, (bf16*)out, ldo);
  else
    hipLaunchKernelGGL(scatter_rows_kernel<float>, dim3(R), dim3(128), 0, st, R, D, (const float*)in,
                       ldi, (float*)out, ldo);
  return (int)hipGetLastError();
}
