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

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
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
      v += load4(res + (size_t)row * ldr + col);
    }
    store4(out + (size_t)row * ldo + col, v);
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
  return gemm_wide<T>(M, N, K, ksplit, la, lb, ep, st);
}

// ---------------- LayerNorm over rows of D ----------------
// one wave per row; fp32 statistics; saves mean/rstd.
template <typename T>
__global__ void layernorm_fwd_kernel(int M, int D, const T* __restrict__ x, const float* __restrict__ gamma,
                                     const float* __restrict__ beta, float eps, T* __restrict__ y,
                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                     float p, uint64_t seed) {
  int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  int l = threadIdx.x & 63;
  if (row >= M) return;
  const T* xr = x + (size_t)row * D;
  float s = 0.f;
  for (int c = l; c < D; c += 64) s += to_f(xr[c]);
  float mean = warp_sum(s) / D;
  float v = 0.f;
  for (int c = l; c < D; c += 64) { float d = to_f(xr[c]) - mean; v += d * d; }
  float rstd = rsqrtf(warp_sum(v) / D + eps);
  T* yr = y + (size_t)row * D;
  for (int c = l; c < D; c += 64) {
    float o = (to_f(xr[c]) - mean) * rstd * gamma[c] + beta[c];
    if (p > 0.f) o *= drop_scale(seed, (uint64_t)row * D + c, p);
    yr[c] = from_f<T>(o);
  }
  if (l == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// LN backward.  dy is the gradient of the LN output (before the output dropout
// when p > 0: the dropout mask is re-generated from the seed).  Writes
//   dx  = LN input gradient (+ addend, e.g. a residual branch)
//   dxd = dx * dropout-mask (gradient of the dropped dense output), optional
// and accumulates dgamma/dbeta.
template <typename T>
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(int M, int D, const T* __restrict__ dy, float p_out, uint64_t seed_out,
                     const T* __restrict__ x, const float* __restrict__ mean,
                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                     T* __restrict__ dx, T* __restrict__ dxd, float p_in, uint64_t seed_in,
                     float* dgamma, float* dbeta) {
  // one wave per row; lane l owns columns l + 64j (j < kLnCols, D <= 512),
  // so the gamma/beta gradient partials live in registers across the wave's
  // rows and meet once per block (LDS) before one atomic per column
  constexpr int NJ = 8;
  __shared__ float part[4][2][NJ * 64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  float pg[NJ], pb[NJ], gm[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    pg[j] = pb[j] = 0.f;
    const int c = l + 64 * j;
    gm[j] = c < D ? gamma[c] : 0.f;
  }
  for (int row = blockIdx.x * 4 + w; row < M; row += gridDim.x * 4) {
    const T* xr = x + (size_t)row * D;
    const T* dyr = dy + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float g[NJ], xh[NJ];
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = l + 64 * j;
      g[j] = 0.f; xh[j] = 0.f;
      if (c < D) {
        g[j] = to_f(dyr[c]);
        if (p_out > 0.f) g[j] *= drop_scale(seed_out, (uint64_t)row * D + c, p_out);
        xh[j] = (to_f(xr[c]) - mu) * rs;
      }
      const float gg = g[j] * gm[j];
      a += gg;
      b += gg * xh[j];
      pg[j] += g[j] * xh[j];
      pb[j] += g[j];
    }
    a = warp_sum(a) / D;
    b = warp_sum(b) / D;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = l + 64 * j;
      if (c < D) {
        const float d = rs * (g[j] * gm[j] - a - xh[j] * b);
        dx[(size_t)row * D + c] = from_f<T>(d);
        if (dxd) {
          const float dd = p_in > 0.f ? d * drop_scale(seed_in, (uint64_t)row * D + c, p_in) : d;
          dxd[(size_t)row * D + c] = from_f<T>(dd);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    part[w][0][l + 64 * j] = pg[j];
    part[w][1][l + 64 * j] = pb[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < D; c += blockDim.x) {
    atomicAdd(dgamma + c, part[0][0][c] + part[1][0][c] + part[2][0][c] + part[3][0][c]);
    atomicAdd(dbeta + c, part[0][1][c] + part[1][1][c] + part[2][1][c] + part[3][1][c]);
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
// One workgroup per (sequence b, head h).  qkv: [B*T][3*Dm] rows (q | k | v),
// head slice [h*dh, (h+1)*dh).  Saves softmax probabilities P[b][h][T][T] (fp32).
constexpr int kMaxT = 64;
constexpr int kMaxDh = 32;

template <typename T>
__global__ void __launch_bounds__(256)
attn_fwd_kernel(int B, int Tn, int H, int dh, const T* __restrict__ qkv,
                const int64_t* __restrict__ amask, T* __restrict__ ctx, float* __restrict__ P,
                float scale, float p, uint64_t seed) {
  __shared__ float q[kMaxT][kMaxDh + 1], k[kMaxT][kMaxDh + 1], v[kMaxT][kMaxDh + 1];
  __shared__ float S[kMaxT][kMaxT + 1];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int Dm = H * dh, ld = 3 * Dm;
  for (int e = threadIdx.x; e < Tn * dh; e += blockDim.x) {
    int t = e / dh, d = e % dh;
    const T* r = qkv + (size_t)(b * Tn + t) * ld + h * dh + d;
    q[t][d] = to_f(r[0]);
    k[t][d] = to_f(r[Dm]);
    v[t][d] = to_f(r[2 * Dm]);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Tn * Tn; e += blockDim.x) {
    int i = e / Tn, j = e % Tn;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += q[i][d] * k[j][d];
    s *= scale;
    if (amask && amask[b * Tn + j] == 0) s = -1e30f;
    S[i][j] = s;
  }
  __syncthreads();
  // row softmax: one wave per row
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int i = wv; i < Tn; i += 4) {
    float x = l < Tn ? S[i][l] : -INFINITY;
    float mx = warp_max(x);
    float ex = l < Tn ? __expf(x - mx) : 0.f;
    float sum = warp_sum(ex);
    if (l < Tn) {
      float pr = ex / sum;
      P[(((size_t)b * H + h) * Tn + i) * Tn + l] = pr;
      if (p > 0.f) pr *= drop_scale(seed, (((uint64_t)b * H + h) * Tn + i) * Tn + l, p);
      S[i][l] = pr;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Tn * dh; e += blockDim.x) {
    int i = e / dh, d = e % dh;
    float s = 0.f;
    for (int j = 0; j < Tn; ++j) s += S[i][j] * v[j][d];
    ctx[(size_t)(b * Tn + i) * Dm + h * dh + d] = from_f<T>(s);
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
attn_bwd_kernel(int B, int Tn, int H, int dh, const T* __restrict__ qkv, const float* __restrict__ P,
                const T* __restrict__ dctx, T* __restrict__ dqkv, float scale, float p, uint64_t seed) {
  __shared__ float q[kMaxT][kMaxDh + 1], k[kMaxT][kMaxDh + 1], v[kMaxT][kMaxDh + 1];
  __shared__ float dc[kMaxT][kMaxDh + 1];
  __shared__ float Pd[kMaxT][kMaxT + 1], dS[kMaxT][kMaxT + 1];
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int Dm = H * dh, ld = 3 * Dm;
  for (int e = threadIdx.x; e < Tn * dh; e += blockDim.x) {
    int t = e / dh, d = e % dh;
    const T* r = qkv + (size_t)(b * Tn + t) * ld + h * dh + d;
    q[t][d] = to_f(r[0]);
    k[t][d] = to_f(r[Dm]);
    v[t][d] = to_f(r[2 * Dm]);
    dc[t][d] = to_f(dctx[(size_t)(b * Tn + t) * Dm + h * dh + d]);
  }
  const float* Pb = P + ((size_t)b * H + h) * Tn * Tn;
  __syncthreads();
  // dPd = dctx . v^T ; dP = dPd * mask ; keep Pd = P * mask for dv
  for (int e = threadIdx.x; e < Tn * Tn; e += blockDim.x) {
    int i = e / Tn, j = e % Tn;
    float s = 0.f;
    for (int d = 0; d < dh; ++d) s += dc[i][d] * v[j][d];
    float m = p > 0.f ? drop_scale(seed, (((uint64_t)b * H + h) * Tn + i) * Tn + j, p) : 1.f;
    dS[i][j] = s * m;
    Pd[i][j] = Pb[e] * m;
  }
  __syncthreads();
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int i = wv; i < Tn; i += 4) {
    float pr = l < Tn ? Pb[i * Tn + l] : 0.f;
    float dp = l < Tn ? dS[i][l] : 0.f;
    float dot = warp_sum(pr * dp);
    if (l < Tn) dS[i][l] = pr * (dp - dot);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Tn * dh; e += blockDim.x) {
    int t = e / dh, d = e % dh;
    float sq = 0.f, sk = 0.f, sv = 0.f;
    for (int j = 0; j < Tn; ++j) {
      sq += dS[t][j] * k[j][d];
      sk += dS[j][t] * q[j][d];
      sv += Pd[j][t] * dc[j][d];
    }
    T* r = dqkv + (size_t)(b * Tn + t) * ld + h * dh + d;
    r[0] = from_f<T>(sq * scale);
    r[Dm] = from_f<T>(sk * scale);
    r[2 * Dm] = from_f<T>(sv);
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

// dx[M][Kin] = dy[M][Nout] W[Nout][Kin]   (mode 1: * gelu'(aux))
VLP_EXPORT int vlp_linear_dgrad(int dtype, int M, int Kin, int Nout, const void* dy, int lddy,
                                const void* w, void* dx, int lddx, int mode, const void* aux,
                                int ldaux, const void* addend, int ldad, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16) {
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
  static const int rows_per_split = getenv("VLP_LINW_ROWS") ? atoi(getenv("VLP_LINW_ROWS")) : 1024;
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

// dW[Nout][Kin] += sum_m dy[m][n] x[m][k] through a split-K workspace
// ws[ks][Nout][Kin] fp32 (ws_elems >= ks * Nout * Kin; Kin % 4 == 0)
VLP_EXPORT int vlp_linear_wgrad_ws(int dtype, int M, int Nout, int Kin, const void* dy, int lddy,
                                   const void* x, int ldx, float* dw, float* ws, long long ws_elems,
                                   void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype != VLP_BF16 || Kin % 4 || !ws) return (int)hipErrorInvalidValue;
  const int tiles = ((Nout + 127) / 128) * ((Kin + 127) / 128);
  int ks = (512 + tiles - 1) / tiles;
  const int maxsplit = (M + 255) / 256;
  if (ks > maxsplit) ks = maxsplit;
  while (ks > 1 && (long long)ks * Nout * Kin > ws_elems) --ks;
  int kc = (M + ks - 1) / ks;
  kc = (kc + 63) / 64 * 64;
  ks = (M + kc - 1) / kc;
  MNMat<bf16> la{(const bf16*)dy, lddy, Nout, M};
  MNMat<bf16> lb{(const bf16*)x, ldx, Kin, M};
  EpiSplitStore ep{nullptr, nullptr, ws, Kin, (size_t)Nout * Kin};
  int r = launch_gemm_bk<128, 128, 2, 2>(Nout, Kin, M, ks, la, lb, ep, st);
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

VLP_EXPORT int vlp_layernorm_fwd(int dtype, int M, int D, const void* x, const float* gamma,
                                 const float* beta, float eps, void* y, float* mean, float* rstd,
                                 float p, unsigned long long seed, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((M + 3) / 4);
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(layernorm_fwd_kernel<bf16>, grid, dim3(256), 0, st, M, D, (const bf16*)x, gamma,
                       beta, eps, (bf16*)y, mean, rstd, p, seed);
  else
    hipLaunchKernelGGL(layernorm_fwd_kernel<float>, grid, dim3(256), 0, st, M, D, (const float*)x,
                       gamma, beta, eps, (float*)y, mean, rstd, p, seed);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_layernorm_bwd(int dtype, int M, int D, const void* dy, float p_out,
                                 unsigned long long seed_out, const void* x, const float* mean,
                                 const float* rstd, const float* gamma, void* dx, void* dxd,
                                 float p_in, unsigned long long seed_in, float* dgamma, float* dbeta,
                                 void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (D > 512) return (int)hipErrorInvalidValue;
  int blocks = (M + 15) / 16;   // 4 rows per wave
  if (blocks > 1024) blocks = 1024;
  size_t lds = 0;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(layernorm_bwd_kernel<bf16>, dim3(blocks), dim3(256), lds, st, M, D,
                       (const bf16*)dy, p_out, seed_out, (const bf16*)x, mean, rstd, gamma, (bf16*)dx,
                       (bf16*)dxd, p_in, seed_in, dgamma, dbeta);
  else
    hipLaunchKernelGGL(layernorm_bwd_kernel<float>, dim3(blocks), dim3(256), lds, st, M, D,
                       (const float*)dy, p_out, seed_out, (const float*)x, mean, rstd, gamma,
                       (float*)dx, (float*)dxd, p_in, seed_in, dgamma, dbeta);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_attn_fwd(int dtype, int B, int Tn, int H, int dh, const void* qkv,
                            const long long* amask, void* ctx, float* P, float scale, float p,
                            unsigned long long seed, void* stream) {
  if (Tn > kMaxT || dh > kMaxDh) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(attn_fwd_kernel<bf16>, dim3(B * H), dim3(256), 0, st, B, Tn, H, dh,
                       (const bf16*)qkv, (const int64_t*)amask, (bf16*)ctx, P, scale, p, seed);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<float>, dim3(B * H), dim3(256), 0, st, B, Tn, H, dh,
                       (const float*)qkv, (const int64_t*)amask, (float*)ctx, P, scale, p, seed);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_attn_bwd(int dtype, int B, int Tn, int H, int dh, const void* qkv, const float* P,
                            const void* dctx, void* dqkv, float scale, float p,
                            unsigned long long seed, void* stream) {
  if (Tn > kMaxT || dh > kMaxDh) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(attn_bwd_kernel<bf16>, dim3(B * H), dim3(256), 0, st, B, Tn, H, dh,
                       (const bf16*)qkv, P, (const bf16*)dctx, (bf16*)dqkv, scale, p, seed);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<float>, dim3(B * H), dim3(256), 0, st, B, Tn, H, dh,
                       (const float*)qkv, P, (const float*)dctx, (float*)dqkv, scale, p, seed);
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
