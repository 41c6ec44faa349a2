// Train-mode BatchNorm2d, residual add + ReLU, max/avg pooling for the ResNet34
// tower (timm BasicBlock semantics: conv-bn-relu-conv-bn (+shortcut) relu;
// stem conv-bn-relu-maxpool3x3/2; global average pool), NHWC layout.
//
// Batch statistics come from the conv epilogues (fp64 sums); everything here
// is an HBM-bound streaming pass over [M = N*H*W][C] tensors in 16-byte chunks.
// Threads own a FIXED channel chunk (grid stride is a multiple of C/EPC), so
// per-channel coefficients are folded once into registers and the inner loop
// is loads, FMAs and stores only.
//
// Reductions over M (BN backward sums) are accumulated per workgroup and then
// added with fp64 atomics into `rep` replicas of the [C] sums (replica =
// workgroup % rep) to avoid serialising thousands of workgroups on C
// addresses; vlp_stat_reduce folds replicas into replica 0.
#include "common.h"

namespace vlp {

constexpr int kEwThreads = 256;

// bit j = (bf16 element j of the 16-B chunk > 0): the ReLU mask of a stored
// activation, 1/16 of its bytes (read back by the data-gradient epilogues)
__device__ __forceinline__ uint8_t relu_bits8(const uint4& u) {
  const unsigned w[4] = {u.x, u.y, u.z, u.w};
  unsigned m = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned lo = w[q] & 0xffffu, hi = w[q] >> 16;
    m |= (unsigned)((lo & 0x8000u) == 0 && lo != 0) << (2 * q);
    m |= (unsigned)((hi & 0x8000u) == 0 && hi != 0) << (2 * q + 1);
  }
  return (uint8_t)m;
}

static inline int ew_blocks(size_t work, int per_block = kEwThreads, int cap = 8192) {
  size_t b = (work + per_block - 1) / per_block;
  if (b > (size_t)cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

// ---- finalize batch statistics -> affine coefficients, running stats ----
__global__ void bn_finalize_kernel(int C, double count, const double* __restrict__ sum,
                                   const double* __restrict__ sumsq, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float eps, float momentum,
                                   float* running_mean, float* running_var, float* scale,
                                   float* shift, float* mean_out, float* invstd_out) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double mean = sum[c] / count;
  double var = sumsq[c] / count - mean * mean;
  if (var < 0) var = 0;
  float invstd = (float)(1.0 / sqrt(var + (double)eps));
  float sc = gamma[c] * invstd;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mean * sc;
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  if (running_mean) {
    float unbiased = (float)(count > 1 ? var * count / (count - 1) : var);
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

// eval-mode coefficients from running statistics
__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rm,
                               const float* rv, float eps, float* scale, float* shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float invstd = 1.f / sqrtf(rv[c] + eps);
  scale[c] = gamma[c] * invstd;
  shift[c] = beta[c] - rm[c] * gamma[c] * invstd;
}

// fold `rep` replicas [rep][C] into replica 0, for up to 3 arrays.  One block
// per (array, 64-channel group); the 4 waves split the replicas so each lane
// has only rep/4 independent loads in flight (latency-bound otherwise).
__global__ void __launch_bounds__(256)
stat_reduce_kernel(int rep, int C, double* a, double* b, double* c) {
  __shared__ double part[4][64];
  double* arr[3] = {a, b, c};
  double* p = arr[blockIdx.y];
  if (!p) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  double s = 0;
  if (ch < C)
    for (int r = w; r < rep; r += 4) s += p[(size_t)r * C + ch];
  part[w][lane] = s;
  __syncthreads();
  if (w == 0 && ch < C) p[ch] = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
}

// replica fold of up to 3 arrays for one 64-channel group: 8 waves split the
// replicas and every lane keeps all its loads in flight (latency-bound
// otherwise); returns the totals in tot[k][lane] and stores them into replica 0
constexpr int kFoldWaves = 8;
__device__ __forceinline__ void fold_replicas(int rep, int C, double* const* arr, int n, double (*tot)[64]) {
  __shared__ double part[3][kFoldWaves][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + lane;
  double s[3] = {0, 0, 0};
  if (ch < C) {
    int r = w;
    for (; r + 3 * kFoldWaves < rep; r += 4 * kFoldWaves) {
      double v[3][4];
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          v[k][j] = (k < n && arr[k]) ? arr[k][(size_t)(r + j * kFoldWaves) * C + ch] : 0.0;
#pragma unroll
      for (int k = 0; k < 3; ++k) s[k] += (v[k][0] + v[k][1]) + (v[k][2] + v[k][3]);
    }
    for (; r < rep; r += kFoldWaves)
#pragma unroll
      for (int k = 0; k < 3; ++k)
        if (k < n && arr[k]) s[k] += arr[k][(size_t)r * C + ch];
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) part[k][w][lane] = s[k];
  __syncthreads();
  if (w == 0 && ch < C)
    for (int k = 0; k < n; ++k) {
      double t = 0;
#pragma unroll
      for (int q = 0; q < kFoldWaves; ++q) t += part[k][q][lane];
      tot[k][lane] = t;
      if (arr[k]) arr[k][ch] = t;
    }
}

// stat_reduce + bn_finalize in one launch (forward BN after a replicated-sum producer)
__global__ void __launch_bounds__(64 * kFoldWaves)
bn_finalize_rep_kernel(int rep, int C, double count, double* sum, double* sumsq, const float* __restrict__ gamma,
                       const float* __restrict__ beta, float eps, float momentum, float* running_mean,
                       float* running_var, float* scale, float* shift, float* mean_out, float* invstd_out) {
  __shared__ double tot[2][64];
  double* arr[2] = {sum, sumsq};
  fold_replicas(rep, C, arr, 2, tot);
  const int lane = threadIdx.x & 63, c = blockIdx.x * 64 + lane;
  if (threadIdx.x >= 64 || c >= C) return;
  double mean = tot[0][lane] / count;
  double var = tot[1][lane] / count - mean * mean;
  if (var < 0) var = 0;
  float invstd = (float)(1.0 / sqrt(var + (double)eps));
  float sc = gamma[c] * invstd;
  scale[c] = sc;
  shift[c] = beta[c] - (float)mean * sc;
  mean_out[c] = (float)mean;
  invstd_out[c] = invstd;
  if (running_mean) {
    float unbiased = (float)(count > 1 ? var * count / (count - 1) : var);
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * (float)mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

// stat_reduce + bn_param_grad: dgamma = sum g*xhat, dbeta = sum g for a BN and
// (optionally) the downsample BN that shares g
__global__ void __launch_bounds__(64 * kFoldWaves)
bn_grad_rep_kernel(int rep, int C, double* sum_g, double* sum_gx, double* sum_gxd, float* dgamma, float* dbeta,
                   float* dgamma_d, float* dbeta_d) {
  __shared__ double tot[3][64];
  double* arr[3] = {sum_g, sum_gx, sum_gxd};
  fold_replicas(rep, C, arr, 3, tot);
  const int lane = threadIdx.x & 63, c = blockIdx.x * 64 + lane;
  if (threadIdx.x >= 64 || c >= C) return;
  dgamma[c] = (float)tot[1][lane];
  dbeta[c] = (float)tot[0][lane];
  if (dgamma_d) {
    dgamma_d[c] = (float)tot[2][lane];
    dbeta_d[c] = (float)tot[0][lane];
  }
}

// ---- out = relu(sc*y + sh + identity), identity = idt or (scd*idt + shd) ----
// U chunks per thread per iteration with every load issued before the first
// store (more bytes in flight per wave); NT: non-temporal stores (streamed
// outputs are not re-read by this pass)
template <int U, bool NT>
__device__ __forceinline__ void ew_st16(void* p, const uint4& v) {
  if constexpr (NT) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u*>(p));
  }
  else stg16(p, v);
}
template <typename T, bool HAS_IDT, int U = 1, bool NT = false>
__global__ void __launch_bounds__(256)
bn_add_relu_kernel(unsigned nchunks, int cpr, const T* __restrict__ y, const float* __restrict__ sc,
                   const float* __restrict__ sh, const T* __restrict__ idt,
                   const float* __restrict__ scd, const float* __restrict__ shd, T* __restrict__ out,
                   uint8_t* __restrict__ rmask) {
  constexpr int E = Chunk<T>::N;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned stride = gridDim.x * blockDim.x;   // multiple of cpr
  const int c0 = (int)(tid % (unsigned)cpr) * E;
  float a[E], b[E], c[E], d[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    a[j] = sc[c0 + j]; b[j] = sh[c0 + j];
    c[j] = scd ? scd[c0 + j] : 1.f;
    d[j] = scd ? shd[c0 + j] : 0.f;
    b[j] += d[j];
  }
  auto one = [&](unsigned i, const uint4& yv, const uint4& iv) __attribute__((always_inline)) {
    float u[E], v[E];
    Chunk<T>::unpack(yv, u);
    if constexpr (HAS_IDT) {
      Chunk<T>::unpack(iv, v);
#pragma unroll
      for (int j = 0; j < E; ++j) u[j] = fmaxf(fmaf(u[j], a[j], fmaf(v[j], c[j], b[j])), 0.f);
    } else {
#pragma unroll
      for (int j = 0; j < E; ++j) u[j] = fmaxf(fmaf(u[j], a[j], b[j]), 0.f);
    }
    const uint4 pk = Chunk<T>::pack(u);
    ew_st16<U, NT>(out + (size_t)i * E, pk);
    if constexpr (E == 8) {
      if (rmask) rmask[i] = relu_bits8(pk);
    }
  };
  unsigned i = tid;
  if constexpr (U > 1) {
    for (; i + (U - 1) * stride < nchunks; i += U * stride) {
      uint4 yv[U], iv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        yv[k] = ldg16(y + (size_t)(i + k * stride) * E);
        if constexpr (HAS_IDT) iv[k] = ldg16(idt + (size_t)(i + k * stride) * E);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) one(i + k * stride, yv[k], HAS_IDT ? iv[k] : yv[k]);
    }
  }
  for (; i < nchunks; i += stride) {
    const uint4 yv = ldg16(y + (size_t)i * E);
    const uint4 iv = HAS_IDT ? ldg16(idt + (size_t)i * E) : yv;
    one(i, yv, iv);
  }
}

// ---- blocked streaming layout (r6) ----
// A workgroup owns contiguous segments of 256 * U 16-B chunks (thread t: chunks
// seg + t + 256 k, k < U), segments grid-strided, every load of a segment issued
// before its first store, non-temporal stores (and loads, NTL).  At the bs = 256 layer-1
// size (537 MB per tensor) a 2-read / 1-write pass runs 5.9 TB/s this way against
// 4.4 TB/s for the thread-strided single-chunk loop (tools/probes/ew_probe.hip,
// profiles/r6_ew_probe.txt): each workgroup's requests sweep whole DRAM pages.
// 256 % cpr == 0 keeps every chunk a thread touches in its own channel group.
__device__ __forceinline__ uint4 ntl16(const void* p) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(w.x, w.y, w.z, w.w);
}
constexpr int kBlkU = 4;   // chunks per thread per segment
static inline int blk_grid(size_t nchunks) {
  size_t b = (nchunks + 256 * kBlkU - 1) / (256 * kBlkU);
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}
template <bool HAS_IDT, bool NTL>
__global__ void __launch_bounds__(256)
bn_add_relu_blk_kernel(unsigned nchunks, int cpr, const bf16* __restrict__ y, const float* __restrict__ sc,
                       const float* __restrict__ sh, const bf16* __restrict__ idt,
                       const float* __restrict__ scd, const float* __restrict__ shd, bf16* __restrict__ out,
                       uint8_t* __restrict__ rmask) {
  constexpr int U = kBlkU;
  const int c0 = (int)(threadIdx.x % (unsigned)cpr) * 8;
  float a[8], b[8], c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {   // as bn_add_relu_kernel
    a[j] = sc[c0 + j]; b[j] = sh[c0 + j];
    c[j] = scd ? scd[c0 + j] : 1.f;
    b[j] += scd ? shd[c0 + j] : 0.f;
  }
  for (unsigned s0 = blockIdx.x * (256u * U); s0 < nchunks; s0 += gridDim.x * (256u * U)) {
    const unsigned i0 = s0 + threadIdx.x;
    uint4 yv[U], iv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned i = i0 + 256u * k;
      if (i < nchunks) {
        yv[k] = NTL ? ntl16(y + (size_t)i * 8) : ldg16(y + (size_t)i * 8);
        if constexpr (HAS_IDT) iv[k] = NTL ? ntl16(idt + (size_t)i * 8) : ldg16(idt + (size_t)i * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned i = i0 + 256u * k;
      if (i >= nchunks) continue;
      float u[8], v[8];
      Chunk<bf16>::unpack(yv[k], u);
      if constexpr (HAS_IDT) {
        Chunk<bf16>::unpack(iv[k], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = fmaxf(fmaf(u[j], a[j], fmaf(v[j], c[j], b[j])), 0.f);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) u[j] = fmaxf(fmaf(u[j], a[j], b[j]), 0.f);
      }
      const uint4 pk = Chunk<bf16>::pack(u);
      ew_st16<1, true>(out + (size_t)i * 8, pk);
      if (rmask) rmask[i] = relu_bits8(pk);
    }
  }
}

// ---- backward reduction: g = dout * (out > 0); sums of g, g*xhat_a, g*xhat_b ----
// dout may instead be a broadcast [N][C] gradient divided by HW (global avg pool).
template <typename T>
__global__ void __launch_bounds__(256)
bn_bwd_reduce_kernel(int M, int C, const T* __restrict__ dout, const float* __restrict__ dbc,
                     int HW, const T* __restrict__ mask, const T* __restrict__ ya,
                     const float* __restrict__ mean_a, const float* __restrict__ istd_a,
                     const T* __restrict__ yb, const float* __restrict__ mean_b,
                     const float* __restrict__ istd_b, double* sum_g, double* sum_ga,
                     double* sum_gb, int rep) {
  constexpr int E = Chunk<T>::N;
  const int cpr = C / E;
  const int rows_per_iter = 256 / cpr;
  const int t = threadIdx.x;
  const int cc = t % cpr, rr = t / cpr;
  const int c0 = cc * E;
  float ag[E], aa[E], ab[E];
  float ma[E], ia[E], mb[E], ib[E];
  const float inv_hw = 1.f / (float)HW;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    ag[j] = aa[j] = ab[j] = 0.f;
    ma[j] = mean_a[c0 + j]; ia[j] = istd_a[c0 + j];
    mb[j] = yb ? mean_b[c0 + j] : 0.f; ib[j] = yb ? istd_b[c0 + j] : 0.f;
  }
  for (int m = blockIdx.x * rows_per_iter + rr; m < M; m += gridDim.x * rows_per_iter) {
    size_t o = (size_t)m * C + c0;
    float g[E], mk[E], y1[E], y2[E];
    if (dbc) {
      int n = m / HW;
#pragma unroll
      for (int j = 0; j < E; ++j) g[j] = dbc[(size_t)n * C + c0 + j] * inv_hw;
    } else {
      Chunk<T>::unpack(ldg16(dout + o), g);
    }
    Chunk<T>::unpack(ldg16(mask + o), mk);
    Chunk<T>::unpack(ldg16(ya + o), y1);
    if (yb) Chunk<T>::unpack(ldg16(yb + o), y2);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      float gg = mk[j] > 0.f ? g[j] : 0.f;
      ag[j] += gg;
      aa[j] += gg * ((y1[j] - ma[j]) * ia[j]);
      if (yb) ab[j] += gg * ((y2[j] - mb[j]) * ib[j]);
    }
  }
  __shared__ float red[3][256][E];
#pragma unroll
  for (int j = 0; j < E; ++j) { red[0][t][j] = ag[j]; red[1][t][j] = aa[j]; red[2][t][j] = ab[j]; }
  __syncthreads();
  if (t < cpr) {
    for (int r = 1; r < rows_per_iter; ++r)
#pragma unroll
      for (int j = 0; j < E; ++j) {
        ag[j] += red[0][t + r * cpr][j];
        aa[j] += red[1][t + r * cpr][j];
        ab[j] += red[2][t + r * cpr][j];
      }
    const size_t ro = (size_t)(blockIdx.x % rep) * C + c0;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      atomicAdd(sum_g + ro + j, (double)ag[j]);
      atomicAdd(sum_ga + ro + j, (double)aa[j]);
      if (yb) atomicAdd(sum_gb + ro + j, (double)ab[j]);
    }
  }
}

// ---- backward apply: dy_s = A_s*g + B_s*y_s + C_s (folded BN backward) ----
struct BnBwdSide {
  const void* y; const float* mean; const float* istd; const float* gamma;
  const double* sum_g; const double* sum_gx; void* dy;
};
template <typename T, bool HAS_B, int U = 1, bool NT = false>
__global__ void __launch_bounds__(256)
bn_bwd_apply_kernel(unsigned nchunks, int cpr, double count, const T* __restrict__ dout,
                    const float* __restrict__ dbc, int HW, const T* __restrict__ mask, BnBwdSide A,
                    BnBwdSide B, T* __restrict__ g_out) {
  constexpr int E = Chunk<T>::N;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned stride = gridDim.x * blockDim.x;   // multiple of cpr
  const int c0 = (int)(tid % (unsigned)cpr) * E;
  const int C = cpr * E;
  const float inv_count = (float)(1.0 / count);
  const float inv_hw = 1.f / (float)HW;
  // dy = k*(g - mg - (y-mu)*istd*mgx) = k*g + (-k*istd*mgx)*y + (-k*mg + k*istd*mgx*mu)
  float ka[E], ba[E], ca[E], kb[E], bb[E], cb[E];
#pragma unroll
  for (int j = 0; j < E; ++j) {
    int c = c0 + j;
    bn_bwd_coef(A.gamma[c], A.istd[c], A.mean[c], A.sum_g[c], A.sum_gx[c], inv_count, ka[j], ba[j], ca[j]);
    if (HAS_B) bn_bwd_coef(B.gamma[c], B.istd[c], B.mean[c], B.sum_g[c], B.sum_gx[c], inv_count, kb[j], bb[j], cb[j]);
  }
  // the plain form (no broadcast gradient, no mask, no g_out, one side) runs
  // U chunks per iteration with both loads of every chunk issued first
  if constexpr (U > 1 && !HAS_B) {
    if (!dbc && !mask && !g_out) {
      unsigned i = tid;
      for (; i + (U - 1) * stride < nchunks; i += U * stride) {
        uint4 gv[U], yv[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
          gv[k] = ldg16(dout + (size_t)(i + k * stride) * E);
          yv[k] = ldg16((const T*)A.y + (size_t)(i + k * stride) * E);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
          float g[E], y[E], d[E];
          Chunk<T>::unpack(gv[k], g);
          Chunk<T>::unpack(yv[k], y);
#pragma unroll
          for (int j = 0; j < E; ++j) d[j] = bn_bwd_dy(ka[j], ba[j], ca[j], g[j], y[j]);
          ew_st16<U, NT>((T*)A.dy + (size_t)(i + k * stride) * E, Chunk<T>::pack(d));
        }
      }
      for (; i < nchunks; i += stride) {
        float g[E], y[E], d[E];
        Chunk<T>::unpack(ldg16(dout + (size_t)i * E), g);
        Chunk<T>::unpack(ldg16((const T*)A.y + (size_t)i * E), y);
#pragma unroll
        for (int j = 0; j < E; ++j) d[j] = bn_bwd_dy(ka[j], ba[j], ca[j], g[j], y[j]);
        ew_st16<U, NT>((T*)A.dy + (size_t)i * E, Chunk<T>::pack(d));
      }
      return;
    }
  }
  for (unsigned i = tid; i < nchunks; i += stride) {
    float g[E], mk[E], y[E], d[E];
    if (dbc) {
      unsigned n = (i / (unsigned)cpr) / (unsigned)HW;
#pragma unroll
      for (int j = 0; j < E; ++j) g[j] = dbc[(size_t)n * C + c0 + j] * inv_hw;
    } else {
      Chunk<T>::unpack(ldg16(dout + (size_t)i * E), g);
    }
    if (mask) {
      Chunk<T>::unpack(ldg16(mask + (size_t)i * E), mk);
#pragma unroll
      for (int j = 0; j < E; ++j) g[j] = mk[j] > 0.f ? g[j] : 0.f;
    }
    if (g_out) stg16(g_out + (size_t)i * E, Chunk<T>::pack(g));
    Chunk<T>::unpack(ldg16((const T*)A.y + (size_t)i * E), y);
#pragma unroll
    for (int j = 0; j < E; ++j) d[j] = bn_bwd_dy(ka[j], ba[j], ca[j], g[j], y[j]);
    stg16((T*)A.dy + (size_t)i * E, Chunk<T>::pack(d));
    if (HAS_B) {
      Chunk<T>::unpack(ldg16((const T*)B.y + (size_t)i * E), y);
#pragma unroll
      for (int j = 0; j < E; ++j) d[j] = bn_bwd_dy(kb[j], bb[j], cb[j], g[j], y[j]);
      stg16((T*)B.dy + (size_t)i * E, Chunk<T>::pack(d));
    }
  }
}

// blocked form of the plain bn_bwd_apply (no broadcast gradient, no mask, no
// g_out): dy_a = k_a g + b_a y_a + c_a [, dy_b likewise]; same arithmetic
template <bool HAS_B, bool NTL>
__global__ void __launch_bounds__(256)
bn_bwd_apply_blk_kernel(unsigned nchunks, int cpr, double count, const bf16* __restrict__ dout, BnBwdSide A,
                        BnBwdSide B) {
  constexpr int U = kBlkU;
  const int c0 = (int)(threadIdx.x % (unsigned)cpr) * 8;
  const float inv_count = (float)(1.0 / count);
  float ka[8], ba[8], ca[8], kb[8], bb[8], cb[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    bn_bwd_coef(A.gamma[c], A.istd[c], A.mean[c], A.sum_g[c], A.sum_gx[c], inv_count, ka[j], ba[j], ca[j]);
    if (HAS_B) bn_bwd_coef(B.gamma[c], B.istd[c], B.mean[c], B.sum_g[c], B.sum_gx[c], inv_count, kb[j], bb[j], cb[j]);
  }
  for (unsigned s0 = blockIdx.x * (256u * U); s0 < nchunks; s0 += gridDim.x * (256u * U)) {
    const unsigned i0 = s0 + threadIdx.x;
    uint4 gv[U], yv[U], zv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned i = i0 + 256u * k;
      if (i < nchunks) {
        gv[k] = NTL ? ntl16(dout + (size_t)i * 8) : ldg16(dout + (size_t)i * 8);
        yv[k] = NTL ? ntl16((const bf16*)A.y + (size_t)i * 8) : ldg16((const bf16*)A.y + (size_t)i * 8);
        if constexpr (HAS_B) zv[k] = NTL ? ntl16((const bf16*)B.y + (size_t)i * 8) : ldg16((const bf16*)B.y + (size_t)i * 8);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const unsigned i = i0 + 256u * k;
      if (i >= nchunks) continue;
      float g[8], y[8], d[8];
      Chunk<bf16>::unpack(gv[k], g);
      Chunk<bf16>::unpack(yv[k], y);
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j] = bn_bwd_dy(ka[j], ba[j], ca[j], g[j], y[j]);
      ew_st16<1, true>((bf16*)A.dy + (size_t)i * 8, Chunk<bf16>::pack(d));
      if constexpr (HAS_B) {
        Chunk<bf16>::unpack(zv[k], y);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = bn_bwd_dy(kb[j], bb[j], cb[j], g[j], y[j]);
        ew_st16<1, true>((bf16*)B.dy + (size_t)i * 8, Chunk<bf16>::pack(d));
      }
    }
  }
}

// dgamma = sum(g*xhat), dbeta = sum(g)
__global__ void bn_param_grad_kernel(int C, const double* sum_g, const double* sum_gx, float* dgamma,
                                     float* dbeta) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  dgamma[c] = (float)sum_gx[c];
  dbeta[c] = (float)sum_g[c];
}

// ---- stem: maxpool 3x3/2 pad 1 over relu(sc*y + sh); records the argmax tap ----
template <typename T>
__global__ void __launch_bounds__(256)
maxpool_fwd_kernel(int N, int H, int W, int C, int Ho, int Wo, const T* __restrict__ y,
                   const float* __restrict__ sc, const float* __restrict__ sh, T* __restrict__ out,
                   uint8_t* __restrict__ idx, T* __restrict__ yarg, uint8_t* __restrict__ rmask) {
  constexpr int E = Chunk<T>::N;
  const int cpr = C / E;
  const unsigned total = (unsigned)N * Ho * Wo * cpr;
  const unsigned tid = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned stride = gridDim.x * blockDim.x;
  const int c0 = (int)(tid % (unsigned)cpr) * E;
  float a[E], b[E];
#pragma unroll
  for (int j = 0; j < E; ++j) { a[j] = sc[c0 + j]; b[j] = sh[c0 + j]; }
  for (unsigned i = tid; i < total; i += stride) {
    unsigned p = i / cpr;
    int wo = (int)(p % Wo);
    unsigned t = p / Wo;
    int ho = (int)(t % Ho);
    int n = (int)(t / Ho);
    float best[E], v[E], ya[E];
    uint8_t bi[E];
#pragma unroll
    for (int j = 0; j < E; ++j) { best[j] = -INFINITY; bi[j] = 0; ya[j] = 0.f; }
    // all nine taps are loaded before any is used (clamped in-bounds addresses,
    // validity applied at the compare), so the gathers of a window fly together
    const T* img = y + (size_t)n * H * W * C + c0;
    uint4 raw[9];
    bool ok[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int h = ho * 2 - 1 + k / 3, w = wo * 2 - 1 + k % 3;
      ok[k] = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const int hc = h < 0 ? 0 : (h >= H ? H - 1 : h), wc = w < 0 ? 0 : (w >= W ? W - 1 : w);
      raw[k] = ldg16(img + ((size_t)hc * W + wc) * C);
    }
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      if (!ok[k]) continue;
      Chunk<T>::unpack(raw[k], v);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        float q = fmaxf(fmaf(v[j], a[j], b[j]), 0.f);
        if (q > best[j]) { best[j] = q; bi[j] = (uint8_t)k; ya[j] = v[j]; }
      }
    }
    const uint4 pk = Chunk<T>::pack(best);
    stg16(out + (size_t)p * C + c0, pk);
    if (yarg) stg16(yarg + (size_t)p * C + c0, Chunk<T>::pack(ya));
    if constexpr (E == 8) {
      if (rmask) rmask[((size_t)p * C + c0) >> 3] = relu_bits8(pk);
    }
    if constexpr (E == 8) {
      uint2 packed;
      packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
      packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
      *reinterpret_cast<uint2*>(idx + (size_t)p * C + c0) = packed;
    } else {
      *reinterpret_cast<unsigned*>(idx + (size_t)p * C + c0) =
          bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    }
  }
}

// ---- stem backward: route pooled gradient to argmax, ReLU mask, BN stats ----
// g[n,h,w,c] = sum of dp over the pooled outputs whose recorded argmax is
// (h, w), masked by the stem ReLU (relu(sc*y + sh) > 0).  A block owns
// kMpRows input rows of one image; each thread a FIXED 8-channel chunk column
// and a strided set of pixels, so all index math is shifts and adds.
constexpr int kMpRows = 16;

// An input row h is covered by pooled rows ho = (h + 1 - dh) / 2 for the
// dh in {0,1,2} of matching parity: one candidate (dh = 1) for even h, two
// (dh = 0, 2) for odd h; the same for columns.  All four candidate gathers
// are issued unconditionally (clamped in-bounds addresses, zeroed by their
// validity) so the loads of a pixel fly together instead of one round trip
// per tap.
struct MpCand { int a, b, ta, tb; bool va, vb; };
__device__ __forceinline__ MpCand mp_cand(int h, int Ho) {
  MpCand c;
  if (h & 1) {
    c.a = (h + 1) >> 1; c.ta = 0; c.va = c.a < Ho;
    c.b = (h - 1) >> 1; c.tb = 2; c.vb = true;
  } else {
    c.a = h >> 1; c.ta = 1; c.va = c.a < Ho;
    c.b = c.a; c.tb = 1; c.vb = false;
  }
  c.a = c.a < Ho ? c.a : Ho - 1;
  c.b = c.b < Ho ? c.b : Ho - 1;
  return c;
}

// The gathers of one pixel (4 candidate pooled outputs + argmax taps + y),
// issued as one batch; the kernel keeps the NEXT pixel's batch in flight
// while it finishes the current one.  (vmcnt retires loads and stores in
// issue order: without the prefetch every pixel's loads would also wait for
// the previous pixel's store.)
template <typename T>
struct MpLoads {
  uint4 v[4];
  uint2 ib[4];
  uint4 y;
  unsigned tap4;   // 4 x 8-bit tap of each candidate, 0xff = invalid
};
template <typename T>
__device__ __forceinline__ void mp_fetch(const T* __restrict__ dp, const uint8_t* __restrict__ idx,
                                         const T* __restrict__ y, int n, int h, const MpCand& ch, int w,
                                         int c0, int C, int H, int W, int Ho, int Wo, MpLoads<T>& L) {
  constexpr int E = Chunk<T>::N;
  const MpCand cw = mp_cand(w, Wo);
  L.tap4 = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ho = (q >> 1) ? ch.b : ch.a, wo = (q & 1) ? cw.b : cw.a;
    const int tp = ((q >> 1) ? ch.tb : ch.ta) * 3 + ((q & 1) ? cw.tb : cw.ta);
    const bool ok = ((q >> 1) ? ch.vb : ch.va) && ((q & 1) ? cw.vb : cw.va);
    L.tap4 |= (unsigned)(ok ? tp : 255) << (8 * q);
    const size_t po = (((size_t)n * Ho + ho) * Wo + wo) * C + c0;
    L.v[q] = ldg16(dp + po);
    if constexpr (E == 8) {
      L.ib[q] = *reinterpret_cast<const uint2*>(idx + po);
    } else {
      L.ib[q].x = *reinterpret_cast<const unsigned*>(idx + po);
      L.ib[q].y = 0;
    }
  }
  L.y = ldg16(y + (((size_t)n * H + h) * W + w) * C + c0);
}
template <typename T>
__device__ __forceinline__ void mp_route(const MpLoads<T>& L, float* g) {
  constexpr int E = Chunk<T>::N;
#pragma unroll
  for (int j = 0; j < E; ++j) g[j] = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float f[E];
    Chunk<T>::unpack(L.v[q], f);
    const unsigned tq = (L.tap4 >> (8 * q)) & 255u;
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const unsigned b = (((j >> 2) ? L.ib[q].y : L.ib[q].x) >> (8 * (j & 3))) & 255u;
      g[j] += (b == tq) ? f[j] : 0.f;
    }
  }
}

// APPLY = false: BN backward sums only (sum g, sum g*xhat), nothing written.
// APPLY = true : dy = k*g + b*y + c (the folded BN backward), written in place
//                of the routed gradient, which is never materialised.
template <typename T, bool APPLY>
__global__ void __launch_bounds__(256)
maxpool_bwd_kernel(int N, int H, int W, int C, int Ho, int Wo, const T* __restrict__ dp,
                   const uint8_t* __restrict__ idx, const T* __restrict__ y,
                   const float* __restrict__ sc, const float* __restrict__ sh,
                   const float* __restrict__ mean, const float* __restrict__ istd,
                   const float* __restrict__ gamma, const double* __restrict__ sg,
                   const double* __restrict__ sgx, T* __restrict__ dy, double* sum_g, double* sum_gx,
                   int rep) {
  constexpr int E = Chunk<T>::N;
  const int cpr = C / E;
  const int t = threadIdx.x;
  const int cc = t % cpr, c0 = cc * E;
  const int wstep = 256 / cpr;
  const int rb = blockIdx.x % ((H + kMpRows - 1) / kMpRows);
  const int n = blockIdx.x / ((H + kMpRows - 1) / kMpRows);
  float a[E], b[E], mu[E], is[E], ka[E], ba[E], ca[E], ag[E], ax[E];
  const float inv_count = 1.f / (float)((double)N * H * W);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int c = c0 + j;
    a[j] = sc[c]; b[j] = sh[c]; mu[j] = mean[c]; is[j] = istd[c];
    ag[j] = ax[j] = 0.f;
    if constexpr (APPLY) {
      const float k = gamma[c] * is[j];
      const float mg = (float)(sg[c] * (double)inv_count), mgx = (float)(sgx[c] * (double)inv_count);
      ka[j] = k; ba[j] = -k * is[j] * mgx; ca[j] = -k * mg + k * is[j] * mgx * mu[j];
    }
  }
  const int w0 = t / cpr;
  const int nw = w0 < W ? (W - w0 + wstep - 1) / wstep : 0;
  int rows = H - rb * kMpRows;
  if (rows > kMpRows) rows = kMpRows;
  const int total = rows * nw;
  if constexpr (!APPLY) {
    // stats pass: no stores, so plain nested walk (loads of consecutive
    // pixels are free to overlap)
    for (int r = 0; r < rows; ++r) {
      const int h = rb * kMpRows + r;
      const MpCand ch = mp_cand(h, Ho);
#pragma unroll 2
      for (int w = w0; w < W; w += wstep) {
        MpLoads<T> L;
        mp_fetch<T>(dp, idx, y, n, h, ch, w, c0, C, H, W, Ho, Wo, L);
        float g[E], yv[E];
        mp_route<T>(L, g);
        Chunk<T>::unpack(L.y, yv);
#pragma unroll
        for (int j = 0; j < E; ++j) {
          const float gg = fmaf(yv[j], a[j], b[j]) > 0.f ? g[j] : 0.f;
          ag[j] += gg;
          ax[j] += gg * ((yv[j] - mu[j]) * is[j]);
        }
      }
    }
    __shared__ float red[2][256][E];
#pragma unroll
    for (int j = 0; j < E; ++j) { red[0][t][j] = ag[j]; red[1][t][j] = ax[j]; }
    __syncthreads();
    if (t < cpr) {
      for (int q = t + cpr; q < 256; q += cpr)
#pragma unroll
        for (int j = 0; j < E; ++j) { ag[j] += red[0][q][j]; ax[j] += red[1][q][j]; }
      const size_t ro = (size_t)(blockIdx.x % rep) * C + c0;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        atomicAdd(sum_g + ro + j, (double)ag[j]);
        atomicAdd(sum_gx + ro + j, (double)ax[j]);
      }
    }
    return;
  }
  // apply pass: flattened (row, pixel) walk, one pixel's gathers ahead
  MpLoads<T> cur, nxt;
  if (total > 0) {
    const int h = rb * kMpRows;
    mp_fetch<T>(dp, idx, y, n, h, mp_cand(h, Ho), w0, c0, C, H, W, Ho, Wo, cur);
  }
  for (int it = 0; it < total; ++it) {
    const int r = it / nw, jw = it - r * nw;
    const int h = rb * kMpRows + r, w = w0 + jw * wstep;
    if (it + 1 < total) {
      const int r1 = (it + 1) / nw, j1 = it + 1 - r1 * nw;
      const int h1 = rb * kMpRows + r1;
      mp_fetch<T>(dp, idx, y, n, h1, mp_cand(h1, Ho), w0 + j1 * wstep, c0, C, H, W, Ho, Wo, nxt);
    }
    float g[E], yv[E], d[E];
    mp_route<T>(cur, g);
    Chunk<T>::unpack(cur.y, yv);
#pragma unroll
    for (int j = 0; j < E; ++j) {
      const float gg = fmaf(yv[j], a[j], b[j]) > 0.f ? g[j] : 0.f;
      d[j] = fmaf(ka[j], gg, fmaf(ba[j], yv[j], ca[j]));
    }
    stg16(dy + (((size_t)n * H + h) * W + w) * C + c0, Chunk<T>::pack(d));
    cur = nxt;
  }
}

// ---- stem backward on 2x2 input blocks (H, W even) ----
// Input rows {2a, 2a+1} x cols {2b, 2b+1} are covered by exactly the pooled
// outputs (a|a+1, b|b+1), so one set of four dp/idx gathers serves four input
// pixels (the per-pixel walk above issues four gathers per pixel).  Taps
// kh*3+kw: (2a,2b) <- P00 tap 4; (2a,2b+1) <- P00 tap 5, P01 tap 3;
// (2a+1,2b) <- P00 tap 7, P10 tap 1; (2a+1,2b+1) <- P00 8, P01 6, P10 2, P11 0.
constexpr int kMpPairs = 8;   // row pairs per block (16 input rows)
template <typename T>
struct Mp4Loads {
  uint4 p[4];     // dp at (a,b) (a,b+1) (a+1,b) (a+1,b+1)
  uint2 ib[4];
  uint4 y[4];     // y at (2a,2b) (2a,2b+1) (2a+1,2b) (2a+1,2b+1)
  bool v01, v10;
};
template <typename T>
__device__ __forceinline__ void mp4_fetch(const T* __restrict__ dp, const uint8_t* __restrict__ idx,
                                          const T* __restrict__ y, int n, int a, int b, int c0, int C,
                                          int H, int W, int Ho, int Wo, Mp4Loads<T>& L) {
  L.v10 = a + 1 < Ho;
  L.v01 = b + 1 < Wo;
  const int a1 = L.v10 ? a + 1 : a, b1 = L.v01 ? b + 1 : b;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int ho = (q >> 1) ? a1 : a, wo = (q & 1) ? b1 : b;
    const size_t po = (((size_t)n * Ho + ho) * Wo + wo) * C + c0;
    L.p[q] = ldg16(dp + po);
    if constexpr (Chunk<T>::N == 8) {
      L.ib[q] = *reinterpret_cast<const uint2*>(idx + po);
    } else {
      L.ib[q].x = *reinterpret_cast<const unsigned*>(idx + po);
      L.ib[q].y = 0;
    }
    const size_t yo = (((size_t)n * H + 2 * a + (q >> 1)) * W + 2 * b + (q & 1)) * C + c0;
    L.y[q] = ldg16(y + yo);
  }
}
template <typename T>
__device__ __forceinline__ void mp4_route(const Mp4Loads<T>& L, float (*g)[Chunk<T>::N]) {
  constexpr int E = Chunk<T>::N;
  float f[4][E];
#pragma unroll
  for (int q = 0; q < 4; ++q) Chunk<T>::unpack(L.p[q], f[q]);
  const bool v11 = L.v01 && L.v10;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    unsigned t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = (((j >> 2) ? L.ib[q].y : L.ib[q].x) >> (8 * (j & 3))) & 255u;
    g[0][j] = t[0] == 4u ? f[0][j] : 0.f;
    g[1][j] = (t[0] == 5u ? f[0][j] : 0.f) + ((L.v01 && t[1] == 3u) ? f[1][j] : 0.f);
    g[2][j] = (t[0] == 7u ? f[0][j] : 0.f) + ((L.v10 && t[2] == 1u) ? f[2][j] : 0.f);
    g[3][j] = (t[0] == 8u ? f[0][j] : 0.f) + ((L.v01 && t[1] == 6u) ? f[1][j] : 0.f) +
              ((L.v10 && t[2] == 2u) ? f[2][j] : 0.f) + ((v11 && t[3] == 0u) ? f[3][j] : 0.f);
  }
}

template <typename T, bool APPLY>
__global__ void __launch_bounds__(256)
maxpool_bwd2_kernel(int N, int H, int W, int C, int Ho, int Wo, const T* __restrict__ dp,
                    const uint8_t* __restrict__ idx, const T* __restrict__ y,
                    const float* __restrict__ sc, const float* __restrict__ sh,
                    const float* __restrict__ mean, const float* __restrict__ istd,
                    const float* __restrict__ gamma, const double* __restrict__ sg,
                    const double* __restrict__ sgx, T* __restrict__ dy, double* sum_g, double* sum_gx,
                    int rep) {
  constexpr int E = Chunk<T>::N;
  const int cpr = C / E;
  const int t = threadIdx.x;
  const int c0 = (t % cpr) * E;
  const int bstep = 256 / cpr;
  const int HP = H / 2, WP = W / 2;
  const int bands = (HP + kMpPairs - 1) / kMpPairs;
  const int band = blockIdx.x % bands;
  const int n = blockIdx.x / bands;
  float a[E], b[E], mu[E], is[E], ka[E], ba[E], ca[E], ag[E], ax[E];
  const float inv_count = 1.f / (float)((double)N * H * W);
#pragma unroll
  for (int j = 0; j < E; ++j) {
    const int c = c0 + j;
    a[j] = sc[c]; b[j] = sh[c]; mu[j] = mean[c]; is[j] = istd[c];
    ag[j] = ax[j] = 0.f;
    if constexpr (APPLY) {
      const float k = gamma[c] * is[j];
      const float mg = (float)(sg[c] * (double)inv_count), mgx = (float)(sgx[c] * (double)inv_count);
      ka[j] = k; ba[j] = -k * is[j] * mgx; ca[j] = -k * mg + k * is[j] * mgx * mu[j];
    } else {
      ka[j] = ba[j] = ca[j] = 0.f;
    }
  }
  const int b0 = t / cpr;
  const int nb = b0 < WP ? (WP - b0 + bstep - 1) / bstep : 0;
  int pairs = HP - band * kMpPairs;
  if (pairs > kMpPairs) pairs = kMpPairs;
  const int total = pairs * nb;
  Mp4Loads<T> cur, nxt;
  if (total > 0) mp4_fetch<T>(dp, idx, y, n, band * kMpPairs, b0, c0, C, H, W, Ho, Wo, cur);
  for (int it = 0; it < total; ++it) {
    const int r = it / nb, jb = it - r * nb;
    const int pa = band * kMpPairs + r, pb = b0 + jb * bstep;
    if (it + 1 < total) {
      const int r1 = (it + 1) / nb, j1 = it + 1 - r1 * nb;
      mp4_fetch<T>(dp, idx, y, n, band * kMpPairs + r1, b0 + j1 * bstep, c0, C, H, W, Ho, Wo, nxt);
    }
    float g[4][E];
    mp4_route<T>(cur, g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float yv[E], d[E];
      Chunk<T>::unpack(cur.y[q], yv);
#pragma unroll
      for (int j = 0; j < E; ++j) {
        const float gg = fmaf(yv[j], a[j], b[j]) > 0.f ? g[q][j] : 0.f;
        if constexpr (APPLY) {
          d[j] = fmaf(ka[j], gg, fmaf(ba[j], yv[j], ca[j]));
        } else {
          ag[j] += gg;
          ax[j] += gg * ((yv[j] - mu[j]) * is[j]);
        }
      }
      if constexpr (APPLY)
        stg16(dy + (((size_t)n * H + 2 * pa + (q >> 1)) * W + 2 * pb + (q & 1)) * C + c0, Chunk<T>::pack(d));
    }
    cur = nxt;
  }
  if constexpr (!APPLY) {
    __shared__ float red[2][256][E];
#pragma unroll
    for (int j = 0; j < E; ++j) { red[0][t][j] = ag[j]; red[1][t][j] = ax[j]; }
    __syncthreads();
    if (t < cpr) {
      for (int q = t + cpr; q < 256; q += cpr)
#pragma unroll
        for (int j = 0; j < E; ++j) { ag[j] += red[0][q][j]; ax[j] += red[1][q][j]; }
      const size_t ro = (size_t)(blockIdx.x % rep) * C + c0;
#pragma unroll
      for (int j = 0; j < E; ++j) {
        atomicAdd(sum_g + ro + j, (double)ag[j]);
        atomicAdd(sum_gx + ro + j, (double)ax[j]);
      }
    }
  }
}

// ---- global average pool: feat[n][c] = mean_hw x[n][hw][c] ----
template <typename T>
__global__ void avgpool_fwd_kernel(int N, int HW, int C, const T* __restrict__ x, T* __restrict__ feat) {
  int n = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int p = 0; p < HW; ++p) s += to_f(x[((size_t)n * HW + p) * C + c]);
    feat[(size_t)n * C + c] = from_f<T>(s / (float)HW);
  }
}

// 16-B loads: thread t owns 8 (bf16) / 4 (fp32) channels of every G-th pixel
// (G = 256 / (C / EPC) pixel lanes per image), the G partial sums meet in LDS in
// a fixed order.  One image per 256-thread block; 16-B rows instead of one
// 2-byte load per thread per pixel (r4: 203 us per bs = 256 step before).
template <typename T>
__global__ void __launch_bounds__(256) avgpool_fwd_vec_kernel(int N, int HW, int C, const T* __restrict__ x,
                                                              T* __restrict__ feat) {
  constexpr int EPC = 16 / (int)sizeof(T);
  extern __shared__ float red[];   // [G][C]
  const int CP = C / EPC, G = 256 / CP;
  const int n = blockIdx.x, t = threadIdx.x, cc = t % CP, pg = t / CP;
  float s[EPC];
#pragma unroll
  for (int j = 0; j < EPC; ++j) s[j] = 0.f;
  const T* xn = x + (size_t)n * HW * C + cc * EPC;
  for (int p = pg; p < HW; p += G) {
    float v[EPC];
    Chunk<T>::unpack(ldg16(xn + (size_t)p * C), v);
#pragma unroll
    for (int j = 0; j < EPC; ++j) s[j] += v[j];
  }
#pragma unroll
  for (int j = 0; j < EPC; ++j) red[pg * C + cc * EPC + j] = s[j];
  __syncthreads();
  const float inv = 1.f / (float)HW;
  for (int c = t; c < C; c += 256) {
    float a = 0.f;
    for (int g = 0; g < G; ++g) a += red[g * C + c];
    feat[(size_t)n * C + c] = from_f<T>(a * inv);
  }
}

// grid whose total thread count is a multiple of cpr (256 % cpr == 0)
static inline int ew_grid(size_t nchunks) { return ew_blocks(nchunks, 256, 4096); }
// streaming-pass variants (A/B switches VLP_EW for bn_add_relu, VLP_EWB for
// bn_bwd_apply): 0 one chunk per iteration, 1 / 2 two / four chunks per
// iteration, 3 four + non-temporal stores, 4 non-temporal stores.  Measured
// (tools/ew_bench.py, bs = 256): unrolling loses at every size; non-temporal
// stores take bn_add_relu from 4.8-4.9 to 5.2-6.3 TB/s at layers 1-2 and do
// not help bn_bwd_apply, so the defaults are 4 and 0.
// r6: the blocked streaming layout (bn_add_relu_blk_kernel, bn_bwd_apply_blk_kernel)
// for the bf16 passes, chosen per pass and per-tensor size from tools/ew_bench.py
// at the bs = 256 ResNet34 sizes (three libraries interleaved x2 on one box,
// profiles/r6_ew_blocked_ab.txt; us per launch, old / blocked / blocked + NT loads):
//   bn_add_relu, no residual: 128^2x64 208 / 206 / 198, 64^2x128 85 / 89 / 104,
//                             32^2x256 47 / 49 / 57, 16^2x512 37 / 29 / 34
//   bn_add_relu + residual + mask bits: 362 / 287 / 278, 159 / 152 / 147, 70 / 75 / 82, 40 / 42 / 48
//   bn_bwd_apply: 318 / 292 / 273, 153 / 145 / 138, 78 / 60 / 72, 33 / 32 / 39
// Non-temporal loads pay only for tensors past the 256 MB MALL (at smaller sizes
// the producer's output may still be there).  0: the thread-strided kernels below,
// 1: blocked, 2: blocked + non-temporal loads.  VLP_EW_BLK=0 forces 0.
#ifndef VLP_EW_BLK
#define VLP_EW_BLK 1
#endif
static inline int ew_form_add_relu(size_t tensor_bytes, bool residual) {
  if (!VLP_EW_BLK) return 0;
  const size_t MB = 1u << 20;
  if (residual) return tensor_bytes >= 256 * MB ? 2 : 0;
  return tensor_bytes >= 512 * MB ? 2 : (tensor_bytes <= 100 * MB ? 1 : 0);
}
static inline int ew_form_bwd_apply(size_t tensor_bytes) {
  if (!VLP_EW_BLK) return 0;
  return tensor_bytes >= (256u << 20) ? 2 : 1;
}
static inline int ew_variant() {
  return 4;
}
static inline int ewb_variant() {
  return 0;
}

}  // namespace vlp

using namespace vlp;

VLP_EXPORT int vlp_bn_finalize(int C, double count, const double* sum, const double* sumsq,
                               const float* gamma, const float* beta, float eps, float momentum,
                               float* running_mean, float* running_var, float* scale, float* shift,
                               float* mean, float* invstd, void* stream) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C,
                     count, sum, sumsq, gamma, beta, eps, momentum, running_mean, running_var, scale,
                     shift, mean, invstd);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* rm,
                                  const float* rv, float eps, float* scale, float* shift,
                                  void* stream) {
  hipLaunchKernelGGL(bn_eval_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C,
                     gamma, beta, rm, rv, eps, scale, shift);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_finalize_rep(int rep, int C, double count, double* sum, double* sumsq,
                                   const float* gamma, const float* beta, float eps, float momentum,
                                   float* running_mean, float* running_var, float* scale, float* shift,
                                   float* mean, float* invstd, void* stream) {
  if (rep < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_finalize_rep_kernel, dim3((C + 63) / 64), dim3(64 * kFoldWaves), 0, (hipStream_t)stream, rep, C,
                     count, sum, sumsq, gamma, beta, eps, momentum, running_mean, running_var, scale, shift, mean,
                     invstd);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_grad_rep(int rep, int C, double* sum_g, double* sum_gx, double* sum_gxd, float* dgamma,
                               float* dbeta, float* dgamma_d, float* dbeta_d, void* stream) {
  if (rep < 1 || (sum_gxd == nullptr) != (dgamma_d == nullptr)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_grad_rep_kernel, dim3((C + 63) / 64), dim3(64 * kFoldWaves), 0, (hipStream_t)stream, rep, C, sum_g,
                     sum_gx, sum_gxd, dgamma, dbeta, dgamma_d, dbeta_d);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_stat_reduce(int rep, int C, double* a, double* b, double* c, void* stream) {
  if (rep <= 1) return 0;
  hipLaunchKernelGGL(stat_reduce_kernel, dim3((C + 63) / 64, 3), dim3(256), 0, (hipStream_t)stream,
                     rep, C, a, b, c);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_add_relu(int dtype, long long M, int C, const void* y, const float* sc,
                               const float* sh, const void* idt, const float* scd, const float* shd,
                               void* out, uint8_t* relu_mask, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int epc = dtype == VLP_BF16 ? 8 : 4;
  if (relu_mask && dtype != VLP_BF16) return (int)hipErrorInvalidValue;
  unsigned n = (unsigned)((size_t)M * C / epc);
  int cpr = C / epc;
  if (256 % cpr) return (int)hipErrorInvalidValue;
  dim3 g(ew_grid(n));
  const int form = dtype == VLP_BF16 ? ew_form_add_relu((size_t)n * 16, idt != nullptr) : 0;
  if (form > 0) {
#define VLP_ADD_RELU_BLK(NTL)                                                                                     \
    if (idt)                                                                                                      \
      hipLaunchKernelGGL((bn_add_relu_blk_kernel<true, NTL>), dim3(blk_grid(n)), dim3(256), 0, st, n, cpr,        \
                         (const bf16*)y, sc, sh, (const bf16*)idt, scd, shd, (bf16*)out, relu_mask);               \
    else                                                                                                          \
      hipLaunchKernelGGL((bn_add_relu_blk_kernel<false, NTL>), dim3(blk_grid(n)), dim3(256), 0, st, n, cpr,       \
                         (const bf16*)y, sc, sh, (const bf16*)idt, scd, shd, (bf16*)out, relu_mask);
    if (form == 2) { VLP_ADD_RELU_BLK(true) } else { VLP_ADD_RELU_BLK(false) }
#undef VLP_ADD_RELU_BLK
  } else if (dtype == VLP_BF16) {
    switch (ew_variant()) {
#define VLP_ADD_RELU(U, NT)                                                                                    \
  if (idt)                                                                                                     \
    hipLaunchKernelGGL((bn_add_relu_kernel<bf16, true, U, NT>), g, dim3(256), 0, st, n, cpr, (const bf16*)y,  \
                       sc, sh, (const bf16*)idt, scd, shd, (bf16*)out, relu_mask);                             \
  else                                                                                                         \
    hipLaunchKernelGGL((bn_add_relu_kernel<bf16, false, U, NT>), g, dim3(256), 0, st, n, cpr, (const bf16*)y, \
                       sc, sh, (const bf16*)idt, scd, shd, (bf16*)out, relu_mask);                             \
  break;
      case 1: VLP_ADD_RELU(2, false)
      case 2: VLP_ADD_RELU(4, false)
      case 3: VLP_ADD_RELU(4, true)
      case 4: VLP_ADD_RELU(1, true)
      default: VLP_ADD_RELU(1, false)
#undef VLP_ADD_RELU
    }
  } else {
    if (idt)
      hipLaunchKernelGGL((bn_add_relu_kernel<float, true>), g, dim3(256), 0, st, n, cpr, (const float*)y,
                         sc, sh, (const float*)idt, scd, shd, (float*)out, nullptr);
    else
      hipLaunchKernelGGL((bn_add_relu_kernel<float, false>), g, dim3(256), 0, st, n, cpr,
                         (const float*)y, sc, sh, (const float*)idt, scd, shd, (float*)out, nullptr);
  }
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_bwd_reduce(int dtype, long long M, int C, const void* dout, const float* dbc,
                                 int HW, const void* mask, const void* ya, const float* mean_a,
                                 const float* istd_a, const void* yb, const float* mean_b,
                                 const float* istd_b, double* sum_g, double* sum_ga, double* sum_gb,
                                 int stat_rep, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int epc = dtype == VLP_BF16 ? 8 : 4;
  int rows_per_iter = 256 / (C / epc);
  int blocks = ew_blocks((size_t)M, rows_per_iter * 16, 2048);
  if (stat_rep < 1) stat_rep = 1;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (int)M, C,
                       (const bf16*)dout, dbc, HW, (const bf16*)mask, (const bf16*)ya, mean_a, istd_a,
                       (const bf16*)yb, mean_b, istd_b, sum_g, sum_ga, sum_gb, stat_rep);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, (int)M, C,
                       (const float*)dout, dbc, HW, (const float*)mask, (const float*)ya, mean_a,
                       istd_a, (const float*)yb, mean_b, istd_b, sum_g, sum_ga, sum_gb, stat_rep);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_bwd_apply(int dtype, long long M, int C, const void* dout, const float* dbc,
                                int HW, const void* mask,
                                const void* ya, const float* mean_a, const float* istd_a,
                                const float* gamma_a, const double* sum_g_a, const double* sum_gx_a,
                                void* dy_a,
                                const void* yb, const float* mean_b, const float* istd_b,
                                const float* gamma_b, const double* sum_g_b, const double* sum_gx_b,
                                void* dy_b, void* g_out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  BnBwdSide A{ya, mean_a, istd_a, gamma_a, sum_g_a, sum_gx_a, dy_a};
  BnBwdSide B{yb, mean_b, istd_b, gamma_b, sum_g_b, sum_gx_b, dy_b};
  int epc = dtype == VLP_BF16 ? 8 : 4;
  int cpr = C / epc;
  if (256 % cpr) return (int)hipErrorInvalidValue;
  unsigned n = (unsigned)((size_t)M * C / epc);
  dim3 g(ew_grid(n));
  bool hb = dy_b != nullptr;
  const int form = dtype == VLP_BF16 && !dbc && !mask && !g_out ? ew_form_bwd_apply((size_t)n * 16) : 0;
  if (form > 0) {
#define VLP_BWD_APPLY_BLK(NTL)                                                                                     \
    if (hb)                                                                                                        \
      hipLaunchKernelGGL((bn_bwd_apply_blk_kernel<true, NTL>), dim3(blk_grid(n)), dim3(256), 0, st, n, cpr,        \
                         (double)M, (const bf16*)dout, A, B);                                                      \
    else                                                                                                           \
      hipLaunchKernelGGL((bn_bwd_apply_blk_kernel<false, NTL>), dim3(blk_grid(n)), dim3(256), 0, st, n, cpr,       \
                         (double)M, (const bf16*)dout, A, B);
    if (form == 2) { VLP_BWD_APPLY_BLK(true) } else { VLP_BWD_APPLY_BLK(false) }
#undef VLP_BWD_APPLY_BLK
  } else if (dtype == VLP_BF16) {
    if (hb)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, true>), g, dim3(256), 0, st, n, cpr, (double)M,
                         (const bf16*)dout, dbc, HW, (const bf16*)mask, A, B, (bf16*)g_out);
    else {
      switch (ewb_variant()) {
#define VLP_BWD_APPLY(U, NT)                                                                            \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, false, U, NT>), g, dim3(256), 0, st, n, cpr, (double)M, \
                     (const bf16*)dout, dbc, HW, (const bf16*)mask, A, B, (bf16*)g_out);               \
  break;
        case 1: VLP_BWD_APPLY(2, false)
        case 2: VLP_BWD_APPLY(4, false)
        case 3: VLP_BWD_APPLY(4, true)
        case 4: VLP_BWD_APPLY(1, true)
        default: VLP_BWD_APPLY(1, false)
#undef VLP_BWD_APPLY
      }
    }
  } else {
    if (hb)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<float, true>), g, dim3(256), 0, st, n, cpr, (double)M,
                         (const float*)dout, dbc, HW, (const float*)mask, A, B, (float*)g_out);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<float, false>), g, dim3(256), 0, st, n, cpr, (double)M,
                         (const float*)dout, dbc, HW, (const float*)mask, A, B, (float*)g_out);
  }
  return (int)hipGetLastError();
}

// k, b, c of the folded BN backward (bn_bwd_coef) -> coef[3][C]: the input
// transform table of the layer-1 rows kernel's data gradient (vlp_conv_dgrad_*_act)
__global__ void bn_bwd_coef_kernel(int C, float inv_count, const float* __restrict__ gamma,
                                   const float* __restrict__ istd, const float* __restrict__ mean,
                                   const double* __restrict__ sum_g, const double* __restrict__ sum_gx,
                                   float* __restrict__ coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float k, b, cc;
  bn_bwd_coef(gamma[c], istd[c], mean[c], sum_g[c], sum_gx[c], inv_count, k, b, cc);
  coef[c] = k;
  coef[C + c] = b;
  coef[2 * C + c] = cc;
}

VLP_EXPORT int vlp_bn_bwd_coef(long long M, int C, const float* gamma, const float* istd, const float* mean,
                               const double* sum_g, const double* sum_gx, float* coef, void* stream) {
  if (M < 1 || C < 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C,
                     (float)(1.0 / (double)M), gamma, istd, mean, sum_g, sum_gx, coef);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_bn_param_grad(int C, const double* sum_g, const double* sum_gx, float* dgamma,
                                 float* dbeta, void* stream) {
  hipLaunchKernelGGL(bn_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                     C, sum_g, sum_gx, dgamma, dbeta);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_maxpool_fwd(int dtype, int N, int H, int W, int C, const void* y, const float* sc,
                               const float* sh, void* out, uint8_t* idx, void* yarg, uint8_t* relu_mask,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (relu_mask && dtype != VLP_BF16) return (int)hipErrorInvalidValue;
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  int epc = dtype == VLP_BF16 ? 8 : 4;
  size_t n = (size_t)N * Ho * Wo * (C / epc);
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16>, dim3(ew_grid(n)), dim3(256), 0, st, N, H, W, C, Ho,
                       Wo, (const bf16*)y, sc, sh, (bf16*)out, idx, (bf16*)yarg, relu_mask);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(ew_grid(n)), dim3(256), 0, st, N, H, W, C, Ho,
                       Wo, (const float*)y, sc, sh, (float*)out, idx, (float*)yarg, nullptr);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_maxpool_bwd(int dtype, int N, int H, int W, int C, const void* dp,
                               const uint8_t* idx, const void* y, const float* sc, const float* sh,
                               const float* mean, const float* istd, double* sum_g,
                               double* sum_gx, int stat_rep, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  int epc = dtype == VLP_BF16 ? 8 : 4;
  if (256 % (C / epc)) return (int)hipErrorInvalidValue;
  if (stat_rep < 1) stat_rep = 1;
  if (!(H & 1) && !(W & 1)) {
    dim3 g2((unsigned)(N * ((H / 2 + kMpPairs - 1) / kMpPairs)));
    if (dtype == VLP_BF16)
      hipLaunchKernelGGL((maxpool_bwd2_kernel<bf16, false>), g2, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                         (const bf16*)dp, idx, (const bf16*)y, sc, sh, mean, istd, nullptr, nullptr,
                         nullptr, nullptr, sum_g, sum_gx, stat_rep);
    else
      hipLaunchKernelGGL((maxpool_bwd2_kernel<float, false>), g2, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                         (const float*)dp, idx, (const float*)y, sc, sh, mean, istd, nullptr, nullptr,
                         nullptr, nullptr, sum_g, sum_gx, stat_rep);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)(N * ((H + kMpRows - 1) / kMpRows)));
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL((maxpool_bwd_kernel<bf16, false>), grid, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                       (const bf16*)dp, idx, (const bf16*)y, sc, sh, mean, istd, nullptr, nullptr, nullptr,
                       nullptr, sum_g, sum_gx, stat_rep);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<float, false>), grid, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                       (const float*)dp, idx, (const float*)y, sc, sh, mean, istd, nullptr, nullptr,
                       nullptr, nullptr, sum_g, sum_gx, stat_rep);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_maxpool_bwd_apply(int dtype, int N, int H, int W, int C, const void* dp,
                                     const uint8_t* idx, const void* y, const float* sc,
                                     const float* sh, const float* mean, const float* istd,
                                     const float* gamma, const double* sum_g, const double* sum_gx,
                                     void* dy, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int Ho = (H + 2 - 3) / 2 + 1, Wo = (W + 2 - 3) / 2 + 1;
  int epc = dtype == VLP_BF16 ? 8 : 4;
  if (256 % (C / epc)) return (int)hipErrorInvalidValue;
  if (!(H & 1) && !(W & 1)) {
    dim3 g2((unsigned)(N * ((H / 2 + kMpPairs - 1) / kMpPairs)));
    if (dtype == VLP_BF16)
      hipLaunchKernelGGL((maxpool_bwd2_kernel<bf16, true>), g2, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                         (const bf16*)dp, idx, (const bf16*)y, sc, sh, mean, istd, gamma, sum_g, sum_gx,
                         (bf16*)dy, nullptr, nullptr, 1);
    else
      hipLaunchKernelGGL((maxpool_bwd2_kernel<float, true>), g2, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                         (const float*)dp, idx, (const float*)y, sc, sh, mean, istd, gamma, sum_g, sum_gx,
                         (float*)dy, nullptr, nullptr, 1);
    return (int)hipGetLastError();
  }
  dim3 grid((unsigned)(N * ((H + kMpRows - 1) / kMpRows)));
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL((maxpool_bwd_kernel<bf16, true>), grid, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                       (const bf16*)dp, idx, (const bf16*)y, sc, sh, mean, istd, gamma, sum_g, sum_gx,
                       (bf16*)dy, nullptr, nullptr, 1);
  else
    hipLaunchKernelGGL((maxpool_bwd_kernel<float, true>), grid, dim3(256), 0, st, N, H, W, C, Ho, Wo,
                       (const float*)dp, idx, (const float*)y, sc, sh, mean, istd, gamma, sum_g, sum_gx,
                       (float*)dy, nullptr, nullptr, 1);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_avgpool_fwd(int dtype, int N, int HW, int C, const void* x, void* feat,
                               void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int epc = dtype == VLP_BF16 ? 8 : 4;
  if (N > 0 && C % epc == 0 && C / epc <= 256 && 256 % (C / epc) == 0 && C * (256 / (C / epc)) * 4 <= 65536) {
    const size_t lds = (size_t)C * (256 / (C / epc)) * sizeof(float);
    if (dtype == VLP_BF16)
      hipLaunchKernelGGL(avgpool_fwd_vec_kernel<bf16>, dim3(N), dim3(256), lds, st, N, HW, C, (const bf16*)x,
                         (bf16*)feat);
    else
      hipLaunchKernelGGL(avgpool_fwd_vec_kernel<float>, dim3(N), dim3(256), lds, st, N, HW, C, (const float*)x,
                         (float*)feat);
    return (int)hipGetLastError();
  }
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(avgpool_fwd_kernel<bf16>, dim3(N), dim3(256), 0, st, N, HW, C, (const bf16*)x,
                       (bf16*)feat);
  else
    hipLaunchKernelGGL(avgpool_fwd_kernel<float>, dim3(N), dim3(256), 0, st, N, HW, C,
                       (const float*)x, (float*)feat);
  return (int)hipGetLastError();
}
