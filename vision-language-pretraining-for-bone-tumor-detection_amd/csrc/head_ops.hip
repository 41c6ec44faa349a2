// CLIP contrastive head (reference src/models/pretrain/VisionLanguageModule.py
// forward :441-461 and _compute_loss :532-554):
//   img = normalize(f_img @ P_img), txt = normalize(f_txt @ P_txt)   (eps 1e-12)
//   s = min(exp(logit_scale), 100);  logits = s * img @ txt^T
//   loss = (CE(logits, arange) + CE(logits^T, arange)) / 2
//
// `vlp_clip_loss_fused` computes the loss AND its gradients in one LDS-tiled
// launch, for the global batch of a data-parallel job: each rank owns B rows
// (images) and B columns (texts) of the N x N logits matrix (N = B * world,
// its rows start at `offset`).  Workgroups of role 0 sweep their 16 local image
// rows against all N texts (row log-sum-exp, image->text CE), role-1
// workgroups sweep 16 local text columns against all N images (text->image
// CE).  Each does two passes over the key tiles held in LDS: online LSE, then
// p = exp(l - lse) and the analytic backward
//   dl_ij = (p_ij - [i == j]) / (2N)
//   dq_i += s * dl_ij k_j   ;   dk_j += s * dl_ij q_i   ;   ds += dl_ij * cos_ij
// Gradients w.r.t. the gathered [N][E] embeddings are accumulated with fp32
// atomics; the owner's rows are then reduce-scattered by the host (RCCL).
#include "gemm.h"

namespace vlp {

constexpr int kQ = 16;        // queries per workgroup
constexpr int kKT = 64;       // keys per LDS tile
constexpr int kMaxE = 256;

__global__ void __launch_bounds__(256)
clip_loss_fused_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
                       const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
                       float* __restrict__ g_img_all, float* __restrict__ g_txt_all,
                       float* __restrict__ d_logit_scale, float* __restrict__ loss_parts,
                       float* __restrict__ lse_out) {
  __shared__ float Q[kQ][kMaxE + 1];
  __shared__ float K[kKT][kMaxE + 1];
  __shared__ float Wt[kQ][kKT + 1];
  __shared__ float lse_s[kQ];
  __shared__ float red[256];

  const int nqb = (B + kQ - 1) / kQ;
  const int role = blockIdx.x / nqb;            // 0: image rows, 1: text columns
  const int q0 = (blockIdx.x % nqb) * kQ;       // local query index
  const float* qsrc = role == 0 ? img_all : txt_all;
  const float* ksrc = role == 0 ? txt_all : img_all;
  float* gq = role == 0 ? g_img_all : g_txt_all;
  float* gk = role == 0 ? g_txt_all : g_img_all;

  const float ls = logit_scale[0];
  const float ex = expf(ls);
  const float s = fminf(ex, 100.f);
  const float inv2n = 0.5f / (float)N;
  const int t = threadIdx.x;
  const int qi = t >> 4, kj = t & 15;           // thread -> (query, key lane)
  const bool qvalid = (q0 + qi) < B;
  const int qglob = offset + q0 + qi;

  for (int e = t; e < kQ * E; e += 256) {
    int i = e / E, d = e % E;
    Q[i][d] = (q0 + i) < B ? qsrc[(size_t)(offset + q0 + i) * E + d] : 0.f;
  }

  // ---- pass 1: online log-sum-exp over all N keys ----
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < N; k0 += kKT) {
    __syncthreads();
    for (int e = t; e < kKT * E; e += 256) {
      int j = e / E, d = e % E;
      K[j][d] = (k0 + j) < N ? ksrc[(size_t)(k0 + j) * E + d] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kKT / 16; ++r) {
      int j = kj + 16 * r;
      if (k0 + j < N) {
        float dot = 0.f;
        for (int d = 0; d < E; ++d) dot += Q[qi][d] * K[j][d];
        float lg = s * dot;
        float mn = fmaxf(m, lg);
        l = l * expf(m - mn) + expf(lg - mn);
        m = mn;
      }
    }
  }
  // combine the 16 key lanes of each query (lanes 16*(qi%4)..+15 of one wave)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
    float mn = fmaxf(m, m2);
    l = (m == -INFINITY ? 0.f : l * expf(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * expf(m2 - mn));
    m = mn;
  }
  if (kj == 0) lse_s[qi] = m + logf(l);
  __syncthreads();
  const float lse = lse_s[qi];

  // ---- pass 2: probabilities and gradients ----
  float dq_acc[8];   // thread owns 8 of the kQ*E dq outputs (E <= 128)
#pragma unroll
  for (int r = 0; r < 8; ++r) dq_acc[r] = 0.f;
  float ds_acc = 0.f, diag = 0.f;
  for (int k0 = 0; k0 < N; k0 += kKT) {
    __syncthreads();
    for (int e = t; e < kKT * E; e += 256) {
      int j = e / E, d = e % E;
      K[j][d] = (k0 + j) < N ? ksrc[(size_t)(k0 + j) * E + d] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kKT / 16; ++r) {
      int j = kj + 16 * r;
      float w = 0.f;
      if (qvalid && k0 + j < N) {
        float dot = 0.f;
        for (int d = 0; d < E; ++d) dot += Q[qi][d] * K[j][d];
        float lg = s * dot;
        float p = expf(lg - lse);
        bool is_diag = (k0 + j) == qglob;
        if (is_diag) diag = lg;
        w = (p - (is_diag ? 1.f : 0.f)) * inv2n;
        ds_acc += w * dot;
      }
      Wt[qi][j] = w;
    }
    __syncthreads();
    // dq[i][d] += s * sum_j W[i][j] K[j][d]   (thread: 8 (i,d) outputs)
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      int o = t + 256 * r;
      int i = o / E, d = o % E;
      if (i < kQ && d < E) {
        float a = 0.f;
        for (int j = 0; j < kKT; ++j) a += Wt[i][j] * K[j][d];
        dq_acc[r] += s * a;
      }
    }
    // dk[j][d] = s * sum_i W[i][j] Q[i][d]
    for (int o = t; o < kKT * E; o += 256) {
      int j = o / E, d = o % E;
      if (k0 + j < N) {
        float a = 0.f;
#pragma unroll
        for (int i = 0; i < kQ; ++i) a += Wt[i][j] * Q[i][d];
        if (a != 0.f) atomicAdd(gk + (size_t)(k0 + j) * E + d, s * a);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    int o = t + 256 * r;
    int i = o / E, d = o % E;
    if (i < kQ && d < E && (q0 + i) < B) atomicAdd(gq + (size_t)(offset + q0 + i) * E + d, dq_acc[r]);
  }
  // loss term of this query: lse - diagonal logit
  float lterm = (qvalid && kj == 0) ? 0.f : 0.f;
  // diag is held by exactly one key lane per query; gather via wave sum
  red[t] = diag;
  __syncthreads();
  if (kj == 0 && qvalid) {
    float dg = 0.f;
    for (int u = 0; u < 16; ++u) dg += red[qi * 16 + u];
    lterm = lse - dg;
  }
  float tot = warp_sum(lterm);
  float dss = warp_sum(ds_acc);
  if ((t & 63) == 0) {
    atomicAdd(loss_parts + role, tot);
    atomicAdd(d_logit_scale, (ex <= 100.f ? dss * s : 0.f));
  }
  if (lse_out && kj == 0 && qvalid) lse_out[role * B + q0 + qi] = lse;
}

// row-wise L2 normalisation (F.normalize, p=2, dim=1, eps=1e-12)
__global__ void l2norm_fwd_kernel(int R, int E, const float* __restrict__ x, float* __restrict__ y,
                                  float* __restrict__ norm) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  int l = threadIdx.x & 63;
  if (r >= R) return;
  float s = 0.f;
  for (int d = l; d < E; d += 64) { float v = x[(size_t)r * E + d]; s += v * v; }
  float n = sqrtf(warp_sum(s));
  float dn = fmaxf(n, 1e-12f);
  for (int d = l; d < E; d += 64) y[(size_t)r * E + d] = x[(size_t)r * E + d] / dn;
  if (l == 0) norm[r] = n;
}
// dx = (dy - y * <y, dy>) / n   (n > eps),   dy / eps otherwise; optional T copy
template <typename T>
__global__ void l2norm_bwd_kernel(int R, int E, const float* __restrict__ y, const float* __restrict__ norm,
                                  const float* __restrict__ dy, const float* __restrict__ gscale,
                                  float* __restrict__ dx, T* __restrict__ dxT) {
  int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  int l = threadIdx.x & 63;
  if (r >= R) return;
  const float gs = gscale ? gscale[0] : 1.f;
  float n = norm[r];
  float dot = 0.f;
  for (int d = l; d < E; d += 64) dot += y[(size_t)r * E + d] * dy[(size_t)r * E + d];
  dot = warp_sum(dot);
  for (int d = l; d < E; d += 64) {
    float g = dy[(size_t)r * E + d];
    float v = gs * (n > 1e-12f ? (g - y[(size_t)r * E + d] * dot) / n : g / 1e-12f);
    if (dx) dx[(size_t)r * E + d] = v;
    if (dxT) dxT[(size_t)r * E + d] = from_f<T>(v);
  }
}

// symmetric CE over an explicit [B][B] logits matrix (API path: _compute_loss)
// out[0] = loss, out[1] = image loss, out[2] = text loss; dlogits = d loss / d logits
__global__ void ce_sym_kernel(int B, const float* __restrict__ logits, float* __restrict__ out,
                              float* __restrict__ dlogits) {
  // role 0: rows, role 1: columns; one wave per row/column
  int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  int l = threadIdx.x & 63;
  if (w >= 2 * B) return;
  int role = w / B, i = w % B;
  float m = -INFINITY;
  for (int j = l; j < B; j += 64) m = fmaxf(m, role ? logits[(size_t)j * B + i] : logits[(size_t)i * B + j]);
  m = warp_max(m);
  float s = 0.f;
  for (int j = l; j < B; j += 64) s += expf((role ? logits[(size_t)j * B + i] : logits[(size_t)i * B + j]) - m);
  s = warp_sum(s);
  float lse = m + logf(s);
  float diag = logits[(size_t)i * B + i];
  if (l == 0) {
    atomicAdd(out + 1 + role, (lse - diag) / B);
    atomicAdd(out, 0.5f * (lse - diag) / B);
  }
  if (dlogits) {
    for (int j = l; j < B; j += 64) {
      size_t o = role ? (size_t)j * B + i : (size_t)i * B + j;
      float p = expf(logits[o] - lse);
      atomicAdd(dlogits + o, 0.5f * (p - (i == j ? 1.f : 0.f)) / B);
    }
  }
}

// y[i] = x[i] * s[0] (+ y[i] if accumulate)
__global__ void scale_kernel(int n, const float* __restrict__ x, const float* __restrict__ s,
                             float* __restrict__ y, int accumulate) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = (accumulate ? y[i] : 0.f) + x[i] * (s ? s[0] : 1.f);
}

// loss outputs from the fused kernel's parts: out = {(p0+p1)/(2N), p0/N, p1/N}
__global__ void clip_loss_finish_kernel(const float* parts, float inv_n, float* out) {
  if (threadIdx.x == 0) {
    out[0] = 0.5f * (parts[0] + parts[1]) * inv_n;
    out[1] = parts[0] * inv_n;
    out[2] = parts[1] * inv_n;
  }
}

template <typename T>
__global__ void cast_kernel(size_t n, const float* __restrict__ x, T* __restrict__ y) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = from_f<T>(x[i]);
}

}  // namespace vlp

using namespace vlp;

VLP_EXPORT int vlp_clip_loss_fused(int B, int N, int E, int offset, const float* img_all,
                                   const float* txt_all, const float* logit_scale, float* g_img_all,
                                   float* g_txt_all, float* d_logit_scale, float* loss_parts,
                                   float* lse_out, void* stream) {
  if (E > 128) return (int)hipErrorInvalidValue;
  int nqb = (B + kQ - 1) / kQ;
  hipLaunchKernelGGL(clip_loss_fused_kernel, dim3(2 * nqb), dim3(256), 0, (hipStream_t)stream, B, N, E,
                     offset, img_all, txt_all, logit_scale, g_img_all, g_txt_all, d_logit_scale,
                     loss_parts, lse_out);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_l2norm_fwd(int R, int E, const float* x, float* y, float* norm, void* stream) {
  hipLaunchKernelGGL(l2norm_fwd_kernel, dim3((R + 3) / 4), dim3(256), 0, (hipStream_t)stream, R, E, x,
                     y, norm);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_l2norm_bwd(int dtype, int R, int E, const float* y, const float* norm,
                              const float* dy, const float* gscale, float* dx, void* dxT,
                              void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(l2norm_bwd_kernel<bf16>, dim3((R + 3) / 4), dim3(256), 0, st, R, E, y, norm, dy,
                       gscale, dx, (bf16*)dxT);
  else
    hipLaunchKernelGGL(l2norm_bwd_kernel<float>, dim3((R + 3) / 4), dim3(256), 0, st, R, E, y, norm,
                       dy, gscale, dx, (float*)dxT);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_scale(int n, const float* x, const float* s, float* y, int accumulate,
                         void* stream) {
  hipLaunchKernelGGL(scale_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, n, x, s, y,
                     accumulate);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_clip_loss_finish(const float* parts, int N, float* out, void* stream) {
  hipLaunchKernelGGL(clip_loss_finish_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, parts,
                     1.f / (float)N, out);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_ce_sym(int B, const float* logits, float* out, float* dlogits, void* stream) {
  hipLaunchKernelGGL(ce_sym_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, logits,
                     out, dlogits);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_cast(int dtype, long long n, const float* x, void* y, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(cast_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (size_t)n, x, (bf16*)y);
  else
    hipLaunchKernelGGL(cast_kernel<float>, dim3(blocks), dim3(256), 0, st, (size_t)n, x, (float*)y);
  return (int)hipGetLastError();
}

// Generic matmul on the MFMA engine: C[M][N] (=|+=) alpha * sum_k A(m,k) B(n,k)
//   a_kc: A stored [M][lda] K-contiguous (else A(m,k) = A[k*lda + m])
//   b_kc: B stored [N][ldb] K-contiguous (else B(n,k) = B[k*ldb + n])
//   out_dtype: VLP_F32 or == dtype; accumulate: fp32 atomics (out must be fp32)
VLP_EXPORT int vlp_matmul(int dtype, int M, int N, int K, const void* A, int lda, int a_kc,
                          const void* Bm, int ldb, int b_kc, void* C, int ldc, int out_f32,
                          float alpha, int accumulate, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  auto run = [&](auto tag) -> int {
    using T = decltype(tag);
    auto go = [&](const auto& la, const auto& lb) -> int {
      if (accumulate) {
        EpiAtomic ep{nullptr, nullptr, (float*)C, ldc, alpha};
        return launch_gemm<T, 64, 64, 2>(M, N, K, 1, la, lb, ep, st);
      }
      if (out_f32) {
        EpiStore<float> ep{nullptr, nullptr, (float*)C, ldc, nullptr, alpha};
        return launch_gemm<T, 64, 64, 2>(M, N, K, 1, la, lb, ep, st);
      }
      EpiStore<T> ep{nullptr, nullptr, (T*)C, ldc, nullptr, alpha};
      return launch_gemm<T, 64, 64, 2>(M, N, K, 1, la, lb, ep, st);
    };
    if (a_kc) {
      KMat<T> la{(const T*)A, lda, M, K};
      if (b_kc) return go(la, KMat<T>{(const T*)Bm, ldb, N, K});
      return go(la, MNMat<T>{(const T*)Bm, ldb, N, K});
    }
    MNMat<T> la{(const T*)A, lda, M, K};
    if (b_kc) return go(la, KMat<T>{(const T*)Bm, ldb, N, K});
    return go(la, MNMat<T>{(const T*)Bm, ldb, N, K});
  };
  if (dtype == VLP_BF16) return run(bf16{});
  return run(0.0f);
}
