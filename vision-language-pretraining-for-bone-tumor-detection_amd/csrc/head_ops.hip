// CLIP contrastive head (reference src/models/pretrain/VisionLanguageModule.py
// forward :441-461 and _compute_loss :532-554):
//   img = normalize(f_img @ P_img), txt = normalize(f_txt @ P_txt)   (eps 1e-12)
//   s = min(exp(logit_scale), 100);  logits = s * img @ txt^T
//   loss = (CE(logits, arange) + CE(logits^T, arange)) / 2
//
// `vlp_clip_loss_fused` computes the loss AND its gradients for the global
// batch of a data-parallel job: each rank owns B rows (images) and B columns
// (texts) of the N x N logits matrix (N = B * world, its rows start at
// `offset`).  Role 0 covers the local image rows against all N texts (row
// log-sum-exp, image->text CE), role 1 the local text columns against all N
// images.  The key dimension is split over workgroups so that a global batch
// of N = 2048 keeps the whole chip busy (2 roles x B/16 query blocks x N/64
// key chunks), in three launches:
//   1. clip_lse_part : per (query block, key chunk) the max and sum of exp of
//                      the 16 x 64 logits tile  -> [2][B][nkc] partials
//   2. clip_grad_part: the partials merged to each query's log-sum-exp, then
//                      p = exp(l - lse), dl = (p - [i == j]) / (2N) and
//                      dq_i = s * sum_j dl_ij k_j  -> slab [2][nkc][B][E]
//                      dk_j = s * sum_i dl_ij q_i  -> slab [2][nqb][N][E]
//                      ds   = sum dl_ij cos_ij     -> [2][nqb][nkc]
//   3. clip_fold     : the slabs summed in a fixed order into the gathered
//                      gradients g_img_all / g_txt_all (written, not added),
//                      loss parts and d logit_scale.
// No atomics: the result is bitwise reproducible run to run.  The owner's
// rows of the gathered gradients are then reduce-scattered by the host (RCCL).
#include "gemm.h"

namespace vlp {

constexpr int kQ = 16;        // queries per workgroup
constexpr int kKC = 64;       // keys per workgroup
constexpr int kMaxE = 128;

struct ClipWs {               // float offsets into the workspace
  size_t pm, pl, dq, dk, lterm, lse, ds, total;
};
__host__ __device__ inline ClipWs clip_ws_layout(int B, int N, int E) {
  const size_t nqb = (B + kQ - 1) / kQ, nkc = (N + kKC - 1) / kKC;
  ClipWs w;
  w.pm = 0;
  w.pl = w.pm + 2 * (size_t)B * nkc;
  w.dq = w.pl + 2 * (size_t)B * nkc;
  w.dk = w.dq + 2 * nkc * (size_t)B * E;
  w.lterm = w.dk + 2 * nqb * (size_t)N * E;
  w.lse = w.lterm + 2 * (size_t)B;
  w.ds = w.lse + 2 * (size_t)B;
  w.total = w.ds + 2 * nqb * nkc;
  return w;
}

// Q[16][E] (this role's local queries) and K[64][E] (a key chunk) into LDS
__device__ __forceinline__ void clip_stage(int B, int N, int E, int offset, int q0, int k0, const float* qsrc,
                                           const float* ksrc, float (*Q)[kMaxE + 1], float (*K)[kMaxE + 1]) {
  const int t = threadIdx.x;
  for (int e = t; e < kQ * E; e += 256) {
    const int i = e / E, d = e - i * E;
    Q[i][d] = (q0 + i) < B ? qsrc[(size_t)(offset + q0 + i) * E + d] : 0.f;
  }
  for (int e = t; e < kKC * E; e += 256) {
    const int j = e / E, d = e - j * E;
    K[j][d] = (k0 + j) < N ? ksrc[(size_t)(k0 + j) * E + d] : 0.f;
  }
}

// thread (qi = t >> 4, kj = t & 15) computes the dot products of query qi with keys kj + 16r
__device__ __forceinline__ void clip_dots(int E, int qi, int kj, const float (*Q)[kMaxE + 1],
                                          const float (*K)[kMaxE + 1], float (&dot)[4]) {
#pragma unroll
  for (int r = 0; r < 4; ++r) dot[r] = 0.f;
  for (int d = 0; d < E; ++d) {
    const float qv = Q[qi][d];
#pragma unroll
    for (int r = 0; r < 4; ++r) dot[r] = fmaf(qv, K[kj + 16 * r][d], dot[r]);
  }
}

__global__ void __launch_bounds__(256)
clip_lse_part_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
                     const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
                     float* __restrict__ ws) {
  __shared__ float Q[kQ][kMaxE + 1];
  __shared__ float K[kKC][kMaxE + 1];
  const int nqb = (B + kQ - 1) / kQ, nkc = (N + kKC - 1) / kKC;
  const int role = blockIdx.x / (nqb * nkc);
  const int rem = blockIdx.x - role * nqb * nkc;
  const int qb = rem / nkc, kc = rem - qb * nkc;
  const int q0 = qb * kQ, k0 = kc * kKC;
  clip_stage(B, N, E, offset, q0, k0, role == 0 ? img_all : txt_all, role == 0 ? txt_all : img_all, Q, K);
  __syncthreads();
  const float s = fminf(expf(logit_scale[0]), 100.f);
  const int t = threadIdx.x, qi = t >> 4, kj = t & 15;
  float dot[4];
  clip_dots(E, qi, kj, Q, K, dot);
  float m = -INFINITY;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (k0 + kj + 16 * r < N) m = fmaxf(m, s * dot[r]);
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  float l = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r)
    if (k0 + kj + 16 * r < N) l += expf(s * dot[r] - m);
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) l += __shfl_xor(l, o, 64);
  if (kj == 0 && q0 + qi < B) {
    const ClipWs L = clip_ws_layout(B, N, E);
    const size_t o = ((size_t)role * B + q0 + qi) * nkc + kc;
    ws[L.pm + o] = m;
    ws[L.pl + o] = l;
  }
}

__global__ void __launch_bounds__(256)
clip_grad_part_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
                      const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
                      float* __restrict__ ws) {
  __shared__ float Q[kQ][kMaxE + 1];
  __shared__ float K[kKC][kMaxE + 1];
  __shared__ float Wt[kQ][kKC + 1];
  __shared__ float red[4];
  const int nqb = (B + kQ - 1) / kQ, nkc = (N + kKC - 1) / kKC;
  const int role = blockIdx.x / (nqb * nkc);
  const int rem = blockIdx.x - role * nqb * nkc;
  const int qb = rem / nkc, kc = rem - qb * nkc;
  const int q0 = qb * kQ, k0 = kc * kKC;
  const ClipWs L = clip_ws_layout(B, N, E);
  clip_stage(B, N, E, offset, q0, k0, role == 0 ? img_all : txt_all, role == 0 ? txt_all : img_all, Q, K);
  const float s = fminf(expf(logit_scale[0]), 100.f);
  const float inv2n = 0.5f / (float)N;
  const int t = threadIdx.x, qi = t >> 4, kj = t & 15;
  const bool qvalid = q0 + qi < B;
  // this query's log-sum-exp from the key-chunk partials (16 lanes share the merge)
  float m = -INFINITY, l = 0.f;
  if (qvalid) {
    const size_t base = ((size_t)role * B + q0 + qi) * nkc;
    for (int c = kj; c < nkc; c += 16) {
      const float m2 = ws[L.pm + base + c], l2 = ws[L.pl + base + c];
      const float mn = fmaxf(m, m2);
      l = (m == -INFINITY ? 0.f : l * expf(m - mn)) + l2 * expf(m2 - mn);
      m = mn;
    }
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(l, o, 64);
    const float mn = fmaxf(m, m2);
    l = (m == -INFINITY ? 0.f : l * expf(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * expf(m2 - mn));
    m = mn;
  }
  const float lse = m + logf(l);
  if (kc == 0 && kj == 0 && qvalid) ws[L.lse + (size_t)role * B + q0 + qi] = lse;
  __syncthreads();
  float dot[4];
  clip_dots(E, qi, kj, Q, K, dot);
  const int qglob = offset + q0 + qi;
  float ds = 0.f;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int j = kj + 16 * r;
    float w = 0.f;
    if (qvalid && k0 + j < N) {
      const float lg = s * dot[r];
      const bool diag = k0 + j == qglob;
      w = (expf(lg - lse) - (diag ? 1.f : 0.f)) * inv2n;
      ds = fmaf(w, dot[r], ds);
      if (diag) ws[L.lterm + (size_t)role * B + q0 + qi] = lse - lg;
    }
    Wt[qi][j] = w;
  }
  ds = warp_sum(ds);
  if ((t & 63) == 0) red[t >> 6] = ds;
  __syncthreads();
  if (t == 0) ws[L.ds + ((size_t)role * nqb + qb) * nkc + kc] = (red[0] + red[1]) + (red[2] + red[3]);
  // dq[i][d] = s * sum_j W[i][j] K[j][d]  (this chunk's part; 8 outputs per thread for E = 128)
  for (int o = t; o < kQ * E; o += 256) {
    const int i = o / E, d = o - i * E;
    if (q0 + i >= B) continue;
    float a = 0.f;
#pragma unroll 8
    for (int j = 0; j < kKC; ++j) a = fmaf(Wt[i][j], K[j][d], a);
    ws[L.dq + (((size_t)role * nkc + kc) * B + q0 + i) * E + d] = s * a;
  }
  // dk[j][d] = s * sum_i W[i][j] Q[i][d]  (this query block's part)
  for (int o = t; o < kKC * E; o += 256) {
    const int j = o / E, d = o - j * E;
    if (k0 + j >= N) continue;
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < kQ; ++i) a = fmaf(Wt[i][j], Q[i][d], a);
    ws[L.dk + (((size_t)role * nqb + qb) * N + k0 + j) * E + d] = s * a;
  }
}

// g_img_all[r] = sum_qb dk[role 1][qb][r] + (own row ? sum_kc dq[role 0][kc][r - offset] : 0);
// g_txt_all likewise with the roles swapped.  Block 0 also writes the loss parts
// (sum of lse - diag over the local queries), d logit_scale and lse_out.
__global__ void __launch_bounds__(256)
clip_fold_kernel(int B, int N, int E, int offset, const float* __restrict__ logit_scale,
                 const float* __restrict__ ws, float* __restrict__ g_img_all, float* __restrict__ g_txt_all,
                 float* __restrict__ d_logit_scale, float* __restrict__ loss_parts, float* __restrict__ lse_out) {
  const int nqb = (B + kQ - 1) / kQ, nkc = (N + kKC - 1) / kKC;
  const ClipWs L = clip_ws_layout(B, N, E);
  const size_t per = (size_t)N * E;
  for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < 2 * per; o += (size_t)gridDim.x * blockDim.x) {
    const int tensor = (int)(o / per);        // 0: g_img_all, 1: g_txt_all
    const size_t e = o - tensor * per;
    const int r = (int)(e / E), d = (int)(e - (size_t)r * E);
    const int krole = 1 - tensor, qrole = tensor;
    float a = 0.f;
    for (int qb = 0; qb < nqb; ++qb) a += ws[L.dk + (((size_t)krole * nqb + qb) * N + r) * E + d];
    if (r >= offset && r < offset + B)
      for (int kc = 0; kc < nkc; ++kc) a += ws[L.dq + (((size_t)qrole * nkc + kc) * B + (r - offset)) * E + d];
    (tensor == 0 ? g_img_all : g_txt_all)[e] = a;
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) {
    const int role = threadIdx.x;
    float lt = 0.f;
    for (int q = 0; q < B; ++q) lt += ws[L.lterm + (size_t)role * B + q];
    loss_parts[role] = lt;
    if (role == 0) {
      float ds = 0.f;
      for (size_t i = 0; i < 2 * (size_t)nqb * nkc; ++i) ds += ws[L.ds + i];
      const float ex = expf(logit_scale[0]);
      d_logit_scale[0] = ex <= 100.f ? ds * fminf(ex, 100.f) : 0.f;
    }
  }
  if (lse_out && blockIdx.x == 0)
    for (int q = threadIdx.x; q < 2 * B; q += blockDim.x) lse_out[q] = ws[L.lse + q];
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

VLP_EXPORT int vlp_clip_loss_ws_floats(int B, int N, int E, long long* n) {
  if (B < 1 || N < B || E < 1 || E > kMaxE) return (int)hipErrorInvalidValue;
  *n = (long long)clip_ws_layout(B, N, E).total;
  return 0;
}

VLP_EXPORT int vlp_clip_loss_fused(int B, int N, int E, int offset, const float* img_all,
                                   const float* txt_all, const float* logit_scale, float* g_img_all,
                                   float* g_txt_all, float* d_logit_scale, float* loss_parts,
                                   float* lse_out, float* ws, long long ws_floats, void* stream) {
  if (B < 1 || N < B || E < 1 || E > kMaxE || offset < 0 || offset + B > N) return (int)hipErrorInvalidValue;
  if ((long long)clip_ws_layout(B, N, E).total > ws_floats) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int nqb = (B + kQ - 1) / kQ, nkc = (N + kKC - 1) / kKC;
  const dim3 grid(2 * nqb * nkc);
  hipLaunchKernelGGL(clip_lse_part_kernel, grid, dim3(256), 0, st, B, N, E, offset, img_all, txt_all, logit_scale,
                     ws);
  hipLaunchKernelGGL(clip_grad_part_kernel, grid, dim3(256), 0, st, B, N, E, offset, img_all, txt_all,
                     logit_scale, ws);
  int fb = (int)((2 * (size_t)N * E + 255) / 256);
  if (fb > 2048) fb = 2048;
  hipLaunchKernelGGL(clip_fold_kernel, dim3(fb), dim3(256), 0, st, B, N, E, offset, logit_scale, ws, g_img_all,
                     g_txt_all, d_logit_scale, loss_parts, lse_out);
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
