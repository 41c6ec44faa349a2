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
// images.  Every product runs on v_mfma_f32_16x16x4f32 (exact fp32 products,
// fixed accumulation order), in three launches:
//   1. clip_scores : per (role, 16-query block, 256-key chunk) the 16 x 256
//                    dot products (one 16 x 64 tile per wave) -> the cosines
//                    cos[2][Bp][Np] and the per-64-key partial max / sum of
//                    exp(s * cos)                      -> pm, pl [2][Bp][Np/64]
//   2. clip_dq     : the partials merged to each query's log-sum-exp; the
//                    cosines (read, not recomputed) become
//                    W = (exp(s cos - lse) - [i == j]) / (2N), written over
//                    cos; dq_i = sum_j W_ij k_j over the chunk -> slab
//                    [2][N/256][Bp][E]; sum W * cos -> [2][nqb][N/256]
//   3. clip_dk     : per (role, 64-key block, column group) dk_j = sum_i W_ij
//                    q_i over all local queries, plus (own rows) the dq slab
//                    fold of the other role -> g_img_all / g_txt_all (written,
//                    not added) = s * (dk + dq); block 0 also reduces the loss
//                    parts and d logit_scale.
// No atomics: the result is bitwise reproducible run to run.  The owner's
// rows of the gathered gradients are then reduce-scattered by the host (RCCL).
// MFMA operand convention (as in gemm.h): mfma(a, b, acc) with lane l = 16g + x
// supplying a[x][k(g)] and b[y = x][k(g)] leaves acc[r] = sum_k a[4g + r][k] b[l & 15][k].
#include "gemm.h"

namespace vlp {

constexpr int kQ = 16;        // queries per query block
constexpr int kKT = 64;       // keys per wave tile (partials granularity)
constexpr int kKC = 256;      // keys per workgroup in launches 1 and 2
constexpr int kKB = 64;       // keys per workgroup in launch 3
constexpr int kETW = 2;       // 16-column tiles per workgroup in launch 3
constexpr int kMaxE = 256;

struct ClipWs {               // float offsets into the workspace
  size_t cw, pm, pl, dq, lterm, lse, ds, total;
  int Bp, Np, nqb, nkt, nkc;
};
__host__ __device__ inline ClipWs clip_ws_layout(int B, int N, int E) {
  ClipWs w;
  w.Bp = (B + kQ - 1) / kQ * kQ;
  w.Np = (N + kKT - 1) / kKT * kKT;
  w.nqb = w.Bp / kQ;
  w.nkt = w.Np / kKT;
  w.nkc = (N + kKC - 1) / kKC;
  w.cw = 0;
  w.pm = w.cw + 2 * (size_t)w.Bp * w.Np;
  w.pl = w.pm + 2 * (size_t)w.Bp * w.nkt;
  w.dq = w.pl + 2 * (size_t)w.Bp * w.nkt;
  w.lterm = w.dq + 2 * (size_t)w.nkc * w.Bp * E;
  w.lse = w.lterm + 2 * (size_t)w.Bp;
  w.ds = w.lse + 2 * (size_t)w.Bp;
  w.total = w.ds + 2 * (size_t)w.nqb * w.nkc;
  return w;
}

__device__ __forceinline__ v4f mfma4(float a, float b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// float4 of row `row` at column `col` (E % 4 == 0); zeros outside [0, rows) x [0, E)
__device__ __forceinline__ v4f ld_row4(const float* base, int row, int rows, int col, int E) {
  if (row < rows && col < E) return *reinterpret_cast<const v4f*>(base + (size_t)row * E + col);
  return v4f{0.f, 0.f, 0.f, 0.f};
}

// Launch 1.  Wave w: keys k0 = kc * 256 + 64 w, 4 sub-tiles of 16 keys.  Lane
// l = 16g + i holds the cosines of query i with keys k0 + 16t + 4g + r (t, r in
// 0..3) -- written as float4 rows of cw.
template <int NCH>
__global__ void __launch_bounds__(256)
clip_scores_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
                   const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
                   float* __restrict__ ws) {
  const ClipWs L = clip_ws_layout(B, N, E);
  const int per_role = L.nqb * L.nkc;
  const int role = blockIdx.x / per_role;
  const int rem = blockIdx.x - role * per_role;
  const int qb = rem / L.nkc, kc = rem - qb * L.nkc;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = l & 15, g = l >> 4;
  const int q0 = qb * kQ, k0 = kc * kKC + w * kKT;
  if (k0 >= L.Np) return;
  const float* qsrc = (role == 0 ? img_all : txt_all) + (size_t)offset * E;
  const float* ksrc = role == 0 ? txt_all : img_all;
  const float s = fminf(expf(logit_scale[0]), 100.f);
  v4f qv[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) qv[c] = ld_row4(qsrc, q0 + x, B, 16 * c + 4 * g, E);
  v4f acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    v4f kv[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) kv[c] = ld_row4(ksrc, k0 + 16 * t + x, N, 16 * c + 4 * g, E);
    acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[t] = mfma4(kv[c][r], qv[c][r], acc[t]);
  }
  // acc[t][r] = cos(query q0 + x, key k0 + 16t + 4g + r)
  float* cw = ws + L.cw + ((size_t)role * L.Bp + q0 + x) * L.Np + k0;
#pragma unroll
  for (int t = 0; t < 4; ++t) *reinterpret_cast<v4f*>(cw + 16 * t + 4 * g) = acc[t];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (k0 + 16 * t + 4 * g + r < N) m = fmaxf(m, s * acc[t][r]);
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (k0 + 16 * t + 4 * g + r < N) sum += expf(s * acc[t][r] - m);
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  if (g == 0 && q0 + x < B) {
    const size_t o = ((size_t)role * L.Bp + q0 + x) * L.nkt + k0 / kKT;
    ws[L.pm + o] = m;
    ws[L.pl + o] = sum;
  }
}

// Launch 2.  Same grid as launch 1; wave w owns keys k0 = kc * 256 + 64 w in two
// halves of 32 staged in LDS ([32][E + 4] per wave).  Lane l = 16g + i: query i.
template <int NCH>
__global__ void __launch_bounds__(256)
clip_dq_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
               const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
               const float* __restrict__ role_w, float* __restrict__ ws) {
  constexpr int EP = NCH * 16 + 4;                       // LDS row stride (floats)
  __shared__ __attribute__((aligned(16))) float lds[4 * 32 * EP];
  __shared__ float red_ds[4];
  const ClipWs L = clip_ws_layout(B, N, E);
  const int per_role = L.nqb * L.nkc;
  const int role = blockIdx.x / per_role;
  const int rem = blockIdx.x - role * per_role;
  const int qb = rem / L.nkc, kc = rem - qb * L.nkc;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = l & 15, g = l >> 4;
  const int q0 = qb * kQ, k0 = kc * kKC + w * kKT;
  const bool active = k0 < L.Np;
  const bool qvalid = q0 + x < B;
  const float* ksrc = role == 0 ? txt_all : img_all;
  const float s = fminf(expf(logit_scale[0]), 100.f);
  // W = d loss / d logit with loss = sum_r role_w[r] * CE_r / 2 (role_w = {1, 1}: the
  // reference's (image_loss + text_loss) / 2); W carries the weight into dq, dk and d s
  const float inv2n = (role_w ? role_w[role] : 1.f) * 0.5f / (float)N;
  // this query's log-sum-exp from the 64-key partials (lane groups g stride them)
  float m = -INFINITY, sl = 0.f;
  if (qvalid) {
    const size_t base = ((size_t)role * L.Bp + q0 + x) * L.nkt;
    for (int c = g; c < L.nkt; c += 4) {
      const float m2 = ws[L.pm + base + c], l2 = ws[L.pl + base + c];
      if (m2 == -INFINITY) continue;
      const float mn = fmaxf(m, m2);
      sl = (m == -INFINITY ? 0.f : sl * expf(m - mn)) + l2 * expf(m2 - mn);
      m = mn;
    }
  }
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    const float m2 = __shfl_xor(m, o, 64), l2 = __shfl_xor(sl, o, 64);
    const float mn = fmaxf(m, m2);
    sl = (m == -INFINITY ? 0.f : sl * expf(m - mn)) + (m2 == -INFINITY ? 0.f : l2 * expf(m2 - mn));
    m = mn;
  }
  const float lse = qvalid ? m + logf(sl) : 0.f;
  if (kc == 0 && w == 0 && g == 0 && qvalid) ws[L.lse + (size_t)role * L.Bp + q0 + x] = lse;
  const int qglob = offset + q0 + x;
  float* kl = lds + w * 32 * EP;
  float* cwrow = ws + L.cw + ((size_t)role * L.Bp + q0 + x) * L.Np;
  v4f acc[NCH];
#pragma unroll
  for (int t = 0; t < NCH; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  float ds = 0.f;
#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    const int j0 = k0 + 32 * h;
    if (active) {
      // stage keys j0 .. j0 + 31 (zero rows past N): 32 x NCH*16 floats, float4 per lane
      for (int e = l; e < 32 * NCH * 4; e += 64) {
        const int row = e / (NCH * 4), c4 = e - row * (NCH * 4);
        *reinterpret_cast<v4f*>(kl + row * EP + 4 * c4) = ld_row4(ksrc, j0 + row, N, 4 * c4, E);
      }
    }
    __syncthreads();
    if (active) {
      v4f wv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int jb = j0 + 16 * u + 4 * g;
        const v4f cv = *reinterpret_cast<const v4f*>(cwrow + jb);
        v4f wr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float wt = 0.f;
          if (qvalid && jb + r < N) {
            const float lg = s * cv[r];
            const bool diag = jb + r == qglob;
            wt = (expf(lg - lse) - (diag ? 1.f : 0.f)) * inv2n;
            ds = fmaf(wt, cv[r], ds);
            if (diag) ws[L.lterm + (size_t)role * L.Bp + q0 + x] = lse - lg;
          }
          wr[r] = wt;
        }
        wv[u] = wr;
        *reinterpret_cast<v4f*>(cwrow + jb) = wr;          // W replaces the cosines (launch 3 reads it)
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float* krow = kl + (16 * u + 4 * g + r) * EP + x;
#pragma unroll
          for (int t = 0; t < NCH; ++t) acc[t] = mfma4(wv[u][r], krow[16 * t], acc[t]);
        }
    }
    __syncthreads();
  }
  // acc[t][r] = sum over this wave's keys of W[q0 + 4g + r][j] k_j[16t + x]; fold the 4 waves
  float* red = lds;                                   // [4][16][NCH*16]
  constexpr int EW = NCH * 16;
#pragma unroll
  for (int t = 0; t < NCH; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(w * 16 + 4 * g + r) * EW + 16 * t + x] = acc[t][r];
  ds = warp_sum(ds);
  if (l == 0) red_ds[w] = ds;
  __syncthreads();
  float* dq = ws + L.dq + (((size_t)role * L.nkc + kc) * L.Bp + q0) * E;
  for (int o = threadIdx.x; o < 16 * E; o += 256) {
    const int i = o / E, e = o - i * E;
    dq[(size_t)i * E + e] = (red[i * EW + e] + red[(16 + i) * EW + e]) + (red[(32 + i) * EW + e] + red[(48 + i) * EW + e]);
  }
  if (threadIdx.x == 0)
    ws[L.ds + ((size_t)role * L.nqb + qb) * L.nkc + kc] = (red_ds[0] + red_ds[1]) + (red_ds[2] + red_ds[3]);
}

// Launch 3.  Workgroup (role, 64-key block kb, column group eg of kETW 16-wide
// tiles); wave w owns keys kb * 64 + 16 w.  W [64 queries][64 keys] and the
// queries' columns are staged per 64-query chunk.  Lane l = 16g + x holds
// dk[key 16w + 4g + r][column 16t + x].
__global__ void __launch_bounds__(256)
clip_dk_kernel(int B, int N, int E, int offset, const float* __restrict__ img_all,
               const float* __restrict__ txt_all, const float* __restrict__ logit_scale,
               const float* __restrict__ ws, float* __restrict__ g_img_all, float* __restrict__ g_txt_all,
               float* __restrict__ d_logit_scale, float* __restrict__ loss_parts, float* __restrict__ lse_out) {
  constexpr int WP = kKB + 4, QP = 16 * kETW + 4;
  __shared__ __attribute__((aligned(16))) float Ws[64 * WP];
  __shared__ __attribute__((aligned(16))) float Qs[64 * QP];
  const ClipWs L = clip_ws_layout(B, N, E);
  const int ncg = (E + 16 * kETW - 1) / (16 * kETW);
  const int nkb = L.Np / kKB;
  const int per_role = nkb * ncg;
  const int role = blockIdx.x / per_role;
  const int rem = blockIdx.x - role * per_role;
  const int kb = rem / ncg, eg = rem - kb * ncg;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int x = l & 15, g = l >> 4;
  const int j0 = kb * kKB, c0 = eg * 16 * kETW;
  const float* qsrc = (role == 0 ? img_all : txt_all) + (size_t)offset * E;
  const float* cw = ws + L.cw + (size_t)role * L.Bp * L.Np;
  v4f acc[kETW];
#pragma unroll
  for (int t = 0; t < kETW; ++t) acc[t] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int i0 = 0; i0 < L.Bp; i0 += 64) {
    for (int e = threadIdx.x; e < 64 * 16; e += 256) {     // W rows i0.., 16 float4 per row
      const int row = e >> 4, c4 = e & 15;
      v4f v = v4f{0.f, 0.f, 0.f, 0.f};
      if (i0 + row < L.Bp) v = *reinterpret_cast<const v4f*>(cw + (size_t)(i0 + row) * L.Np + j0 + 4 * c4);
      *reinterpret_cast<v4f*>(Ws + row * WP + 4 * c4) = v;
    }
    for (int e = threadIdx.x; e < 64 * 4 * kETW; e += 256) {
      const int row = e / (4 * kETW), c4 = e - row * (4 * kETW);
      *reinterpret_cast<v4f*>(Qs + row * QP + 4 * c4) = ld_row4(qsrc, i0 + row, B, c0 + 4 * c4, E);
    }
    __syncthreads();
    // 64 queries = 4 blocks of 16; MFMA (kk, r) takes queries 16kk + 4g + r of lane group g
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * kk + 4 * g + r;
        const float a = Ws[i * WP + 16 * w + x];
#pragma unroll
        for (int t = 0; t < kETW; ++t) acc[t] = mfma4(a, Qs[i * QP + 16 * t + x], acc[t]);
      }
    __syncthreads();
  }
  const float s = fminf(expf(logit_scale[0]), 100.f);
  float* gout = role == 0 ? g_txt_all : g_img_all;       // keys of role 0 are texts
  const int orole = 1 - role;                            // its queries are this tensor's own rows
  const float* dq = ws + L.dq + (size_t)orole * L.nkc * L.Bp * E;
#pragma unroll
  for (int t = 0; t < kETW; ++t) {
    const int col = c0 + 16 * t + x;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = j0 + 16 * w + 4 * g + r;
      if (j >= N || col >= E) continue;
      float a = acc[t][r];
      if (j >= offset && j < offset + B) {
        float f = 0.f;
        for (int c = 0; c < L.nkc; ++c) f += dq[((size_t)c * L.Bp + (j - offset)) * E + col];
        a += f;
      }
      gout[(size_t)j * E + col] = s * a;
    }
  }
  if (blockIdx.x == 0 && w == 0) {
    // loss parts, d logit_scale and lse_out: fixed-order lane-strided sums + xor tree
    float lt0 = 0.f, lt1 = 0.f, dsum = 0.f;
    for (int q = l; q < B; q += 64) {
      lt0 += ws[L.lterm + q];
      lt1 += ws[L.lterm + L.Bp + q];
    }
    const int nds = L.nqb * L.nkc;
    for (int i = l; i < 2 * nds; i += 64) dsum += ws[L.ds + i];
    lt0 = warp_sum(lt0);
    lt1 = warp_sum(lt1);
    dsum = warp_sum(dsum);
    if (l == 0) {
      loss_parts[0] = lt0;
      loss_parts[1] = lt1;
      const float ex = expf(logit_scale[0]);
      d_logit_scale[0] = ex <= 100.f ? dsum * fminf(ex, 100.f) : 0.f;
    }
    if (lse_out)
      for (int q = l; q < B; q += 64) {
        lse_out[q] = ws[L.lse + q];
        lse_out[B + q] = ws[L.lse + L.Bp + q];
      }
  }
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
                              float* __restrict__ dlogits, const float* __restrict__ role_w) {
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
  if (dlogits) {   // d (sum_r role_w[r] * CE_r / 2) / d logits
    const float wr = (role_w ? role_w[role] : 1.f) * 0.5f / B;
    for (int j = l; j < B; j += 64) {
      size_t o = role ? (size_t)j * B + i : (size_t)i * B + j;
      float p = expf(logits[o] - lse);
      atomicAdd(dlogits + o, wr * (p - (i == j ? 1.f : 0.f)));
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
  if (B < 1 || N < B || E < 4 || E > kMaxE || E % 4) return (int)hipErrorInvalidValue;
  *n = (long long)clip_ws_layout(B, N, E).total;
  return 0;
}

VLP_EXPORT int vlp_clip_loss_fused(int B, int N, int E, int offset, const float* img_all,
                                   const float* txt_all, const float* logit_scale, float* g_img_all,
                                   float* g_txt_all, float* d_logit_scale, float* loss_parts,
                                   float* lse_out, const float* role_w, float* ws, long long ws_floats,
                                   void* stream) {
  if (B < 1 || N < B || E < 4 || E > kMaxE || E % 4 || offset < 0 || offset + B > N)
    return (int)hipErrorInvalidValue;
  const ClipWs L = clip_ws_layout(B, N, E);
  if ((long long)L.total > ws_floats) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g12(2 * L.nqb * L.nkc);
  if (E <= 128) {
    hipLaunchKernelGGL(clip_scores_kernel<8>, g12, dim3(256), 0, st, B, N, E, offset, img_all, txt_all, logit_scale, ws);
    hipLaunchKernelGGL(clip_dq_kernel<8>, g12, dim3(256), 0, st, B, N, E, offset, img_all, txt_all, logit_scale,
                       role_w, ws);
  } else {
    hipLaunchKernelGGL(clip_scores_kernel<16>, g12, dim3(256), 0, st, B, N, E, offset, img_all, txt_all, logit_scale, ws);
    hipLaunchKernelGGL(clip_dq_kernel<16>, g12, dim3(256), 0, st, B, N, E, offset, img_all, txt_all, logit_scale,
                       role_w, ws);
  }
  const int ncg = (E + 16 * kETW - 1) / (16 * kETW);
  hipLaunchKernelGGL(clip_dk_kernel, dim3(2 * (L.Np / kKB) * ncg), dim3(256), 0, st, B, N, E, offset, img_all,
                     txt_all, logit_scale, (const float*)ws, g_img_all, g_txt_all, d_logit_scale, loss_parts, lse_out);
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

VLP_EXPORT int vlp_ce_sym(int B, const float* logits, float* out, float* dlogits, const float* role_w,
                          void* stream) {
  hipLaunchKernelGGL(ce_sym_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, (hipStream_t)stream, B, logits,
                     out, dlogits, role_w);
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
  // the loaders move 16-B chunks along the contiguous dimension and the epilogues
  // store 4-column groups: every contiguous extent and leading dimension must be a
  // whole number of chunks (a ragged tail would read the next row's elements)
  const int epc = dtype == VLP_BF16 ? 8 : 4;
  if (M < 0 || N < 0 || K < 0 || (a_kc ? K : M) % epc || lda % epc || (b_kc ? K : N) % epc || ldb % epc ||
      N % 4 || ldc % 4)
    return (int)hipErrorInvalidValue;
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
