// Fused ResNet34 stem for the single-channel upload (bf16): conv 7x7/2 +
// BatchNorm statistics + max-pool 3x3/2 in ONE pass that never writes the
// full-resolution conv output y0, and the matching backward that recomputes
// y0 instead of reading it.  Replaces, on the hot path, the timm stem
// conv1 -> bn1 -> act1 -> maxpool called through
// /root/reference/src/models/pretrain/VisionLanguageModule.py:30-32.
//
// Why pooling the raw conv output is exact: relu(sc*y + sh) is monotone in y,
// non-decreasing for sc >= 0 and non-increasing for sc < 0, and sc = gamma *
// istd has the sign of gamma (istd > 0), known before the batch statistics.
// So the max-pool of relu(bn(y0)) over a window equals relu(bn(.)) of the
// window's max of y0 (gamma >= 0) or of its min (gamma < 0).  The forward
// pools s*y0 with s = sign(gamma) folded into the weights, and stores the
// raw y0 at the arg-max tap (`yarg`) and the tap (`idx`, kh*3 + kw, first
// maximum in row-major tap order, as torch's max_pool2d).  Once the stats are
// final, p = relu(sc*yarg + sh) is one pass over the pooled tensor
// (vlp_bn_add_relu).
//
// Backward: dy0 = k*g + b*y0 + c (the folded BatchNorm backward) where g is
// the pooled gradient routed to each window's arg-max.  The pooled gradient
// must arrive ReLU-masked (p > 0), as the layer-1 data gradient's epilogue
// writes it: the arg-max pixel's relu(bn(y0)) IS p, so the pixel-level ReLU
// mask adds nothing.  y0 is recomputed on the MFMA pipe
// (K = 64, cheap) rather than read back: the 2.1 GB y0 tensor of a bs = 256,
// 512^2 batch never exists.
//
// Work split (both kernels): a workgroup owns a band of rows of ONE image;
// per conv-output row its 4 waves compute Wo / 4 output columns each
// (v_mfma_f32_16x16x32_bf16, weights in registers, patch fragments loaded
// straight from the 4 shifted copies of stem_geom.h), the row goes to LDS as
// bf16 [px][64] with the 16-B chunk XOR-swizzled by px, and the pooling /
// routing runs on (column, 8-channel chunk) items from there.
#include "common.h"
#include "stem_geom.h"

namespace vlp {

constexpr int kStemBand = 8;      // pooled rows per workgroup (forward)
#ifndef VLP_STEM_PK
#define VLP_STEM_PK 1                 // forward BN sums in packed fp32 (two channels per instruction)
#endif
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kStemPairs = 8;     // conv-output row pairs per workgroup (backward)

// byte offset of 16-B chunk `chunk` of pixel px in a [px][64] bf16 tile: rows of 128 B
// fill half a 256-B bank row, so px pairs {4m+2, 4m+3} swap halves (the stride-2
// pixel reads of the pooling / routing items then alternate halves), and the chunk
// is XOR-swizzled by px (16 consecutive px written at one chunk spread over the bank row)
__device__ __forceinline__ int stile_off(int px, int chunk) {
  return (px ^ ((px >> 1) & 1)) * 128 + ((chunk ^ (px & 7)) << 4);
}

__device__ __forceinline__ uint4 neg_bf16x8(uint4 u) {
  u.x ^= 0x80008000u; u.y ^= 0x80008000u; u.z ^= 0x80008000u; u.w ^= 0x80008000u;
  return u;
}

__device__ __forceinline__ unsigned lds_addr_stem(const void* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ v8bf as_v8bf(const uint4& u) { return *reinterpret_cast<const v8bf*>(&u); }

// LDS-only barrier: waits for this wave's LDS traffic, not for its global
// loads / stores (which __syncthreads() would drain: the next row's patch
// prefetch and the pooled-row stores stay in flight across it)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// W1 [64 co][64 k] bf16 -> LDS (16-B chunks swizzled by co), sign(gamma) folded in when given
__device__ __forceinline__ void stage_w(const bf16* __restrict__ wp1, const float* __restrict__ gamma_sign,
                                        char* wl) {
  for (int q = threadIdx.x; q < 64 * 8; q += blockDim.x) {
    const int co = q >> 3, ch = q & 7;
    uint4 u = ldg16(wp1 + co * 64 + ch * 8);
    if (gamma_sign != nullptr && gamma_sign[co] < 0.f) u = neg_bf16x8(u);
    *reinterpret_cast<uint4*>(wl + stile_off(co, ch)) = u;
  }
}

// The conv-output row of one workgroup: wave w computes columns [16*NA*w, 16*NA*(w + 1))
// (NA = Wo / 64 px fragments of 16 per wave), all 64 output channels.
// Patch fragments (MFMA B operand) patch[k = 32s + 8(lane >> 4) ..][px = 16a + (lane & 15)].
template <int NA>
struct StemP {
  v8bf p[NA][2];
  // patches of conv-output row ho.  kh = 7 is the zero-weight pad row of the K = 64
  // layout: its image row 2ho + 7 < Hp exists and is finite, so it is loaded like the
  // others (no lane-divergent branch around the load)
  // xn: this image's base in copy 0 (xs + n * Hp * Wp1); the lane offsets (copy wo & 3,
  // row, column) are 32-bit byte offsets from it (4 copies < 4 GB: checked by the host)
  __device__ void load(const Stem1Geom& g, const bf16* __restrict__ xn, int ho) {
    const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const char* xb = reinterpret_cast<const char*>(xn);
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int wo = 16 * NA * wv + 16 * a + (l & 15);
      const int sh = wo & 3;
      const unsigned e = (unsigned)sh * (unsigned)g.copy + (unsigned)(2 * ho + (l >> 4)) * (unsigned)g.Wp1 +
                         (unsigned)(2 * wo - 2 * sh);
#pragma unroll
      for (int s = 0; s < 2; ++s)
        p[a][s] = as_v8bf(ldg16(xb + 2u * (e + (unsigned)(4 * s) * (unsigned)g.Wp1)));
    }
  }
};
// acc = D[co = 16b + 4(lane >> 4) + r][px = 16*NA*w + 16a + (lane & 15)]; the MFMA A operand
// W1[co = 16b + (lane & 15)][k = 32s + 8(lane >> 4) .. +7] comes from the LDS copy
template <int NA>
__device__ __forceinline__ void stem_mfma(const StemP<NA>& P, const char* wl, v4f (&acc)[NA][4]) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int co = 16 * b + (l & 15);
    const v8bf w0 = *reinterpret_cast<const v8bf*>(wl + stile_off(co, l >> 4));
    const v8bf w1 = *reinterpret_cast<const v8bf*>(wl + stile_off(co, 4 + (l >> 4)));
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      v4f c = v4f{0.f, 0.f, 0.f, 0.f};
      c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, P.p[a][0], c, 0, 0, 0);
      acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, P.p[a][1], c, 0, 0, 0);
    }
  }
}
// the row as bf16 [px][64] into an LDS tile
template <int NA>
__device__ __forceinline__ void stem_store(const v4f (&acc)[NA][4], char* tile) {
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int px = 16 * NA * wv + 16 * a + (l & 15);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int co0 = 16 * b + 4 * (l >> 4);
      v4bf v;
      v[0] = (bf16)acc[a][b][0]; v[1] = (bf16)acc[a][b][1]; v[2] = (bf16)acc[a][b][2]; v[3] = (bf16)acc[a][b][3];
      *reinterpret_cast<v4bf*>(tile + stile_off(px, co0 >> 3) + ((co0 >> 2) & 1) * 8) = v;
    }
  }
}

__device__ __forceinline__ void unpack8(const uint4& u, float* f) { Chunk<bf16>::unpack(u, f); }
__device__ __forceinline__ void ld8f_lds(const float* p, float (&o)[8]) {
  const v4f x = *reinterpret_cast<const v4f*>(p), y = *reinterpret_cast<const v4f*>(p + 4);
#pragma unroll
  for (int j = 0; j < 4; ++j) { o[j] = x[j]; o[4 + j] = y[j]; }
}

// byte e of a 2-dword tap word pair := t (compile-time e and t: one v_bfi)
template <int E>
__device__ __forceinline__ void set_tap(uint32_t (&tp)[2], bool on, uint32_t t) {
  constexpr uint32_t m = 0xffu << (8 * (E & 3));
  const uint32_t nv = (tp[E >> 2] & ~m) | ((t << (8 * (E & 3))) & m);
  tp[E >> 2] = on ? nv : tp[E >> 2];
}

// ---------------------------------------------------------------- forward
// grid: N * ceil(Hq / kStemBand) workgroups of 256 threads; NA = Wo / 64.
// stat_sum / stat_sumsq: [rep][64] fp64 replicas of sum(y0), sum(y0^2) (null: eval mode).
// LDS: W1 (8 KB) + 2 conv-row tiles of Wo * 128 B (bf16 [px][64]).
template <int NA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
stem1_pool_fwd_kernel(Stem1Geom g, const bf16* __restrict__ xs, const bf16* __restrict__ wp1,
                      const float* __restrict__ gamma, int Hq, int Wq, bf16* __restrict__ yarg,
                      uint8_t* __restrict__ idx, double* __restrict__ stat_sum, double* __restrict__ stat_sumsq,
                      int rep) {
  constexpr int NI = NA;                    // pooling items per thread: Wq * 8 / 256
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  char* tiles = smem + 8192;
  const int bands = (Hq + kStemBand - 1) / kStemBand;
  const int n = blockIdx.x / bands, band = blockIdx.x - n * bands;
  const int i0 = band * kStemBand;
  int i1 = i0 + kStemBand;
  if (i1 > Hq) i1 = Hq;
  const int tid = threadIdx.x;
  const int c = tid & 7;                    // this thread's 8-channel chunk in every item
  const bool stats = stat_sum != nullptr;
  const int tile_bytes = g.Wo * 128;
  float sgn[8];                             // sign(gamma) of this thread's channels
#pragma unroll
  for (int e = 0; e < 8; ++e) sgn[e] = gamma[8 * c + e] < 0.f ? -1.f : 1.f;

  StemP<NA> P;
  v4f acc[NA][4];
  bf16* yarg_n = yarg + (size_t)n * Hq * Wq * 64;
  uint8_t* idx_n = idx + (size_t)n * Hq * Wq * 64;
  // conv-output rows 2*i0 - 1 .. 2*i1 - 1: the first is the top row of pooled row i0's
  // window (pooled row i0 - 1's bottom row, owned by the band above for the statistics)
  const int ylo = 2 * i0 - 1, yhi = 2 * i1 - 1;
  const bf16* xn = xs + (size_t)n * g.Hp * g.Wp1;
  P.load(g, xn, ylo >= 0 ? ylo : 0);
  stage_w(wp1, gamma, wl);
  float s1[8], s2[8];   // sum and sum of squares of s*y0 over this thread's pixels, chunk c
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
#if VLP_STEM_PK
  v2f s1p[4], s2p[4];
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) s1p[e2] = s2p[e2] = v2f{0.f, 0.f};
#endif
  // running window maxima of s*y0 per item (column j = item >> 3) and their taps
  float best[NI][8];
  uint32_t tap[NI][2];
  __syncthreads();
  for (int y = ylo; y <= yhi; ++y) {
    const int rr = y - ylo;
    char* tile = tiles + (rr & 1) * tile_bytes;
    const bool have = y >= 0;               // y <= yhi <= Ho - 1
    if (have) {
      stem_mfma(P, wl, acc);
      if (y + 1 <= yhi) P.load(g, xn, y + 1);
      stem_store(acc, tile);
    }
    lds_barrier();
    // pooling: this row is dh = 1 of pooled row y / 2 when y is even; dh = 2 of
    // pooled row (y - 1) / 2 and dh = 0 of pooled row (y + 1) / 2 when y is odd
    const bool odd = (y & 1) != 0;          // y = -1 is odd
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int j = (tid >> 3) + 32 * it;
      float hv[8];
      uint32_t hd[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 8; ++e) hv[e] = -INFINITY;
      if (have) {
        // dw = 0 (column 2j - 1: padding for j = 0), dw = 1 (2j), dw = 2 (2j + 1)
        float vl[8], vc[8], vr[8];
        unpack8(*reinterpret_cast<const uint4*>(tile + stile_off(2 * j, c)), vc);
        unpack8(*reinterpret_cast<const uint4*>(tile + stile_off(2 * j + 1, c)), vr);
        const bool left = j > 0;
        unpack8(*reinterpret_cast<const uint4*>(tile + stile_off(left ? 2 * j - 1 : 0, c)), vl);
        if (stats && rr >= 1) {
#if VLP_STEM_PK
          // packed fp32 (v_pk_add_f32 / v_pk_fma_f32: two channels per instruction)
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const v2f c2 = {vc[2 * e2], vc[2 * e2 + 1]}, r2 = {vr[2 * e2], vr[2 * e2 + 1]};
            s1p[e2] += c2 + r2;
            s2p[e2] = __builtin_elementwise_fma(c2, c2, __builtin_elementwise_fma(r2, r2, s2p[e2]));
          }
#else
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += vc[e] + vr[e];
            s2[e] = fmaf(vc[e], vc[e], fmaf(vr[e], vr[e], s2[e]));
          }
#endif
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float l0 = left ? vl[e] : -INFINITY;
          const bool c1 = vc[e] > l0;
          float m = c1 ? vc[e] : l0;
          const bool c2 = vr[e] > m;
          hv[e] = c2 ? vr[e] : m;
          const uint32_t t = c2 ? 2u : (c1 ? 1u : 0u);
          hd[e >> 2] |= t << (8 * (e & 3));
        }
      }
      if (!odd) {   // dh = 1 (the center row always exists)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool up = hv[e] > best[it][e];
          best[it][e] = up ? hv[e] : best[it][e];
          const uint32_t t = 3u + ((hd[e >> 2] >> (8 * (e & 3))) & 0xffu);
          const uint32_t m = 0xffu << (8 * (e & 3));
          tap[it][e >> 2] = up ? ((tap[it][e >> 2] & ~m) | (t << (8 * (e & 3)))) : tap[it][e >> 2];
        }
      } else {
        if (rr > 0) {   // dh = 2 of pooled row (y - 1) / 2, then emit it
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const bool up = hv[e] > best[it][e];
            best[it][e] = up ? hv[e] : best[it][e];
            const uint32_t t = 6u + ((hd[e >> 2] >> (8 * (e & 3))) & 0xffu);
            const uint32_t m = 0xffu << (8 * (e & 3));
            tap[it][e >> 2] = up ? ((tap[it][e >> 2] & ~m) | (t << (8 * (e & 3)))) : tap[it][e >> 2];
          }
          const int i = (y - 1) >> 1;
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = sgn[e] * best[it][e];
          const unsigned off = ((unsigned)i * Wq + j) * 64 + 8 * c;
          stg16(yarg_n + off, Chunk<bf16>::pack(o));
          *reinterpret_cast<uint2*>(idx_n + off) = make_uint2(tap[it][0], tap[it][1]);
        }
        if (y < yhi) {  // dh = 0 of pooled row (y + 1) / 2 starts the window (row -1 is padding)
#pragma unroll
          for (int e = 0; e < 8; ++e) best[it][e] = hv[e];
          tap[it][0] = hd[0];
          tap[it][1] = hd[1];
        }
      }
    }
  }
  if (!stats) return;
#if VLP_STEM_PK
#pragma unroll
  for (int e2 = 0; e2 < 4; ++e2) {
    s1[2 * e2] = s1p[e2][0]; s1[2 * e2 + 1] = s1p[e2][1];
    s2[2 * e2] = s2p[e2][0]; s2[2 * e2 + 1] = s2p[e2][1];
  }
#endif
  // statistics: each thread summed its columns {2j, 2j + 1} of chunk c over the owned
  // rows; the 32 threads sharing a chunk meet in LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(tiles);   // [256 threads][16]
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[tid * 16 + e] = s1[e];
    red[tid * 16 + 8 + e] = s2[e];
  }
  __syncthreads();
  if (tid < 128) {
    const int co = tid & 63, which = tid >> 6;   // which: 0 = sum, 1 = sum of squares
    const int cc = co >> 3, e = co & 7;
    float a = 0.f;
    for (int t = cc; t < 256; t += 8) a += red[t * 16 + which * 8 + e];
    const size_t ro = (size_t)(blockIdx.x % rep) * 64 + co;
    if (which == 0) atomicAdd(stat_sum + ro, (double)(gamma[co] < 0.f ? -a : a));
    else atomicAdd(stat_sumsq + ro, (double)a);
  }
}

// ---------------------------------------------------------------- backward
// dy0[n][h][w][c] = k*g + b*y0 + c0 with y0 recomputed, g the pooled gradient dp
// routed through idx (2x2 blocks of conv-output pixels share one set of four
// pooled-gradient gathers: rows {2a, 2a+1} x cols {2q, 2q+1} are covered by
// the pooled outputs (a|a+1, q|q+1)).  grid: N * ceil(Ho / (2 kStemPairs)).
// LDS: W1 (8 KB) + 2 conv-row tiles + the per-channel coefficients.
template <int NA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
stem1_route_bwd_kernel(Stem1Geom g, const bf16* __restrict__ xs, const bf16* __restrict__ wp1, int Hq, int Wq,
                       const bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                       const float* __restrict__ sc, const float* __restrict__ sh, const float* __restrict__ mean,
                       const float* __restrict__ istd, const float* __restrict__ gamma,
                       const double* __restrict__ sg, const double* __restrict__ sgx, bf16* __restrict__ dy) {
  constexpr int NI = NA;                    // (column pair, chunk) items per thread: (Wo / 2) * 8 / 256
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  char* tiles = smem + 8192;
  const int Ho = g.Ho, Wo = g.Wo;
  const int HP = Ho / 2;
  const int bands = (HP + kStemPairs - 1) / kStemPairs;
  const int n = blockIdx.x / bands, band = blockIdx.x - n * bands;
  const int a0 = band * kStemPairs;
  int a1 = a0 + kStemPairs;
  if (a1 > HP) a1 = HP;
  const int tid = threadIdx.x;
  const int c = tid & 7;                    // this thread's 8-channel chunk (fixed: 256 % 8 == 0)
  const int tile_bytes = Wo * 128;

  StemP<NA> P0, P1;                         // conv-output rows 2pa / 2pa + 1 (patches prefetched)
  v4f acc[NA][4];
  const bf16* xn = xs + (size_t)n * g.Hp * g.Wp1;
  const bf16* dp_n = dp + (size_t)n * Hq * Wq * 64;
  const uint8_t* idx_n = idx + (size_t)n * Hq * Wq * 64;
  bf16* dy_n = dy + (size_t)n * Ho * Wo * 64;
  P0.load(g, xn, 2 * a0);
  P1.load(g, xn, 2 * a0 + 1);
  stage_w(wp1, nullptr, wl);
  // per-channel coefficients in LDS ([5][64]: BN scale, shift (unused: dp arrives
  // ReLU-masked), and the folded backward k, b, c of dy = k*g + b*y + c)
  float* cl = reinterpret_cast<float*>(tiles + 2 * tile_bytes);
  if (tid < 64) {
    const int co = tid;
    const float inv_count = 1.f / (float)((double)g.N * Ho * Wo);
    const float is = istd[co];
    const float k = gamma[co] * is;
    const float mg = (float)(sg[co] * (double)inv_count), mgx = (float)(sgx[co] * (double)inv_count);
    cl[co] = sc[co];
    cl[64 + co] = sh[co];
    cl[128 + co] = k;
    cl[192 + co] = -k * is * mgx;
    cl[256 + co] = -k * mg + k * is * mgx * mean[co];
  }
  // the four pooled-gradient / tap gathers of one (column pair, chunk) item
  struct Gather { uint4 pv[4]; uint2 ib[4]; };
  auto gather = [&](int pa, int q, Gather& G) __attribute__((always_inline)) {
    const int pa1 = pa + 1 < Hq ? pa + 1 : pa, q1 = q + 1 < Wq ? q + 1 : q;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4) {
      const int ho = (k4 >> 1) ? pa1 : pa, wo = (k4 & 1) ? q1 : q;
      const unsigned po = ((unsigned)ho * Wq + wo) * 64 + 8 * c;
      G.pv[k4] = ldg16(dp_n + po);
      G.ib[k4] = *reinterpret_cast<const uint2*>(idx_n + po);
    }
  };
  __syncthreads();
  for (int pa = a0; pa < a1; ++pa) {
    Gather cur, nxt;
    stem_mfma(P0, wl, acc);
    stem_store(acc, tiles);
    stem_mfma(P1, wl, acc);
    stem_store(acc, tiles + tile_bytes);
    if (pa + 1 < a1) P0.load(g, xn, 2 * pa + 2);   // flies during the routing
    gather(pa, tid >> 3, cur);              // item 0's gathers fly across the barrier
    lds_barrier();
    const bool v10 = pa + 1 < Hq;
#pragma unroll 1
    for (int it = 0; it < NI; ++it) {
      const int q = (tid >> 3) + 32 * it;   // column pair: conv-output columns 2q, 2q + 1
      if (it + 1 < NI) gather(pa, q + 32, nxt);
      const bool v01 = q + 1 < Wq;
      float ka[8], ba[8], ca[8];
      ld8f_lds(cl + 128 + 8 * c, ka);
      ld8f_lds(cl + 192 + 8 * c, ba);
      ld8f_lds(cl + 256 + 8 * c, ca);
      float f[4][8];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) unpack8(cur.pv[k4], f[k4]);
      const bool v11 = v01 && v10;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {   // pixel (2pa + (k4 >> 1), 2q + (k4 & 1))
        float yv[8], d[8];
        const int px = 2 * q + (k4 & 1);
        unpack8(*reinterpret_cast<const uint4*>(tiles + (k4 >> 1) * tile_bytes + stile_off(px, c)), yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          unsigned t[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) t[m] = (((e >> 2) ? cur.ib[m].y : cur.ib[m].x) >> (8 * (e & 3))) & 255u;
          float gsum;
          if (k4 == 0) gsum = t[0] == 4u ? f[0][e] : 0.f;
          else if (k4 == 1) gsum = (t[0] == 5u ? f[0][e] : 0.f) + ((v01 && t[1] == 3u) ? f[1][e] : 0.f);
          else if (k4 == 2) gsum = (t[0] == 7u ? f[0][e] : 0.f) + ((v10 && t[2] == 1u) ? f[2][e] : 0.f);
          else
            gsum = (t[0] == 8u ? f[0][e] : 0.f) + ((v01 && t[1] == 6u) ? f[1][e] : 0.f) +
                   ((v10 && t[2] == 2u) ? f[2][e] : 0.f) + ((v11 && t[3] == 0u) ? f[3][e] : 0.f);
          d[e] = fmaf(ka[e], gsum, fmaf(ba[e], yv[e], ca[e]));
        }
        const unsigned yo = ((unsigned)(2 * pa + (k4 >> 1)) * Wo + px) * 64 + 8 * c;
        stg16(dy_n + yo, Chunk<bf16>::pack(d));
      }
      if (it + 1 < NI) cur = nxt;
    }
    if (pa + 1 < a1) P1.load(g, xn, 2 * pa + 3);   // flies during the barrier and row 2pa + 2
    lds_barrier();   // the tiles are rewritten by the next pair
  }
}


// ---------------------------------------------------------------- fused backward
// The stem's whole backward, y0 and dy never materialised.  With dy = k*g +
// b*y0 + c (the folded BatchNorm backward, per-channel k, b, c) and y0 = W1 P
// (P = the K = 64 patch of a conv-output pixel), the weight gradient is linear
// in three batch sums:
//   dW1[co][k] = k_co R[co][k] + b_co (W1 G)[co][k] + c_co S[k]
//   R = sum_px g(px) P(px)^T   (g: the pooled gradient routed to its arg-max pixel)
//   G = sum_px P(px) P(px)^T   (the 64 x 64 Gram matrix of the patches)
//   S = sum_px P(px)
// so the backward never recomputes y0 and never forms dy per pixel: it routes
// each pooled gradient to its arg-max pixel once into a bf16 tile of routed
// gradients, and runs R, G and S on MFMA over the patch tile (the y0 term is
// exact here -- W1 G in fp64 in the fold -- where the per-pixel form rounds y0
// and dy to bf16).
//
// Work split: a workgroup owns one image, a band of kGramBand pooled rows and a
// column block of CW conv-output columns.  Iteration a (pooled row a = conv rows
// 2a, 2a + 1, which only the windows of pooled rows a and a + 1 reach):
//   A. the patch tile P [2 rows][CW px][64 k] of conv rows 2a, 2a + 1 is stored
//      (prefetched one iteration ahead in registers), and the routed-gradient
//      tile Gt [2 rows][CW px][64] is GATHERED: one thread per (column pair
//      {2q, 2q + 1}, 8-channel chunk) reads the four windows (a|a+1, q|q+1) and
//      sums, per pixel and channel, the windows whose arg-max tap is that pixel
//      (pixel (2a, 2q): window (a, q) tap 4; (2a, 2q+1): (a, q) tap 5 + (a, q+1)
//      tap 3; (2a+1, 2q): (a, q) 7 + (a+1, q) 1; (2a+1, 2q+1): (a, q) 8 +
//      (a, q+1) 6 + (a+1, q) 2 + (a+1, q+1) 0), in fp32, in that fixed order,
//      rounded once to bf16: no LDS atomics, bit-identical runs.  Pooled row
//      a + 1's windows are kept in registers for the next iteration, so every
//      window is read from HBM once per column block;
//   B. R += Gt^T P, G += P^T P, S += 1^T P on MFMA (operands read transposed from
//      LDS, ds_read_b64_tr_b16).
// Each workgroup writes one fp32 slab [R | G | S]; vlp_stem1_bwd_fused's fold
// sums the slabs in a fixed order (deterministic) and forms dW1.  512 threads;
// LDS 4 * CW * 128 B (P and Gt, two conv rows each).
constexpr int kGramBand = 32;                   // pooled rows per workgroup
constexpr int kGramSlab = 64 * 64 * 2 + 64;     // R, G, S floats per workgroup
constexpr int kGramGroups = 32;                 // first-level slab groups of the fold

// transposed fragment of a [px][64] tile (stile_off layout): lane (i, g) gets
// column col0 + i of rows row0 + 8g .. +7 (the MFMA operand with k = px)
__device__ __forceinline__ v8bf tile_tr(const char* tile, int row0, int col0) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, g = l >> 4;
  const int q = i >> 2, p = i & 3;
  const int col = col0 + 4 * p;
  const int r = row0 + 8 * g + q;
  const char* a0 = tile + stile_off(r, col >> 3) + ((col >> 2) & 1) * 8;
  const char* a1 = tile + stile_off(r + 4, col >> 3) + ((col >> 2) & 1) * 8;
  v4bf lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr_stem(a0)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_addr_stem(a1)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// one pooled window's 8-channel chunk: pooled gradient and arg-max taps
struct GramWin { uint4 pv; uint2 ib; };

#ifndef VLP_GRAM_PF
#define VLP_GRAM_PF 1    // patch prefetch distance of the Gram backward, in row pairs (1 or 2)
#endif
#ifndef VLP_GRAM_WPE
#define VLP_GRAM_WPE 2   // waves per SIMD the Gram kernel is compiled for (4: <= 128 VGPRs, two workgroups per CU)
#endif
template <int CW>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(VLP_GRAM_WPE)))
stem1_bwd_gram_kernel(Stem1Geom g, const bf16* __restrict__ xs, int Hq, int Wq, const bf16* __restrict__ dp,
                      const uint8_t* __restrict__ idx, float* __restrict__ slabs) {
  constexpr int RB = CW * 128;                          // bytes of one conv row in a [px][64] tile
  constexpr int NP = 2 * CW * 8 / 512;                  // patch chunks per thread per iteration
  constexpr int NG = CW / 2 * 8;                        // routing items (column pair, chunk) <= 512
  constexpr int KS = 2 * CW / 32;                       // 32-px k-steps per iteration
  static_assert(NG <= 512 && NP >= 1, "CW in {64, 128}");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* ptile = smem;
  char* gtile = smem + 2 * RB;
  const int CB = g.Wo / CW;
  const int bands = (Hq + kGramBand - 1) / kGramBand;
  int bid = blockIdx.x;
  const int cb = bid % CB;
  bid /= CB;
  const int band = bid % bands, n = bid / bands;
  const int i0 = band * kGramBand;
  const int i1 = i0 + kGramBand < Hq ? i0 + kGramBand : Hq;
  const int c0 = cb * CW;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const char* xb = reinterpret_cast<const char*>(xs + (size_t)n * g.Hp * g.Wp1);
  const bf16* dp_n = dp + (size_t)n * Hq * Wq * 64;
  const uint8_t* idx_n = idx + (size_t)n * Hq * Wq * 64;

  // ---- patch staging: item (row r, pixel px, kh) -> 16 B of xs
  // patch prefetch distance VLP_GRAM_PF pairs (2: two register sets, the loop unrolled by 2)
  uint4 pf0[NP], pf1[NP];
  auto p_load = [&](int a, uint4 (&pf)[NP]) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int item = tid + 512 * it;
      const int r = item / (CW * 8), rem = item - r * (CW * 8);
      const int px = rem >> 3, kh = rem & 7;
      const int rr = 2 * a + r, wo = c0 + px, sh = wo & 3;
      const unsigned e = (unsigned)sh * (unsigned)g.copy + (unsigned)(2 * rr + kh) * (unsigned)g.Wp1 +
                         (unsigned)(2 * wo - 2 * sh);
      pf[it] = ldg16(xb + 2u * e);
    }
  };
  auto p_store = [&](const uint4 (&pf)[NP]) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int item = tid + 512 * it;
      const int r = item / (CW * 8), rem = item - r * (CW * 8);
      *reinterpret_cast<uint4*>(ptile + r * RB + stile_off(rem >> 3, rem & 7)) = pf[it];
    }
  };
  // ---- routing item of this thread: column pair q (local pixels 2q', 2q' + 1), chunk c
  const bool router = tid < NG;
  const int qq = tid >> 3, c = tid & 7;
  const int q = c0 / 2 + qq;
  auto ldwin = [&](int i, int qw, GramWin& w) __attribute__((always_inline)) {
    if (router && i < Hq && qw < Wq) {
      const unsigned po = ((unsigned)i * Wq + qw) * 64 + 8 * c;
      w.pv = ldg16(dp_n + po);
      w.ib = *reinterpret_cast<const uint2*>(idx_n + po);
    } else {
      w.pv = make_uint4(0u, 0u, 0u, 0u);
      w.ib = make_uint2(0xffffffffu, 0xffffffffu);    // tap 255: routes nowhere
    }
  };
  auto route = [&](const GramWin& w0, const GramWin& w1, const GramWin& w2, const GramWin& w3)
      __attribute__((always_inline)) {
    float f0[8], f1[8], f2[8], f3[8], o[4][8];
    unpack8(w0.pv, f0); unpack8(w1.pv, f1); unpack8(w2.pv, f2); unpack8(w3.pv, f3);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int sh = 8 * (e & 3);
      const unsigned t0 = (((e >> 2) ? w0.ib.y : w0.ib.x) >> sh) & 255u;
      const unsigned t1 = (((e >> 2) ? w1.ib.y : w1.ib.x) >> sh) & 255u;
      const unsigned t2 = (((e >> 2) ? w2.ib.y : w2.ib.x) >> sh) & 255u;
      const unsigned t3 = (((e >> 2) ? w3.ib.y : w3.ib.x) >> sh) & 255u;
      o[0][e] = t0 == 4u ? f0[e] : 0.f;
      o[1][e] = (t0 == 5u ? f0[e] : 0.f) + (t1 == 3u ? f1[e] : 0.f);
      o[2][e] = (t0 == 7u ? f0[e] : 0.f) + (t2 == 1u ? f2[e] : 0.f);
      o[3][e] = (t0 == 8u ? f0[e] : 0.f) + (t1 == 6u ? f1[e] : 0.f) + (t2 == 2u ? f2[e] : 0.f) +
                (t3 == 0u ? f3[e] : 0.f);
    }
    if (router) {
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4)
        *reinterpret_cast<uint4*>(gtile + (k4 >> 1) * RB + stile_off(2 * qq + (k4 & 1), c)) = Chunk<bf16>::pack(o[k4]);
    }
  };

  // accumulators: wave (quadrant qd = wv & 3: rows 32a.., columns 32b..; k-step parity wv >> 2)
  const int a_ = (wv >> 1) & 1, b = wv & 1, par = wv >> 2;
  v4f accR[2][2], accG[2][2], accS[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    accS[j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) accR[j][jj] = accG[j][jj] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  v8bf ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (bf16)1.f;

  // ---- one pair: A (patch tile + gathered routed gradients), B (R, G, S on MFMA).
  // The fragment reads of k-step ks + 2 are issued before the MFMAs of ks (12
  // ds_read_b64_tr per k-step, waited for with a counted lgkmcnt).
  auto frags = [&](int ks, v8bf (&fg)[2], v8bf (&fp)[2], v8bf (&fb)[2]) __attribute__((always_inline)) {
    const int r = (32 * ks) / CW, px0 = 32 * ks - r * CW;
    const char* gt = gtile + r * RB;
    const char* pt = ptile + r * RB;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fg[j] = tile_tr(gt, px0, 32 * a_ + 16 * j);
      fp[j] = tile_tr(pt, px0, 32 * a_ + 16 * j);
      fb[j] = tile_tr(pt, px0, 32 * b + 16 * j);
    }
  };
  auto mfmas = [&](const v8bf (&fg)[2], const v8bf (&fp)[2], const v8bf (&fb)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        accR[j][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fg[j], fb[jj], accR[j][jj], 0, 0, 0);
        accG[j][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fp[j], fb[jj], accG[j][jj], 0, 0, 0);
      }
    if (a_ == 0) {
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) accS[jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fb[jj], accS[jj], 0, 0, 0);
    }
  };
  static_assert(KS % 4 == 0, "k-steps per wave even");
  GramWin wa0, wa1, wb0, wb1, wn0, wn1;                  // pooled rows a, a + 1 (columns q, q + 1); a + 2 ahead
  auto pair = [&](int a, uint4 (&pf)[NP]) __attribute__((always_inline)) {
    p_store(pf);
    if (a + VLP_GRAM_PF < i1) p_load(a + VLP_GRAM_PF, pf);
    ldwin(a + 2, q, wn0);
    ldwin(a + 2, q + 1, wn1);
    route(wa0, wa1, wb0, wb1);
    lds_barrier();
    v8bf g0[2], p0[2], b0[2], g1[2], p1[2], b1[2];
    frags(par, g0, p0, b0);
#pragma unroll
    for (int ks = par; ks < KS; ks += 4) {
      frags(ks + 2, g1, p1, b1);
      asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");   // k-step ks's 12 reads (LDS returns in order)
      __builtin_amdgcn_sched_barrier(0);
      mfmas(g0, p0, b0);
      if (ks + 4 < KS) {
        frags(ks + 4, g0, p0, b0);
        asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      mfmas(g1, p1, b1);
    }
    lds_barrier();                                       // P and Gt are rewritten by the next pair
    wa0 = wb0; wa1 = wb1; wb0 = wn0; wb1 = wn1;
  };
  // ---- prologue: patches of pairs i0, i0 + 1; windows of pooled rows i0, i0 + 1
  p_load(i0, pf0);
  if (VLP_GRAM_PF == 2 && i0 + 1 < i1) p_load(i0 + 1, pf1);
  ldwin(i0, q, wa0);
  ldwin(i0, q + 1, wa1);
  ldwin(i0 + 1, q, wb0);
  ldwin(i0 + 1, q + 1, wb1);
  if constexpr (VLP_GRAM_PF == 2) {
    for (int a = i0; a < i1; a += 2) {
      pair(a, pf0);
      if (a + 1 < i1) pair(a + 1, pf1);
    }
  } else {
    for (int a = i0; a < i1; ++a) pair(a, pf0);
  }
  // ---- the two k-parity halves summed through LDS: one slab [R | G | S] per workgroup
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (par == pass) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = 32 * a_ + 16 * j + 4 * (l >> 4) + r, k = 32 * b + 16 * jj + (l & 15);
            float* pr = red + m * 64 + k;
            float* pg = red + 4096 + m * 64 + k;
            if (pass == 0) { *pr = accR[j][jj][r]; *pg = accG[j][jj][r]; }
            else { *pr += accR[j][jj][r]; *pg += accG[j][jj][r]; }
          }
      if (a_ == 0 && l < 16) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          float* ps = red + 8192 + 32 * b + 16 * jj + l;
          if (pass == 0) *ps = accS[jj][0];
          else *ps += accS[jj][0];
        }
      }
    }
    __syncthreads();
  }
  float* slab = slabs + (size_t)blockIdx.x * kGramSlab;
  for (int e = tid; e < kGramSlab; e += 512) slab[e] = red[e];
}

// fold, level 1: part[grp][e] = sum of slabs grp, grp + G, ... (fixed order)
__global__ void __launch_bounds__(256) stem1_gram_part_kernel(int ns, const float* __restrict__ slabs,
                                                              float* __restrict__ part) {
  const int e = blockIdx.x * 256 + threadIdx.x, grp = blockIdx.y;
  if (e >= kGramSlab) return;
  float acc0 = 0.f, acc1 = 0.f;
  int s = grp;
  for (; s + kGramGroups < ns; s += 2 * kGramGroups) {
    acc0 += slabs[(size_t)s * kGramSlab + e];
    acc1 += slabs[(size_t)(s + kGramGroups) * kGramSlab + e];
  }
  if (s < ns) acc0 += slabs[(size_t)s * kGramSlab + e];
  part[(size_t)grp * kGramSlab + e] = acc0 + acc1;
}
// fold, level 2: tot[e] = sum over the groups in fp64 (fixed order)
__global__ void __launch_bounds__(256) stem1_gram_tot_kernel(const float* __restrict__ part, double* __restrict__ tot) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= kGramSlab) return;
  double s = 0.0;
  for (int grp = 0; grp < kGramGroups; ++grp) s += (double)part[(size_t)grp * kGramSlab + e];
  tot[e] = s;
}
// fold, level 3: dW1[co][k] = k R + b (W1 G) + c S in fp64, replicated over the 3
// input channels ([64][3][7][7]).  One workgroup per co, one thread per k.
__global__ void __launch_bounds__(64) stem1_gram_grad_kernel(const double* __restrict__ tot, const bf16* __restrict__ wp1,
                                                             const float* __restrict__ mean, const float* __restrict__ istd,
                                                             const float* __restrict__ gamma, const double* __restrict__ sg,
                                                             const double* __restrict__ sgx, double inv_count,
                                                             float* __restrict__ grad) {
  __shared__ double w1[64];
  const int co = blockIdx.x, k = threadIdx.x;
  w1[k] = (double)(float)wp1[co * 64 + k];
  __syncthreads();
  double wg = 0.0;
  for (int k2 = 0; k2 < 64; ++k2) wg += w1[k2] * tot[4096 + k2 * 64 + k];
  const double is = istd[co], kk = (double)gamma[co] * is;
  const double mg = sg[co] * inv_count, mgx = sgx[co] * inv_count;
  const double bco = -kk * is * mgx, cco = -kk * mg + kk * is * mgx * (double)mean[co];
  const double v = kk * tot[co * 64 + k] + bco * wg + cco * tot[8192 + k];
  const int kh = k >> 3, kw = k & 7;
  if (kh < 7 && kw < 7) {
#pragma unroll
    for (int c = 0; c < 3; ++c) grad[((co * 3 + c) * 7 + kh) * 7 + kw] = (float)v;
  }
}

}  // namespace vlp

using namespace vlp;

// Shapes the fused stem takes: Wo a multiple of 64 (<= 256) and Ho even (the
// 2x2 backward blocks); otherwise the caller keeps the unfused stem.
VLP_EXPORT int vlp_stem1_fused_ok(int H, int W) {
  const Stem1Geom g = make_stem1(1, H, W);
  return (g.Wo % 64 == 0 && g.Wo <= 256 && g.Wo >= 64 && g.Ho % 2 == 0 && g.Ho >= 2) ? 1 : 0;
}

#define VLP_STEM_NA_SWITCH(NA_, ...)                       \
  switch (NA_) {                                           \
    case 1: { constexpr int NAC = 1; __VA_ARGS__; break; } \
    case 2: { constexpr int NAC = 2; __VA_ARGS__; break; } \
    case 3: { constexpr int NAC = 3; __VA_ARGS__; break; } \
    case 4: { constexpr int NAC = 4; __VA_ARGS__; break; } \
    default: return (int)hipErrorInvalidValue;             \
  }

// xs: the 4 shifted bf16 copies (vlp_stem1_prep_u8); wp1: [64][64] bf16 (vlp_pack_stem1);
// yarg / idx: [N][Hq][Wq][64] (Hq = Ho / 2, Wq = Wo / 2); stats null in eval mode.
static inline bool stem1_offsets_fit(const Stem1Geom& g) {   // 32-bit lane byte offsets into xs
  return 2.0 * (3.0 * (double)g.copy + (double)g.Hp * g.Wp1) < 4294967296.0;
}

VLP_EXPORT int vlp_stem1_pool_fwd(const void* xs, const void* wp1, const float* gamma, void* yarg, uint8_t* idx,
                                  int N, int H, int W, double* stat_sum, double* stat_sumsq, int stat_rep,
                                  void* stream) {
  if (!vlp_stem1_fused_ok(H, W) || N < 1 || stat_rep < 1) return (int)hipErrorInvalidValue;
  const Stem1Geom g = make_stem1(N, H, W);
  if (!stem1_offsets_fit(g)) return (int)hipErrorInvalidValue;
  const int Hq = (g.Ho + 2 - 3) / 2 + 1, Wq = (g.Wo + 2 - 3) / 2 + 1;
  const int bands = (Hq + kStemBand - 1) / kStemBand;
  const size_t lds = 8192 + 2 * (size_t)g.Wo * 128;
  hipStream_t st = (hipStream_t)stream;
  VLP_STEM_NA_SWITCH(g.Wo / 64,
                     hipLaunchKernelGGL(stem1_pool_fwd_kernel<NAC>, dim3(N * bands), dim3(256), lds, st, g,
                                        (const bf16*)xs, (const bf16*)wp1, gamma, Hq, Wq, (bf16*)yarg, idx,
                                        stat_sum, stat_sumsq, stat_rep));
  return (int)hipGetLastError();
}

// dp: [N][Hq][Wq][64] pooled-output gradient (ReLU-masked); sc / sh / mean / istd: the stem BN's
// batch coefficients; sum_g / sum_gx: its finished backward sums (replica 0 = totals);
// dy: [N][Ho][Wo][64] bf16 gradient of the conv output (for vlp_stem1_wgrad_ws).
VLP_EXPORT int vlp_stem1_route_bwd(const void* xs, const void* wp1, const void* dp, const uint8_t* idx,
                                   const float* sc, const float* sh, const float* mean, const float* istd,
                                   const float* gamma, const double* sum_g, const double* sum_gx, void* dy, int N,
                                   int H, int W, void* stream) {
  if (!vlp_stem1_fused_ok(H, W) || N < 1) return (int)hipErrorInvalidValue;
  const Stem1Geom g = make_stem1(N, H, W);
  if (!stem1_offsets_fit(g)) return (int)hipErrorInvalidValue;
  const int Hq = (g.Ho + 2 - 3) / 2 + 1, Wq = (g.Wo + 2 - 3) / 2 + 1;
  const int bands = (g.Ho / 2 + kStemPairs - 1) / kStemPairs;
  const size_t lds = 8192 + 2 * (size_t)g.Wo * 128 + 5 * 64 * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  VLP_STEM_NA_SWITCH(g.Wo / 64,
                     hipLaunchKernelGGL(stem1_route_bwd_kernel<NAC>, dim3(N * bands), dim3(256), lds, st, g,
                                        (const bf16*)xs, (const bf16*)wp1, Hq, Wq, (const bf16*)dp, idx, sc, sh,
                                        mean, istd, gamma, sum_g, sum_gx, (bf16*)dy));
  return (int)hipGetLastError();
}

#ifndef VLP_GRAM_CW
#define VLP_GRAM_CW 128   // widest column block the Gram backward takes (64 or 128)
#endif
static int stem1_gram_cw(int Wo) { return (VLP_GRAM_CW == 128 && Wo % 128 == 0) ? 128 : 64; }
static int stem1_bwd_fused_wgs(int N, int H, int W) {
  const Stem1Geom g = make_stem1(N, H, W);
  const int Hq = g.Ho / 2;
  return N * ((Hq + kGramBand - 1) / kGramBand) * (g.Wo / stem1_gram_cw(g.Wo));
}
// fp32 workspace of vlp_stem1_bwd_fused: one [R | G | S] slab per workgroup + the fold's partials
VLP_EXPORT int vlp_stem1_bwd_fused_ws_floats(int N, int H, int W, long long* n) {
  if (!n || N < 1) return (int)hipErrorInvalidValue;
  *n = ((long long)stem1_bwd_fused_wgs(N, H, W) + kGramGroups + 2) * kGramSlab;
  return 0;
}

// The whole stem backward (routing + BN backward + weight gradient), y0 and dy never
// materialised: grad [64][3][7][7] (overwritten).  ws >= vlp_stem1_bwd_fused_ws_floats.
VLP_EXPORT int vlp_stem1_bwd_fused(const void* xs, const void* wp1, const void* dp, const uint8_t* idx,
                                   const float* mean, const float* istd, const float* gamma, const double* sum_g,
                                   const double* sum_gx, float* ws, long long ws_floats, float* grad, int N, int H,
                                   int W, void* stream) {
  if (!vlp_stem1_fused_ok(H, W) || N < 1 || !ws || !grad) return (int)hipErrorInvalidValue;
  const Stem1Geom g = make_stem1(N, H, W);
  if (!stem1_offsets_fit(g)) return (int)hipErrorInvalidValue;
  const int nwg = stem1_bwd_fused_wgs(N, H, W);
  if (((long long)nwg + kGramGroups + 2) * kGramSlab > ws_floats) return (int)hipErrorInvalidValue;
  const int Hq = g.Ho / 2, Wq = g.Wo / 2;
  hipStream_t st = (hipStream_t)stream;
  float* part = ws + (size_t)nwg * kGramSlab;
  const int cw = stem1_gram_cw(g.Wo);
  if (cw == 128) {
    constexpr size_t lds = 4 * 128 * 128;
    // per device and cheap: set on every call (a process-wide flag missed a second GPU)
    const hipError_t ae = hipFuncSetAttribute((const void*)&stem1_bwd_gram_kernel<128>,
                                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (ae != hipSuccess) return (int)ae;
    hipLaunchKernelGGL(stem1_bwd_gram_kernel<128>, dim3(nwg), dim3(512), lds, st, g, (const bf16*)xs, Hq, Wq,
                       (const bf16*)dp, idx, ws);
  } else {
    constexpr size_t lds = 4 * 64 * 128 > kGramSlab * 4 ? 4 * 64 * 128 : kGramSlab * 4;   // the slab reduction reuses it
    hipLaunchKernelGGL(stem1_bwd_gram_kernel<64>, dim3(nwg), dim3(512), lds, st, g, (const bf16*)xs, Hq, Wq,
                       (const bf16*)dp, idx, ws);
  }
  hipLaunchKernelGGL(stem1_gram_part_kernel, dim3((kGramSlab + 255) / 256, kGramGroups), dim3(256), 0, st, nwg,
                     (const float*)ws, part);
  double* tot = reinterpret_cast<double*>(part + (size_t)kGramGroups * kGramSlab);   // 8-B aligned: slabs are even
  hipLaunchKernelGGL(stem1_gram_tot_kernel, dim3((kGramSlab + 255) / 256), dim3(256), 0, st, (const float*)part, tot);
  hipLaunchKernelGGL(stem1_gram_grad_kernel, dim3(64), dim3(64), 0, st, (const double*)tot, (const bf16*)wp1, mean,
                     istd, gamma, sum_g, sum_gx, 1.0 / ((double)N * g.Ho * g.Wo), grad);
  return (int)hipGetLastError();
}
