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
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += vc[e] + vr[e];
            s2[e] = fmaf(vc[e], vc[e], fmaf(vr[e], vr[e], s2[e]));
          }
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
// The stem's whole backward in one pass: per pair of conv-output rows,
//   1. the patch tile P [2 rows][Wo px][64 k] (bf16, from xs) is staged in LDS,
//   2. y0 = W1 * P is recomputed on MFMA into the row tile Y [2][Wo][64],
//   3. the pooled gradient is routed and dy = k*g + b*y0 + c written over Y,
//   4. dW1[co][k] += sum_px dy[px][co] * P[px][k] on MFMA, both operands read
//      transposed from LDS (ds_read_b64_tr_b16: lane i of a 16-lane group gets
//      column i of 4 consecutive rows),
// so neither y0 nor dy ever reaches HBM.  Each workgroup accumulates its
// band's 64 x 64 weight gradient in registers (each wave a 32 x 32 quadrant
// over every other k-step), sums the pairs in LDS and writes one fp32 slab [64][64];
// vlp_stem1_wgrad_fold sums the slabs and replicates them over the 3 input
// channels.  512 threads; LDS: W1 8 KB + P 2*Wo*128 + Y 2*Wo*128 + 1.25 KB.
constexpr int kStemFusedPairs = 16;   // row pairs per workgroup

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

template <int NA>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2)))
stem1_bwd_fused_kernel(Stem1Geom g, const bf16* __restrict__ xs, const bf16* __restrict__ wp1, int Hq, int Wq,
                       const bf16* __restrict__ dp, const uint8_t* __restrict__ idx,
                       const float* __restrict__ mean, const float* __restrict__ istd,
                       const float* __restrict__ gamma, const double* __restrict__ sg,
                       const double* __restrict__ sgx, float* __restrict__ slabs) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Ho = g.Ho, Wo = g.Wo;
  const int tile_bytes = 2 * Wo * 128;                // two conv-output rows
  char* wl = smem;
  char* ptile = smem + 8192;
  char* ytile = ptile + tile_bytes;
  float* cl = reinterpret_cast<float*>(smem + 8192 + (2 * tile_bytes > 131072 ? 2 * tile_bytes : 131072));
  const int HP = Ho / 2;
  const int bands = (HP + kStemFusedPairs - 1) / kStemFusedPairs;
  const int n = blockIdx.x / bands, band = blockIdx.x - n * bands;
  const int a0 = band * kStemFusedPairs;
  int a1 = a0 + kStemFusedPairs;
  if (a1 > HP) a1 = HP;
  const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6;
  const int c = tid & 7;                               // routing: this thread's 8-channel chunk
  const bf16* xn = xs + (size_t)n * g.Hp * g.Wp1;
  const bf16* dp_n = dp + (size_t)n * Hq * Wq * 64;
  const uint8_t* idx_n = idx + (size_t)n * Hq * Wq * 64;
  const char* xb = reinterpret_cast<const char*>(xn);

  // patch tile staging: item = (row r, pixel px, chunk kh) -> 16 B of xs
  constexpr int NP = 2 * NA;                           // 2 rows * Wo * 8 chunks / 512 threads
  uint4 pf[NP];
  auto p_load = [&](int pa) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int item = tid + 512 * it;
      const int r = item / (Wo * 8), rem = item - r * Wo * 8;
      const int px = rem >> 3, kh = rem & 7;
      const int sh = px & 3, ho = 2 * pa + r;
      const unsigned e = (unsigned)sh * (unsigned)g.copy + (unsigned)(2 * ho + kh) * (unsigned)g.Wp1 +
                         (unsigned)(2 * px - 2 * sh);
      pf[it] = ldg16(xb + 2u * e);
    }
  };
  auto p_store = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < NP; ++it) {
      const int item = tid + 512 * it;
      const int r = item / (Wo * 8), rem = item - r * Wo * 8;
      *reinterpret_cast<uint4*>(ptile + r * (Wo * 128) + stile_off(rem >> 3, rem & 7)) = pf[it];
    }
  };
  p_load(a0);
  stage_w(wp1, nullptr, wl);
  if (tid < 64) {
    const int co = tid;
    const float inv_count = 1.f / (float)((double)g.N * Ho * Wo);
    const float is = istd[co];
    const float k = gamma[co] * is;
    const float mg = (float)(sg[co] * (double)inv_count), mgx = (float)(sgx[co] * (double)inv_count);
    cl[co] = k;
    cl[64 + co] = -k * is * mgx;
    cl[128 + co] = -k * mg + k * is * mgx * mean[co];
  }
  // dW1[co][k] split over the waves: wave wv owns the 32 x 32 quadrant (co half
  // (wv >> 1) & 1, k half wv & 1) and every other 32-px k-step (parity wv >> 2)
  const int qco = 32 * ((wv >> 1) & 1), qk = 32 * (wv & 1);
  v4f dw[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) dw[a][b] = v4f{0.f, 0.f, 0.f, 0.f};
  // y0 recompute split: wave -> row (wv >> 2), columns 16*NA*(wv & 3) ..
  const int yr = wv >> 2, yseg = 16 * NA * (wv & 3);
  for (int pa = a0; pa < a1; ++pa) {
    p_store();
    if (pa + 1 < a1) p_load(pa + 1);                   // the next pair's patches fly across this pair
    lds_barrier();
    // ---- 2: y0 on MFMA (A = W1 from LDS, B = patch fragments from the P tile), one
    //         16-px fragment at a time (16 accumulator registers live) ----
    {
      const char* prow = ptile + yr * (Wo * 128);
      char* yrow = ytile + yr * (Wo * 128);
#pragma unroll 1
      for (int a = 0; a < NA; ++a) {
        const int px = yseg + 16 * a + (l & 15);
        const v8bf p0 = *reinterpret_cast<const v8bf*>(prow + stile_off(px, l >> 4));
        const v8bf p1 = *reinterpret_cast<const v8bf*>(prow + stile_off(px, 4 + (l >> 4)));
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int co = 16 * b + (l & 15);
          const v8bf w0 = *reinterpret_cast<const v8bf*>(wl + stile_off(co, l >> 4));
          const v8bf w1 = *reinterpret_cast<const v8bf*>(wl + stile_off(co, 4 + (l >> 4)));
          v4f t = v4f{0.f, 0.f, 0.f, 0.f};
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w0, p0, t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1, p1, t, 0, 0, 0);
          const int co0 = 16 * b + 4 * (l >> 4);
          v4bf v;
          v[0] = (bf16)t[0]; v[1] = (bf16)t[1]; v[2] = (bf16)t[2]; v[3] = (bf16)t[3];
          *reinterpret_cast<v4bf*>(yrow + stile_off(px, co0 >> 3) + ((co0 >> 2) & 1) * 8) = v;
        }
      }
    }
    lds_barrier();
    // ---- 3: route the pooled gradient; dy = k*g + b*y0 + c over the Y tile ----
    const bool v10 = pa + 1 < Hq;
#pragma unroll 1
    for (int item = tid; item < 4 * Wo; item += 512) {
      const int q = item >> 3;                         // column pair 2q, 2q + 1 (chunk c = item & 7)
      const bool v01 = q + 1 < Wq;
      const int pa1 = v10 ? pa + 1 : pa, q1 = v01 ? q + 1 : q;
      uint4 pv[4];
      uint2 ib[4];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const int ho = (k4 >> 1) ? pa1 : pa, wo = (k4 & 1) ? q1 : q;
        const unsigned po = ((unsigned)ho * Wq + wo) * 64 + 8 * c;
        pv[k4] = ldg16(dp_n + po);
        ib[k4] = *reinterpret_cast<const uint2*>(idx_n + po);
      }
      float ka[8], ba[8], ca[8];
      ld8f_lds(cl + 8 * c, ka);
      ld8f_lds(cl + 64 + 8 * c, ba);
      ld8f_lds(cl + 128 + 8 * c, ca);
      float f[4][8];
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) unpack8(pv[k4], f[k4]);
      const bool v11 = v01 && v10;
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {   // pixel (2pa + (k4 >> 1), 2q + (k4 & 1))
        float yv[8], d[8];
        const int px = 2 * q + (k4 & 1);
        char* at = ytile + (k4 >> 1) * (Wo * 128) + stile_off(px, c);
        unpack8(*reinterpret_cast<const uint4*>(at), yv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          unsigned t[4];
#pragma unroll
          for (int m = 0; m < 4; ++m) t[m] = (((e >> 2) ? ib[m].y : ib[m].x) >> (8 * (e & 3))) & 255u;
          float gsum;
          if (k4 == 0) gsum = t[0] == 4u ? f[0][e] : 0.f;
          else if (k4 == 1) gsum = (t[0] == 5u ? f[0][e] : 0.f) + ((v01 && t[1] == 3u) ? f[1][e] : 0.f);
          else if (k4 == 2) gsum = (t[0] == 7u ? f[0][e] : 0.f) + ((v10 && t[2] == 1u) ? f[2][e] : 0.f);
          else
            gsum = (t[0] == 8u ? f[0][e] : 0.f) + ((v01 && t[1] == 6u) ? f[1][e] : 0.f) +
                   ((v10 && t[2] == 2u) ? f[2][e] : 0.f) + ((v11 && t[3] == 0u) ? f[3][e] : 0.f);
          d[e] = fmaf(ka[e], gsum, fmaf(ba[e], yv[e], ca[e]));
        }
        *reinterpret_cast<uint4*>(at) = Chunk<bf16>::pack(d);
      }
    }
    lds_barrier();
    // ---- 4: dW1 += dy^T P over this pair's 2*Wo pixels (k-steps of 32 px split over the waves) ----
    for (int ks = wv >> 2; ks < Wo / 16; ks += 2) {
      const int r = (32 * ks) / Wo, px0 = 32 * ks - r * Wo;
      const char* yb = ytile + r * (Wo * 128);
      const char* pb = ptile + r * (Wo * 128);
      v8bf fa[2], fb[2];
#pragma unroll
      for (int a = 0; a < 2; ++a) fa[a] = tile_tr(yb, px0, qco + 16 * a);
#pragma unroll
      for (int b = 0; b < 2; ++b) fb[b] = tile_tr(pb, px0, qk + 16 * b);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the asm reads' results (hipcc does not track them)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) dw[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], dw[a][b], 0, 0, 0);
    }
    lds_barrier();                                     // P and Y are rewritten by the next pair
  }
  // ---- the two k-parity waves of each quadrant summed through LDS: one fp32 slab per workgroup ----
  float* red = reinterpret_cast<float*>(ptile);        // [2 parities][64 co][64 k]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = qco + 16 * a + 4 * (l >> 4) + r, k = qk + 16 * b + (l & 15);
        red[((wv >> 2) * 64 + co) * 64 + k] = dw[a][b][r];
      }
  __syncthreads();
  float* slab = slabs + (size_t)blockIdx.x * 4096;
  for (int e = tid; e < 4096; e += 512) slab[e] = red[e] + red[4096 + e];
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

static int stem1_bwd_fused_wgs(int N, int H, int W) {
  const Stem1Geom g = make_stem1(N, H, W);
  return N * ((g.Ho / 2 + kStemFusedPairs - 1) / kStemFusedPairs);
}
// Number of fp32 [64][64] slabs vlp_stem1_bwd_fused writes (one per workgroup).
VLP_EXPORT int vlp_stem1_bwd_fused_slabs(int N, int H, int W, int* nslabs) {
  *nslabs = stem1_bwd_fused_wgs(N, H, W);
  return 0;
}

// The whole stem backward (route + BN backward + weight gradient), y0 and dy
// never materialised: slabs [vlp_stem1_bwd_fused_slabs][64][64] -> vlp_stem1_wgrad_fold.
VLP_EXPORT int vlp_stem1_bwd_fused(const void* xs, const void* wp1, const void* dp, const uint8_t* idx,
                                   const float* mean, const float* istd, const float* gamma, const double* sum_g,
                                   const double* sum_gx, float* slabs, long long slab_floats, int N, int H, int W,
                                   void* stream) {
  if (!vlp_stem1_fused_ok(H, W) || N < 1) return (int)hipErrorInvalidValue;
  const Stem1Geom g = make_stem1(N, H, W);
  if (!stem1_offsets_fit(g)) return (int)hipErrorInvalidValue;
  const int nwg = stem1_bwd_fused_wgs(N, H, W);
  if ((long long)nwg * 4096 > slab_floats) return (int)hipErrorInvalidValue;
  const int Hq = (g.Ho + 2 - 3) / 2 + 1, Wq = (g.Wo + 2 - 3) / 2 + 1;
  // the P and Y tiles (4 * Wo * 128 B), at least the 8 x 16 KB of the final cross-wave sum
  const size_t tiles = 4 * (size_t)g.Wo * 128 > 131072 ? 4 * (size_t)g.Wo * 128 : 131072;
  const size_t lds = 8192 + tiles + 3 * 64 * sizeof(float);
  hipStream_t st = (hipStream_t)stream;
  VLP_STEM_NA_SWITCH(g.Wo / 64, {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)&stem1_bwd_fused_kernel<NAC>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 8192 + 4 * 256 * 128 + 3 * 64 * 4);
      attr = true;
    }
    hipLaunchKernelGGL(stem1_bwd_fused_kernel<NAC>, dim3(nwg), dim3(512), lds, st, g, (const bf16*)xs,
                       (const bf16*)wp1, Hq, Wq, (const bf16*)dp, idx, mean, istd, gamma, sum_g, sum_gx, slabs);
  });
  return (int)hipGetLastError();
}
