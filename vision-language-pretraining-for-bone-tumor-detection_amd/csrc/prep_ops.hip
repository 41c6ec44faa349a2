// Radiograph preprocessing and augmentation on the device.
//
// The reference runs these per sample in CPU DataLoader workers
// (src/data/PretrainDataModule.py:157-198, two workers in its configs):
//   HistogramNormalized (MONAI histogram_normalize: 256-bin histogram over
//   [min, max], cumsum rescaled to [0, 255], np.interp) -> 3-channel repeat ->
//   CropLargerDimension (<= 5 % of the larger side) -> PadToSquaredEdgeAverage
//   -> Resized(224, mode "area") -> NormalizeIntensityd((x - mean) / std)
// and, for training, RandAffined / RandRotated / RandFlipd / RandZoomd (p 0.3
// each) + RandGaussianNoised (p 0.5).
//
// Here a batch of decoded grayscale images of arbitrary sizes (uint8 or fp32,
// packed back to back) goes through four launches covering every image at
// once: per-image min/max partials, the 256-bin histogram (LDS-privatised),
// the crop/pad edge means, and the area resize that applies the equalisation
// LUT on the fly and writes the normalised [n][C][S][S] batch.  The
// histogram follows numpy's float32 arithmetic (np.histogram with the float32
// range MONAI passes: float32 linspace edges, the bin index and its +-1
// correction against the edges) and the LUT follows MONAI's float32
// rescale_array and numpy's float64 np.interp, separately rounded (the object
// is built with -ffp-contract=off: HIP's default contraction would fuse the
// multiply-adds of the bin edges and the interpolation into FMAs).
//
// The augmentation composes the four geometric transforms of one sample into
// one output->source map (2x3, host-drawn) and resamples once, bilinear with
// border clamping, adding per-channel Gaussian noise from a counter-based
// generator.  MONAI resamples after every transform; one resample is the same
// geometric distribution with less interpolation blur.
#include "common.h"

namespace vlp {

constexpr int kBins = 256;
constexpr int kPrepNB = 64;   // blocks per image for the min/max and histogram passes

template <typename TI> __device__ __forceinline__ float pix(const TI* p, size_t i);
template <> __device__ __forceinline__ float pix<uint8_t>(const uint8_t* p, size_t i) { return (float)p[i]; }
template <> __device__ __forceinline__ float pix<float>(const float* p, size_t i) { return p[i]; }

struct ImgDesc {
  const long long* off;   // element offset of image i in the packed source
  const int* hw;          // [n][2] height, width
};

__device__ __forceinline__ float block_reduce_min(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fminf(fminf(sh[0], sh[1]), fminf(sh[2], sh[3]));
  __syncthreads();
  return v;
}
__device__ __forceinline__ float block_reduce_max(float v, float* sh) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  v = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
  __syncthreads();
  return v;
}

// pass 1: per-block min / max partials  mm[(i * kPrepNB + blk) * 2 + {0,1}]
template <typename TI>
__global__ void __launch_bounds__(256) prep_minmax_kernel(const TI* __restrict__ src, ImgDesc d,
                                                         float* __restrict__ mm) {
  __shared__ float sh[4];
  const int i = blockIdx.y;
  const size_t npx = (size_t)d.hw[2 * i] * d.hw[2 * i + 1];
  const TI* p = src + d.off[i];
  float lo = INFINITY, hi = -INFINITY;
  for (size_t e = blockIdx.x * 256 + threadIdx.x; e < npx; e += (size_t)kPrepNB * 256) {
    const float v = pix(p, e);
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
  lo = block_reduce_min(lo, sh);
  hi = block_reduce_max(hi, sh);
  if (threadIdx.x == 0) {
    mm[((size_t)i * kPrepNB + blockIdx.x) * 2] = lo;
    mm[((size_t)i * kPrepNB + blockIdx.x) * 2 + 1] = hi;
  }
}

// np.histogram's outer edges (range = (img.min(), img.max()), float32; equal
// edges widen by 0.5) and its float32 linspace bin edges
struct HistEdges {
  float first, last, denom;
  __device__ void init(const float* mm, int i) {
    float lo = INFINITY, hi = -INFINITY;
    for (int b = 0; b < kPrepNB; ++b) {
      lo = fminf(lo, mm[((size_t)i * kPrepNB + b) * 2]);
      hi = fmaxf(hi, mm[((size_t)i * kPrepNB + b) * 2 + 1]);
    }
    if (lo == hi) { lo = __fsub_rn(lo, 0.5f); hi = __fadd_rn(hi, 0.5f); }
    first = lo; last = hi;
    denom = __fsub_rn(hi, lo);
  }
  // linspace(first, last, 257, dtype=float32): k * step + first, last exact
  __device__ float edge(int k) const {
    if (k == kBins) return last;
    const float step = __fdiv_rn(__fsub_rn(last, first), (float)kBins);
    return __fadd_rn(__fmul_rn((float)k, step), first);
  }
  // bin of v (first <= v <= last): truncation of (v - first) / denom * 256, then
  // numpy's corrections against the edges
  __device__ int bin(float v, const float* edges) const {
    int k = (int)__fmul_rn(__fdiv_rn(__fsub_rn(v, first), denom), (float)kBins);
    if (k == kBins) k -= 1;
    if (v < edges[k]) k -= 1;
    if (k != kBins - 1 && v >= edges[k + 1]) k += 1;
    return k;
  }
};

// pass 2: histogram  hist[i][256] (u32, zeroed by the launcher)
template <typename TI>
__global__ void __launch_bounds__(256) prep_hist_kernel(const TI* __restrict__ src, ImgDesc d,
                                                       const float* __restrict__ mm, unsigned* __restrict__ hist) {
  __shared__ unsigned h[kBins];
  __shared__ float edges[kBins + 1];
  const int i = blockIdx.y;
  HistEdges he;
  he.init(mm, i);
  for (int k = threadIdx.x; k <= kBins; k += 256) edges[k] = he.edge(k);
  for (int k = threadIdx.x; k < kBins; k += 256) h[k] = 0;
  __syncthreads();
  const size_t npx = (size_t)d.hw[2 * i] * d.hw[2 * i + 1];
  const TI* p = src + d.off[i];
  for (size_t e = blockIdx.x * 256 + threadIdx.x; e < npx; e += (size_t)kPrepNB * 256)
    atomicAdd(&h[he.bin(pix(p, e), edges)], 1u);
  __syncthreads();
  for (int k = threadIdx.x; k < kBins; k += 256)
    if (h[k]) atomicAdd(hist + (size_t)i * kBins + k, h[k]);
}

// The equalisation map of one image, built in LDS by a block: xp = the left
// bin edges (float32 -> double), fp = MONAI rescale_array(cumsum, 0, 255) in
// float32 (-> double), slopes as np.interp precomputes them.
struct Lut {
  double xp[kBins], fp[kBins], sl[kBins];
  float first, step;
  __device__ void build(const unsigned* hist, const float* mm, int i) {
    __shared__ long long cum[kBins];
    HistEdges he;
    he.init(mm, i);
    if (threadIdx.x == 0) {
      long long c = 0;
      for (int k = 0; k < kBins; ++k) { c += hist[(size_t)i * kBins + k]; cum[k] = c; }
    }
    __syncthreads();
    const float cmin = (float)cum[0], cmax = (float)cum[kBins - 1];
    for (int k = threadIdx.x; k < kBins; k += blockDim.x) {
      float f;
      if (cmin == cmax) f = 0.f;   // rescale_array: arr * minv
      else f = __fmul_rn(__fdiv_rn(__fsub_rn((float)cum[k], cmin), __fsub_rn(cmax, cmin)), 255.f);
      fp[k] = (double)f;
      xp[k] = (double)he.edge(k);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kBins - 1; k += blockDim.x)
      sl[k] = __ddiv_rn(__dsub_rn(fp[k + 1], fp[k]), __dsub_rn(xp[k + 1], xp[k]));
    if (threadIdx.x == 0) {
      first = he.first;
      step = __fdiv_rn(__fsub_rn(he.last, he.first), (float)kBins);
    }
    __syncthreads();
  }
  // np.interp(v, xp, fp) in double, cast to float32
  __device__ float apply(float v) const {
    const double x = (double)v;
    if (x < xp[0]) return (float)fp[0];
    if (x >= xp[kBins - 1]) return (float)fp[kBins - 1];
    int j = (int)((v - first) / step);
    j = j < 0 ? 0 : (j > kBins - 2 ? kBins - 2 : j);
    while (j < kBins - 2 && x >= xp[j + 1]) ++j;
    while (j > 0 && x < xp[j]) --j;
    if (xp[j] == x) return (float)fp[j];
    return __double2float_rn(__dadd_rn(__dmul_rn(sl[j], __dsub_rn(x, xp[j])), fp[j]));
  }
};

// crop (CropLargerDimension.py:43-54) and pad (PadToSquaredEdgeAverage.py:43-73)
// geometry: the square side L, the cropped image's rows [r0, r0+h2) x cols
// [c0, c0+w2) of the source, and its placement (pt, pl) inside the square
struct Geom {
  int L, r0, c0, h2, w2, pt, pl;
  __device__ Geom(int h, int w) {
    r0 = c0 = 0; h2 = h; w2 = w;
    if (h > w) {
      int crop = (int)(h * 0.05);
      if (h - crop < w) crop = h - w;
      r0 = crop / 2;
      h2 = h - 2 * r0;
    } else if (w > h) {
      int crop = (int)(w * 0.05);
      if (w - crop < h) crop = w - h;
      c0 = crop / 2;
      w2 = w - 2 * c0;
    }
    L = h2 > w2 ? h2 : w2;
    pt = (L - h2) / 2;
    pl = (L - w2) / 2;
  }
};

// pass 3: the two edge means of the equalised, cropped image (the pad values):
// left/right columns when h2 > w2, top/bottom rows when w2 > h2.  edge[i][2].
template <typename TI>
__global__ void __launch_bounds__(256) prep_edges_kernel(const TI* __restrict__ src, ImgDesc d,
                                                        const float* __restrict__ mm,
                                                        const unsigned* __restrict__ hist, float* __restrict__ edge) {
  __shared__ Lut lut;
  __shared__ float sh[4];
  const int i = blockIdx.x;
  lut.build(hist, mm, i);
  const int h = d.hw[2 * i], w = d.hw[2 * i + 1];
  const Geom g(h, w);
  const TI* p = src + d.off[i];
  float a = 0.f, b = 0.f;
  if (g.h2 > g.w2) {
    for (int r = threadIdx.x; r < g.h2; r += 256) {
      const size_t row = (size_t)(g.r0 + r) * w;
      a += lut.apply(pix(p, row + g.c0));
      b += lut.apply(pix(p, row + g.c0 + g.w2 - 1));
    }
  } else if (g.w2 > g.h2) {
    for (int c = threadIdx.x; c < g.w2; c += 256) {
      a += lut.apply(pix(p, (size_t)g.r0 * w + g.c0 + c));
      b += lut.apply(pix(p, (size_t)(g.r0 + g.h2 - 1) * w + g.c0 + c));
    }
  }
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
  __shared__ float sa[4], sb[4];
  if ((threadIdx.x & 63) == 0) { sa[threadIdx.x >> 6] = a; sb[threadIdx.x >> 6] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int n = g.h2 > g.w2 ? g.h2 : g.w2;
    edge[2 * i] = (sa[0] + sa[1] + sa[2] + sa[3]) / (float)n;
    edge[2 * i + 1] = (sb[0] + sb[1] + sb[2] + sb[3]) / (float)n;
  }
  (void)sh;
}

// pass 4: area resize of the padded square to S x S (adaptive average pooling:
// output o covers [floor(o L / S), ceil((o+1) L / S))), equalising on load,
// then (x - mean) / std into out[i][c][S][S] for every channel
template <typename TI>
__global__ void __launch_bounds__(256) prep_resize_kernel(const TI* __restrict__ src, ImgDesc d,
                                                         const float* __restrict__ mm,
                                                         const unsigned* __restrict__ hist,
                                                         const float* __restrict__ edge, int S, float mean,
                                                         float inv_std, int C, float* __restrict__ out) {
  __shared__ Lut lut;
  const int i = blockIdx.y;
  lut.build(hist, mm, i);
  const int h = d.hw[2 * i], w = d.hw[2 * i + 1];
  const Geom g(h, w);
  const TI* p = src + d.off[i];
  const float e0 = edge[2 * i], e1 = edge[2 * i + 1];
  for (int o = blockIdx.x * 256 + threadIdx.x; o < S * S; o += gridDim.x * 256) {
    const int oy = o / S, ox = o - oy * S;
    const int y0 = (int)((long long)oy * g.L / S), y1 = (int)(((long long)(oy + 1) * g.L + S - 1) / S);
    const int x0 = (int)((long long)ox * g.L / S), x1 = (int)(((long long)(ox + 1) * g.L + S - 1) / S);
    float s = 0.f;
    for (int y = y0; y < y1; ++y) {
      const int r = y - g.pt;
      for (int x = x0; x < x1; ++x) {
        const int c = x - g.pl;
        float v;
        if (g.h2 > g.w2) v = c < 0 ? e0 : (c >= g.w2 ? e1 : lut.apply(pix(p, (size_t)(g.r0 + r) * w + g.c0 + c)));
        else if (g.w2 > g.h2) v = r < 0 ? e0 : (r >= g.h2 ? e1 : lut.apply(pix(p, (size_t)(g.r0 + r) * w + g.c0 + c)));
        else v = lut.apply(pix(p, (size_t)(g.r0 + r) * w + g.c0 + c));
        s += v;
      }
    }
    const float v = (s / (float)(y1 - y0) / (float)(x1 - x0) - mean) * inv_std;   // as torch's sum / kh / kw
    for (int c = 0; c < C; ++c) out[(((size_t)i * C + c) * S + oy) * S + ox] = v;
  }
}

// ---------------- augmentation ----------------
// out[b][c][y][x] = bilinear(in[b][ci][.][.]) at source (row, col) =
// M_b (y - cy, x - cx) + (cy, cx) + t_b, clamped to the image (border), plus
// N(0, noise_std[b]) per element (counter-based: Box-Muller on hash_uniform of
// (seed, element)).  maps[b] = {m00, m01, t0, m10, m11, t1} in (row, col).
// Input fp32 [B][Cin][H][W], or uint8 [B][1][H][W] normalised on load
// ((v - mean) * inv_std; Cin = 1, broadcast to C output channels).
template <typename TI>
__global__ void __launch_bounds__(256) aug_warp_kernel(int B, int Cin, int C, int H, int W,
                                                      const TI* __restrict__ in, float mean, float inv_std,
                                                      const float* __restrict__ maps,
                                                      const float* __restrict__ noise_std, uint64_t seed,
                                                      float* __restrict__ out) {
  // grid (pixel blocks, Cin, B): a 1-channel source is sampled once per pixel
  // and written to all C output channels (each with its own noise)
  const int b = blockIdx.z, ci = blockIdx.y;
  const float* m = maps + 6 * b;
  const float cy = 0.5f * (H - 1), cx = 0.5f * (W - 1);
  const float sd = noise_std[b];
  const TI* img = in + ((size_t)b * Cin + ci) * H * W;
  const int c_lo = Cin == 1 ? 0 : ci, c_hi = Cin == 1 ? C : ci + 1;
  for (int o = blockIdx.x * 256 + threadIdx.x; o < H * W; o += gridDim.x * 256) {
    const int y = o / W, x = o - y * W;
    const float dy = y - cy, dx = x - cx;
    float sr = fminf(fmaxf(m[0] * dy + m[1] * dx + m[2] + cy, 0.f), (float)(H - 1));
    float sc = fminf(fmaxf(m[3] * dy + m[4] * dx + m[5] + cx, 0.f), (float)(W - 1));
    int r0 = (int)sr, c0 = (int)sc;
    r0 = r0 > H - 2 ? (H > 1 ? H - 2 : 0) : r0;
    c0 = c0 > W - 2 ? (W > 1 ? W - 2 : 0) : c0;
    const int r1 = r0 + 1 < H ? r0 + 1 : r0, c1 = c0 + 1 < W ? c0 + 1 : c0;
    const float fr = sr - r0, fc = sc - c0;
    float v00 = pix(img, (size_t)r0 * W + c0), v01 = pix(img, (size_t)r0 * W + c1);
    float v10 = pix(img, (size_t)r1 * W + c0), v11 = pix(img, (size_t)r1 * W + c1);
    if (sizeof(TI) == 1) {
      v00 = (v00 - mean) * inv_std; v01 = (v01 - mean) * inv_std;
      v10 = (v10 - mean) * inv_std; v11 = (v11 - mean) * inv_std;
    }
    const float v = v00 * (1.f - fr) * (1.f - fc) + v01 * (1.f - fr) * fc + v10 * fr * (1.f - fc) + v11 * fr * fc;
    for (int c = c_lo; c < c_hi; ++c) {
      const size_t idx = (((size_t)b * C + c) * H + y) * W + x;
      float u = v;
      if (sd > 0.f) {
        const float u1 = fmaxf(hash_uniform(seed, 2 * idx), 1e-12f), u2 = hash_uniform(seed, 2 * idx + 1);
        u += sd * sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
      }
      out[idx] = u;
    }
  }
}

}  // namespace vlp

using namespace vlp;

template <typename TI>
static int prep_t(int n, const void* src, const long long* off, const int* hw, int S, float mean, float std_,
                  int C, float* out, void* work, hipStream_t st) {
  float* mm = (float*)work;
  unsigned* hist = (unsigned*)(mm + (size_t)n * kPrepNB * 2);
  float* edge = (float*)(hist + (size_t)n * kBins);
  ImgDesc d{off, hw};
  hipError_t e = hipMemsetAsync(hist, 0, (size_t)n * kBins * 4, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(prep_minmax_kernel<TI>, dim3(kPrepNB, n), dim3(256), 0, st, (const TI*)src, d, mm);
  hipLaunchKernelGGL(prep_hist_kernel<TI>, dim3(kPrepNB, n), dim3(256), 0, st, (const TI*)src, d, mm, hist);
  hipLaunchKernelGGL(prep_edges_kernel<TI>, dim3(n), dim3(256), 0, st, (const TI*)src, d, mm, hist, edge);
  const int blocks = (S * S + 255) / 256 < 64 ? (S * S + 255) / 256 : 64;
  hipLaunchKernelGGL(prep_resize_kernel<TI>, dim3(blocks, n), dim3(256), 0, st, (const TI*)src, d, mm, hist, edge,
                     S, mean, 1.f / std_, C, out);
  return (int)hipGetLastError();
}

// src_u8 != 0: src holds uint8 pixels, else fp32.  hw is a DEVICE array [n][2],
// off a DEVICE array [n] (element offsets).  out fp32 [n][C][S][S].  work:
// n * (64*2 + 256 + 2) * 4 bytes (min/max partials, histograms, edge means).
VLP_EXPORT int vlp_prep_images(int n, const void* src, int src_u8, const long long* off, const int* hw, int S,
                               float mean, float std_, int C, float* out, void* work, void* stream) {
  if (n < 1 || S < 1 || C < 1 || !(std_ > 0.f) || n > 65535) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  return src_u8 ? prep_t<uint8_t>(n, src, off, hw, S, mean, std_, C, out, work, st)
                : prep_t<float>(n, src, off, hw, S, mean, std_, C, out, work, st);
}

// in_u8 != 0: in is uint8 [B][1][H][W] normalised on load, else fp32 [B][Cin][H][W]
VLP_EXPORT int vlp_aug_warp(int B, int Cin, int C, int H, int W, const void* in, int in_u8, float mean, float std_,
                            const float* maps, const float* noise_std, unsigned long long seed, float* out,
                            void* stream) {
  if (B < 1 || C < 1 || H < 1 || W < 1 || B > 65535 || C > 65535 || (Cin != 1 && Cin != C) ||
      (in_u8 && (Cin != 1 || !(std_ > 0.f))))
    return (int)hipErrorInvalidValue;
  const int blocks = (H * W + 255) / 256 < 1024 ? (H * W + 255) / 256 : 1024;
  const dim3 grid(blocks, Cin, B);
  hipStream_t st = (hipStream_t)stream;
  if (in_u8)
    hipLaunchKernelGGL(aug_warp_kernel<uint8_t>, grid, dim3(256), 0, st, B, Cin, C, H, W, (const uint8_t*)in, mean,
                       1.f / std_, maps, noise_std, (uint64_t)seed, out);
  else
    hipLaunchKernelGGL(aug_warp_kernel<float>, grid, dim3(256), 0, st, B, Cin, C, H, W, (const float*)in, mean,
                       1.f / std_, maps, noise_std, (uint64_t)seed, out);
  return (int)hipGetLastError();
}
