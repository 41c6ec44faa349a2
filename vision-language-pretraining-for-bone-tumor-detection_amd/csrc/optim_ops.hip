// Optimizer step and per-step weight packing.
//
// AdamW follows torch.optim.AdamW (reference optimizer: configs/optimizer/adamw.yaml,
// built in VisionLanguageModule.configure_optimizers :130-184) element-for-element:
//   p *= 1 - lr*wd;  m = b1 m + (1-b1) g;  v = b2 v + (1-b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// over flat fp32 parameter / gradient / state arenas (one launch per group).
//
// Packing turns the fp32 master conv weights (timm [Co][C][KH][KW]) into the
// GEMM operand layouts of conv_ops.hip, and the weight-gradient workspaces back.
#include "common.h"

namespace vlp {

__global__ void adamw_kernel(size_t n, float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, float lr, float b1,
                             float b2, float eps, float wd, float step_size, float bc2_sqrt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    float pi = p[i] * (1.f - lr * wd);
    float gi = g[i];
    float mi = fmaf(1.f - b1, gi - m[i], m[i]);   // torch exp_avg.lerp_(grad, 1-beta1)
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = pi - step_size * (mi / denom);
  }
}

template <typename T>
__global__ void pack_conv_kernel(int Co, int C, int KH, int KW, const float* __restrict__ w,
                                 T* __restrict__ wp, T* __restrict__ wt) {
  size_t total = (size_t)Co * C * KH * KW;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    int kw = (int)(i % KW);
    size_t t = i / KW;
    int kh = (int)(t % KH);
    t /= KH;
    int c = (int)(t % C);
    int co = (int)(t / C);
    T v = from_f<T>(w[i]);
    if (wp) wp[(((size_t)co * KH + kh) * KW + kw) * C + c] = v;
    if (wt) wt[(((size_t)c * KH + kh) * KW + kw) * Co + co] = v;
  }
}

// All convolutions of the tower packed in one launch (blockIdx.y = conv).
// wp: thread per (co, c) -> 16-bit stores coalesced over c for each tap;
// wt: thread per (c, co) -> stores coalesced over co (the strided fp32 reads
// hit the lines the other taps of the same (co, c) just pulled in).
constexpr int kPackMax = 48;
struct PackDesc {
  const float* w;
  void* wp;
  void* wt;
  int Co, C, T;
  int tiled;   // bf16, Co % 64 == C % 64 == 0, T <= 9, w 16-B aligned: 64 x 64 LDS tiles
};
struct PackBatch {
  PackDesc d[kPackMax];
};
template <typename T>
__global__ void __launch_bounds__(256) pack_conv_batch_kernel(PackBatch b) {
  const PackDesc& d = b.d[blockIdx.y];
  const int n = d.Co * d.C;
  T* wp = (T*)d.wp;
  T* wt = (T*)d.wt;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < 2 * n; i += gridDim.x * 256) {
    if (i < n) {
      if (!wp) continue;
      const int co = i / d.C, c = i - co * d.C;
      const float* src = d.w + (size_t)i * d.T;
      for (int t = 0; t < d.T; ++t) wp[((size_t)co * d.T + t) * d.C + c] = from_f<T>(src[t]);
    } else {
      if (!wt) continue;
      const int j = i - n, c = j / d.Co, co = j - c * d.Co;
      const float* src = d.w + ((size_t)co * d.C + c) * d.T;
      for (int t = 0; t < d.T; ++t) wt[((size_t)c * d.T + t) * d.Co + co] = from_f<T>(src[t]);
    }
  }
}

// The same packing by 64 (co) x 64 (c) tiles through LDS (bf16 only): each of
// the tile's 64 weight rows w[co][c0 .. c0+63][0 .. T) is 64*T contiguous fp32,
// read as float4 and rounded to bf16 into LDS once; both layouts are then
// written as 16-B rows (wp: 8 consecutive c of one (co, tap); wt: 8 consecutive
// co of one (c, tap)).  The element-per-thread kernel above read every weight
// twice with 36-B strided lanes (157 us per step for the 34 convs).
constexpr int kPackRow = 64 * 9 + 8;   // LDS row pitch (bf16), padded
__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (bf16)x); }
__global__ void __launch_bounds__(256) pack_conv_tile_kernel(PackBatch b) {
  const PackDesc& d = b.d[blockIdx.y];
  if (!d.tiled) return;
  const int tco = d.Co / 64, tc = d.C / 64;
  if ((int)blockIdx.x >= tco * tc) return;
  extern __shared__ __attribute__((aligned(16))) uint16_t pk[];   // [64 co][kPackRow]
  const int co0 = (blockIdx.x / tc) * 64, c0 = (blockIdx.x % tc) * 64;
  const int T = d.T, RL = 64 * T;   // elements per tile row
  const int tid = threadIdx.x;
  // load: 64 rows x RL fp32 (RL % 4 == 0 since 64 * T is)
  const int q4 = RL / 4;
  for (int i = tid; i < 64 * q4; i += 256) {
    const int r = i / q4, k = (i - r * q4) * 4;
    const float4 v = *reinterpret_cast<const float4*>(d.w + ((size_t)(co0 + r) * d.C + c0) * T + k);
    uint16_t* dst = pk + r * kPackRow + k;
    dst[0] = bf16_bits(v.x); dst[1] = bf16_bits(v.y); dst[2] = bf16_bits(v.z); dst[3] = bf16_bits(v.w);
  }
  __syncthreads();
  // wp[co][t][c]: chunk = (co, t, 8 c)
  if (d.wp) {
    uint16_t* wp = (uint16_t*)d.wp;
    for (int i = tid; i < 64 * T * 8; i += 256) {
      const int co = i / (T * 8), rem = i - co * T * 8, t = rem >> 3, cg = (rem & 7) * 8;
      const uint16_t* src = pk + co * kPackRow + cg * T + t;
      uint4 u;
      u.x = (uint32_t)src[0] | ((uint32_t)src[T] << 16);
      u.y = (uint32_t)src[2 * T] | ((uint32_t)src[3 * T] << 16);
      u.z = (uint32_t)src[4 * T] | ((uint32_t)src[5 * T] << 16);
      u.w = (uint32_t)src[6 * T] | ((uint32_t)src[7 * T] << 16);
      *reinterpret_cast<uint4*>(wp + ((size_t)(co0 + co) * T + t) * d.C + c0 + cg) = u;
    }
  }
  // wt[c][t][co]: chunk = (c, t, 8 co)
  if (d.wt) {
    uint16_t* wt = (uint16_t*)d.wt;
    for (int i = tid; i < 64 * T * 8; i += 256) {
      const int c = i / (T * 8), rem = i - c * T * 8, t = rem >> 3, og = (rem & 7) * 8;
      const uint16_t* src = pk + og * kPackRow + c * T + t;
      uint4 u;
      u.x = (uint32_t)src[0] | ((uint32_t)src[kPackRow] << 16);
      u.y = (uint32_t)src[2 * kPackRow] | ((uint32_t)src[3 * kPackRow] << 16);
      u.z = (uint32_t)src[4 * kPackRow] | ((uint32_t)src[5 * kPackRow] << 16);
      u.w = (uint32_t)src[6 * kPackRow] | ((uint32_t)src[7 * kPackRow] << 16);
      *reinterpret_cast<uint4*>(wt + ((size_t)(c0 + c) * T + t) * d.Co + co0 + og) = u;
    }
  }
}

// stem [64][3][7][7] -> Wp[64][kh:8][kw:8][c:4] (zeros outside)
template <typename T>
__global__ void pack_stem_kernel(const float* __restrict__ w, T* __restrict__ wp) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 256) return;
  int co = i >> 8, k = i & 255;
  int kh = k >> 5, kw = (k >> 2) & 7, c = k & 3;
  float v = 0.f;
  if (kh < 7 && kw < 7 && c < 3) v = w[((co * 3 + c) * 7 + kh) * 7 + kw];
  wp[i] = from_f<T>(v);
}

// ws[Co][KH][KW][C] -> g[Co][C][KH][KW]
__global__ void unpack_conv_grad_kernel(int Co, int C, int KH, int KW, const float* __restrict__ ws,
                                        float* __restrict__ g) {
  size_t total = (size_t)Co * C * KH * KW;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    int kw = (int)(i % KW);
    size_t t = i / KW;
    int kh = (int)(t % KH);
    t /= KH;
    int c = (int)(t % C);
    int co = (int)(t / C);
    g[i] = ws[(((size_t)co * KH + kh) * KW + kw) * C + c];
  }
}

__global__ void unpack_stem_grad_kernel(const float* __restrict__ ws, float* __restrict__ g) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 64 * 3 * 49) return;
  int kw = i % 7, kh = (i / 7) % 7, c = (i / 49) % 3, co = i / 147;
  g[i] = ws[co * 256 + kh * 32 + kw * 4 + c];
}

static inline int grid_for(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace vlp

using namespace vlp;

// step_size = lr / (1 - beta1^t), bc2_sqrt = sqrt(1 - beta2^t), computed in fp64 on the host
VLP_EXPORT int vlp_adamw(long long n, float* p, const float* g, float* m, float* v, float lr,
                         float beta1, float beta2, float eps, float wd, float step_size,
                         float bc2_sqrt, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, (size_t)n, p, g,
                     m, v, lr, beta1, beta2, eps, wd, step_size, bc2_sqrt);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_pack_conv_batch(int dtype, int n, const long long* desc, void* stream) {
  if (n < 1 || n > kPackMax) return (int)hipErrorInvalidValue;
  PackBatch b;
  int maxn = 0, maxt = 0, untiled = 0;
  for (int i = 0; i < n; ++i) {
    const long long* e = desc + 6 * i;
    const int Co = (int)e[3], C = (int)e[4], T = (int)e[5];
    const int tiled = dtype == VLP_BF16 && Co % 64 == 0 && C % 64 == 0 && T >= 1 && T <= 9 && (e[0] & 15) == 0 &&
                      (e[1] & 15) == 0 && (e[2] & 15) == 0;
    b.d[i] = PackDesc{(const float*)e[0], (void*)e[1], (void*)e[2], Co, C, T, tiled};
    if (tiled) {
      if ((Co / 64) * (C / 64) > maxt) maxt = (Co / 64) * (C / 64);
    } else {
      ++untiled;
      if (e[3] * e[4] > maxn) maxn = (int)(e[3] * e[4]);
    }
  }
  hipStream_t st = (hipStream_t)stream;
  if (maxt > 0) {
    constexpr int lds = 64 * kPackRow * 2;
    // per call (the attribute is per device; a process may drive several)
    if (hipFuncSetAttribute((const void*)&pack_conv_tile_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
      return (int)hipGetLastError();
    hipLaunchKernelGGL(pack_conv_tile_kernel, dim3(maxt, n), dim3(256), lds, st, b);
    if (hipGetLastError() != hipSuccess) return (int)hipErrorLaunchFailure;
  }
  if (untiled > 0) {   // the element-per-thread kernel skips the tiled entries
    for (int i = 0; i < n; ++i)
      if (b.d[i].tiled) b.d[i].wp = b.d[i].wt = nullptr;
    int gx = (2 * maxn + 255) / 256;
    if (gx > 2048) gx = 2048;
    if (dtype == VLP_BF16)
      hipLaunchKernelGGL(pack_conv_batch_kernel<bf16>, dim3(gx, n), dim3(256), 0, st, b);
    else
      hipLaunchKernelGGL(pack_conv_batch_kernel<float>, dim3(gx, n), dim3(256), 0, st, b);
  }
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_pack_conv(int dtype, int Co, int C, int KH, int KW, const float* w, void* wp,
                             void* wt, void* stream) {
  size_t n = (size_t)Co * C * KH * KW;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(pack_conv_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, st, Co, C, KH, KW, w,
                       (bf16*)wp, (bf16*)wt);
  else
    hipLaunchKernelGGL(pack_conv_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, Co, C, KH, KW, w,
                       (float*)wp, (float*)wt);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_pack_stem(int dtype, const float* w, void* wp, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == VLP_BF16)
    hipLaunchKernelGGL(pack_stem_kernel<bf16>, dim3(64), dim3(256), 0, st, w, (bf16*)wp);
  else
    hipLaunchKernelGGL(pack_stem_kernel<float>, dim3(64), dim3(256), 0, st, w, (float*)wp);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_unpack_conv_grad(int Co, int C, int KH, int KW, const float* ws, float* g,
                                    void* stream) {
  size_t n = (size_t)Co * C * KH * KW;
  hipLaunchKernelGGL(unpack_conv_grad_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, Co,
                     C, KH, KW, ws, g);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_unpack_stem_grad(const float* ws, float* g, void* stream) {
  hipLaunchKernelGGL(unpack_stem_grad_kernel, dim3((64 * 147 + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, ws, g);
  return (int)hipGetLastError();
}

// 2: vlp_clip_loss_fused takes (ws, ws_floats) and writes (not adds) its outputs (r3);
//    MFMA head kernels, E <= 256 with E % 4 == 0 (r4)
VLP_EXPORT int vlp_abi_version() { return 3; }
