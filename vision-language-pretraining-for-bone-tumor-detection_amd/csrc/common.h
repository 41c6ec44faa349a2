// Common device helpers for the MI355X (gfx950) CLIP pretraining hot path.
//
// Storage types: every activation / gradient tensor on the hot path is either
// bf16 (throughput mode) or fp32 (parity mode).  Kernels are templated on the
// storage type T and move data in 16-byte "chunks" (8 bf16 or 4 fp32 values),
// which is the unit the GEMM engine stages through LDS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vlp {

typedef __bf16 bf16;
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

// dtype codes used across the C ABI
enum { VLP_F32 = 0, VLP_BF16 = 1 };

template <typename T> struct Elem;
template <> struct Elem<bf16> {
  static constexpr int EPC = 8;    // elements per 16-B chunk
  static constexpr int BK = 64;    // GEMM K-step (128 B per row)
};
template <> struct Elem<float> {
  static constexpr int EPC = 4;
  static constexpr int BK = 32;
};

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// A 16-byte chunk viewed as EPC floats (unpack) / packed back.
template <typename T> struct Chunk;
template <> struct Chunk<bf16> {
  static constexpr int N = 8;
  __device__ static __forceinline__ void unpack(const uint4& u, float* f) {
    const bf16* b = reinterpret_cast<const bf16*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (float)b[j];
  }
  __device__ static __forceinline__ uint4 pack(const float* f) {
    uint4 u;
    bf16* b = reinterpret_cast<bf16*>(&u);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = (bf16)f[j];
    return u;
  }
};
template <> struct Chunk<float> {
  static constexpr int N = 4;
  __device__ static __forceinline__ void unpack(const uint4& u, float* f) {
    const float* b = reinterpret_cast<const float*>(&u);
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = b[j];
  }
  __device__ static __forceinline__ uint4 pack(const float* f) {
    uint4 u;
    float* b = reinterpret_cast<float*>(&u);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = f[j];
    return u;
  }
};

__device__ __forceinline__ uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

__device__ __forceinline__ uint4 ldg16(const void* p) {
  return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ void stg16(void* p, const uint4& v) {
  *reinterpret_cast<uint4*>(p) = v;
}

// Store 4 consecutive values (8 B for bf16, 16 B for fp32).
__device__ __forceinline__ void store4(bf16* p, v4f v) {
  v4bf b;
  b[0] = (bf16)v[0]; b[1] = (bf16)v[1]; b[2] = (bf16)v[2]; b[3] = (bf16)v[3];
  *reinterpret_cast<v4bf*>(p) = b;
}
__device__ __forceinline__ void store4(float* p, v4f v) { *reinterpret_cast<v4f*>(p) = v; }
__device__ __forceinline__ v4f load4(const bf16* p) {
  v4bf b = *reinterpret_cast<const v4bf*>(p);
  v4f r;
  r[0] = (float)b[0]; r[1] = (float)b[1]; r[2] = (float)b[2]; r[3] = (float)b[3];
  return r;
}
__device__ __forceinline__ v4f load4(const float* p) { return *reinterpret_cast<const v4f*>(p); }

// Unsigned division by a runtime constant (n < 2^31, d >= 1), branch-free
// (Granlund-Montgomery round-up): t = umulhi(n, mul); q = (t + ((n - t) >> s1)) >> s2.
struct FastDiv {
  uint32_t d, mul, s1, s2;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;  // l = ceil(log2 d)
  uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  f.mul = (uint32_t)m;          // d == 1: mul = 1, s1 = s2 = 0 -> q = n
  f.s1 = l < 1 ? l : 1;
  f.s2 = l > 1 ? l - 1 : 0;
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t t = __umulhi(n, f.mul);
  return (t + ((n - t) >> f.s1)) >> f.s2;
}

// Folded BatchNorm backward, dy = k*g + b*y + c with k = gamma*istd,
// mg = mean(g), mgx = mean(g*xhat): b = -k*istd*mgx, c = -k*mg + k*istd*mgx*mean.
// Every operation rounded as written (no contraction), so the elementwise pass
// (bn_ops) and the layer-1 rows kernel's ring transform (conv_ops) produce the
// same bits.
__device__ __forceinline__ void bn_bwd_coef(float gamma, float istd, float mean, double sum_g, double sum_gx,
                                            float inv_count, float& k, float& b, float& c) {
  k = __fmul_rn(gamma, istd);
  const float mg = __fmul_rn((float)sum_g, inv_count), mgx = __fmul_rn((float)sum_gx, inv_count);
  const float t = __fmul_rn(__fmul_rn(k, istd), mgx);
  b = -t;
  c = __fadd_rn(-__fmul_rn(k, mg), __fmul_rn(t, mean));
}
__device__ __forceinline__ float bn_bwd_dy(float k, float b, float c, float g, float y) {
  return __fmaf_rn(k, g, __fmaf_rn(b, y, c));
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based hash RNG for dropout masks: uniform in [0,1) from (seed, index).
__device__ __forceinline__ float hash_uniform(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (float)(uint32_t)(z >> 40) * (1.0f / 16777216.0f);
}

}  // namespace vlp

#define VLP_LAUNCH_CHECK() \
  do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

#define VLP_EXPORT extern "C" __attribute__((visibility("default")))
