// Probe (r6): streaming-pass shapes for the BN elementwise passes at the layer-1
// size (bs 256, 128 x 128 x 64 bf16 = 537 MB per tensor).  Each variant computes
// out = relu(y * a + r * c + b) (bn_add_relu with a residual, 2 reads + 1 write)
// or a plain copy, and prints the achieved HBM rate.
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/ew_probe tools/probes/ew_probe.hip && /tmp/ew_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ unsigned pk(float a, float b) {
  // RNE to bf16 (finite inputs)
  unsigned x = __float_as_uint(a), y = __float_as_uint(b);
  x += 0x7fffu + ((x >> 16) & 1u);
  y += 0x7fffu + ((y >> 16) & 1u);
  return (x >> 16) | (y & 0xffff0000u);
}
__device__ __forceinline__ v4u op(v4u y, v4u r, const float* a, const float* b, const float* c) {
  v4u o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float u0 = fmaxf(fmaf(lo(y[j]), a[2 * j], fmaf(lo(r[j]), c[2 * j], b[2 * j])), 0.f);
    const float u1 = fmaxf(fmaf(hi(y[j]), a[2 * j + 1], fmaf(hi(r[j]), c[2 * j + 1], b[2 * j + 1])), 0.f);
    o[j] = pk(u0, u1);
  }
  return o;
}

// grid-stride, U chunks per iteration (loads first), optional non-temporal loads / stores
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) gs_kernel(unsigned n, const v4u* __restrict__ y, const v4u* __restrict__ r,
                                                 v4u* __restrict__ out, const float* __restrict__ coef) {
  const unsigned tid = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  float a[8], b[8], c[8];
  const int c0 = (tid & 7) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = coef[c0 + j]; b[j] = coef[64 + c0 + j]; c[j] = coef[128 + c0 + j]; }
  unsigned i = tid;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    v4u yv[U], rv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NTL) { yv[k] = __builtin_nontemporal_load(y + i + k * stride); rv[k] = __builtin_nontemporal_load(r + i + k * stride); }
      else { yv[k] = y[i + k * stride]; rv[k] = r[i + k * stride]; }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const v4u o = op(yv[k], rv[k], a, b, c);
      if (NTS) __builtin_nontemporal_store(o, out + i + k * stride);
      else out[i + k * stride] = o;
    }
  }
  for (; i < n; i += stride) {
    const v4u o = op(y[i], r[i], a, b, c);
    if (NTS) __builtin_nontemporal_store(o, out + i);
    else out[i] = o;
  }
}

// blocked: a workgroup owns contiguous segments of 256 * U chunks (thread t: chunks
// seg + t + 256 k), segments grid-strided
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) blk_kernel(unsigned n, const v4u* __restrict__ y, const v4u* __restrict__ r,
                                                  v4u* __restrict__ out, const float* __restrict__ coef) {
  float a[8], b[8], c[8];
  const int c0 = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int j = 0; j < 8; ++j) { a[j] = coef[c0 + j]; b[j] = coef[64 + c0 + j]; c[j] = coef[128 + c0 + j]; }
  const unsigned seg = 256u * U;
  for (unsigned s = blockIdx.x * seg; s < n; s += gridDim.x * seg) {
    const unsigned i = s + threadIdx.x;
    v4u yv[U], rv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NTL) { yv[k] = __builtin_nontemporal_load(y + i + 256 * k); rv[k] = __builtin_nontemporal_load(r + i + 256 * k); }
      else { yv[k] = y[i + 256 * k]; rv[k] = r[i + 256 * k]; }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const v4u o = op(yv[k], rv[k], a, b, c);
      if (NTS) __builtin_nontemporal_store(o, out + i + 256 * k);
      else out[i + 256 * k] = o;
    }
  }
}

template <bool NTS>
__global__ void __launch_bounds__(256) copy_kernel(unsigned n, const v4u* __restrict__ y, v4u* __restrict__ out) {
  const unsigned stride = gridDim.x * 256;
  for (unsigned i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    if (NTS) __builtin_nontemporal_store(y[i], out + i);
    else out[i] = y[i];
  }
}

int main() {
  const size_t elems = (size_t)256 * 128 * 128 * 64;   // bf16 elements per tensor
  const unsigned n = (unsigned)(elems / 8);            // 16-B chunks
  const size_t bytes = elems * 2;
  v4u *y, *r, *o;
  float* coef;
  hipMalloc(&y, bytes); hipMalloc(&r, bytes); hipMalloc(&o, bytes); hipMalloc(&coef, 192 * 4);
  hipMemset(y, 0x3c, bytes); hipMemset(r, 0x3b, bytes); hipMemset(coef, 0, 192 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](const char* name, double mult, auto launch) {
    for (int w = 0; w < 3; ++w) launch();
    hipDeviceSynchronize();
    const int it = 20;
    hipEventRecord(e0);
    for (int k = 0; k < it; ++k) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / it;
    printf("%-34s %8.1f us  %5.2f TB/s\n", name, us, mult * bytes / us / 1e6);
  };
#define GS(U, NTL, NTS, G) run("gs U=" #U " ntl=" #NTL " nts=" #NTS " grid=" #G, 3.0, [&] { hipLaunchKernelGGL((gs_kernel<U, NTL, NTS>), dim3(G), dim3(256), 0, 0, n, y, r, o, coef); })
#define BK(U, NTL, NTS, G) run("blk U=" #U " ntl=" #NTL " nts=" #NTS " grid=" #G, 3.0, [&] { hipLaunchKernelGGL((blk_kernel<U, NTL, NTS>), dim3(G), dim3(256), 0, 0, n, y, r, o, coef); })
  run("copy grid=4096", 2.0, [&] { hipLaunchKernelGGL((copy_kernel<false>), dim3(4096), dim3(256), 0, 0, n, y, o); });
  run("copy nts grid=4096", 2.0, [&] { hipLaunchKernelGGL((copy_kernel<true>), dim3(4096), dim3(256), 0, 0, n, y, o); });
  run("copy grid=2048", 2.0, [&] { hipLaunchKernelGGL((copy_kernel<false>), dim3(2048), dim3(256), 0, 0, n, y, o); });
  run("copy grid=16384", 2.0, [&] { hipLaunchKernelGGL((copy_kernel<false>), dim3(16384), dim3(256), 0, 0, n, y, o); });
  GS(1, false, true, 4096);    // the product's default shape (bn_add_relu_kernel<bf16, true, 1, NT>)
  GS(1, true, true, 4096);
  BK(4, false, true, 2048);
  BK(2, true, true, 2048);
  BK(4, true, true, 1024);
  BK(4, true, true, 2048);
  BK(4, true, true, 4096);
  BK(8, true, true, 1024);
  BK(8, true, true, 2048);
  BK(16, true, true, 1024);
  BK(4, true, false, 2048);
  return 0;
}
