// Epoch-end retrieval metrics: precision@k over image
// embeddings (VisionLanguageModule.py:364-400) and image->text recall@k
// (:402-439) need the top-k most similar keys of every query over tens of
// thousands of cached embeddings.  The reference materialises the full N x N
// similarity matrix and calls topk; here the host walks query chunks (the
// similarity tile of one chunk is an fp32 GEMM, vlp_linear_fwd) and this
// kernel reduces each row of the tile to its top-K (value, index) pairs, so the
// memory is bounded by the chunk, not N^2.
#include "common.h"
#include <climits>

namespace vlp {

constexpr int kTopK = 16;   // largest k the metrics ask for + 1 (precision@15 drops the self match)

// (a, ia) ranks before (b, ib): larger value first, the lower index on ties
__device__ __forceinline__ bool tk_before(float a, int ia, float b, int ib) {
  return a > b || (a == b && ia < ib);
}

// One wave per row.  Each lane keeps its best kTopK in a descending register
// list (compare-swap chain, no dynamic indexing); then K rounds of a
// wave-wide (value, index) max pop the heads.
__global__ void __launch_bounds__(256) row_topk_kernel(int R, int N, const float* __restrict__ x, long long ldx,
                                                       int K, float* __restrict__ vals, int* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;   // wave-uniform
  const float* xr = x + (size_t)row * ldx;
  float v[kTopK];
  int ix[kTopK];
#pragma unroll
  for (int j = 0; j < kTopK; ++j) { v[j] = -INFINITY; ix[j] = INT_MAX; }
  for (int n = lane; n < N; n += 64) {
    const float s = xr[n];
    if (tk_before(s, n, v[kTopK - 1], ix[kTopK - 1])) {
      v[kTopK - 1] = s;
      ix[kTopK - 1] = n;
#pragma unroll
      for (int j = kTopK - 1; j > 0; --j) {
        const bool up = tk_before(v[j], ix[j], v[j - 1], ix[j - 1]);
        const float tv = v[j];
        const int ti = ix[j];
        v[j] = up ? v[j - 1] : v[j];
        ix[j] = up ? ix[j - 1] : ix[j];
        v[j - 1] = up ? tv : v[j - 1];
        ix[j - 1] = up ? ti : ix[j - 1];
      }
    }
  }
  for (int r = 0; r < K; ++r) {
    float bv = v[0];
    int bi = ix[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o);
      const int oi = __shfl_xor(bi, o);
      if (tk_before(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) {
      vals[(size_t)row * K + r] = bv;
      idx[(size_t)row * K + r] = bi < N ? bi : -1;
    }
    if (ix[0] == bi && bi != INT_MAX) {   // the owner pops its head
#pragma unroll
      for (int j = 0; j < kTopK - 1; ++j) { v[j] = v[j + 1]; ix[j] = ix[j + 1]; }
      v[kTopK - 1] = -INFINITY;
      ix[kTopK - 1] = INT_MAX;
    }
  }
}

}  // namespace vlp

using namespace vlp;

VLP_EXPORT int vlp_row_topk(int R, int N, const float* x, long long ldx, int K, float* vals, int* idx,
                            void* stream) {
  if (R < 0 || N < 0 || K < 1 || K > kTopK || ldx < N) return (int)hipErrorInvalidValue;
  if (R == 0) return 0;
  hipLaunchKernelGGL(row_topk_kernel, dim3((R + 3) / 4), dim3(256), 0, (hipStream_t)stream, R, N, x, ldx, K, vals,
                     idx);
  return (int)hipGetLastError();
}
