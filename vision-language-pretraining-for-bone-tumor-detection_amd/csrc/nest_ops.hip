// NesT-Small image encoder kernels (BASELINE configs[3]).
//
// The reference reaches NesT through ImageEncoder's generic
// timm.create_model(model, num_classes=0, global_pool="avg", ...)
// (src/models/pretrain/VisionLanguageModule.py:27-35; timm==1.0.15 nest.py,
// not installed here).  Besides the GEMMs / LayerNorms shared with the text
// tower (bert_ops.hip), NesT needs:
//   * blocked local self-attention: every image block of N = 1024 tokens
//     (512x512 input) attends within itself, head dim 32 -- flash attention
//     on MFMA, forward + two backward kernels (dK/dV over key tiles, dQ over
//     query tiles), log-sum-exp saved by the forward;
//   * blockify / deblockify (+ the level's positional embedding);
//   * ConvPool's 3x3/2 max pool (after the channel LayerNorm);
//   * the patch-embedding im2col (4x4/4, non-overlapping) from the collated
//     batch (uint8 1-channel upload or the reference's fp32 3-channel tensor);
//   * DropPath (stochastic depth, timm's default drop_path_rate = 0.5) as a
//     per-sample scale on each residual branch.
// Attention layout: q/k/v are the columns [0,C), [C,2C), [2C,3C) of the
// qkv Linear's output rows, head h at h*32.. (nn.Linear(dim, 3*dim) reshaped
// (3, heads, 32)); the output is written head-major [row][h*32 + d].  timm
// NesT's Attention emits channel d*H + h instead (permute(0,2,3,4,1)); the
// host folds that permutation into the proj weight (vlp_nest_permute_cols).
#include "common.h"
#include "gemm.h"

namespace vlp {

constexpr int kDh = 32;                 // head dim (every NesT variant: C / heads = 32)
constexpr int kTileRows = 64;           // key / query tokens per staged tile
constexpr int kQBlock = 128;            // queries per forward / dQ workgroup (4 waves x 32)

// ---------------- fragments (MFMA 16x16x32 bf16 / 16x16x4 f32) ----------------
// Convention as bert_ops.hip: D[m][n] = sum_k X[m][k] Y[n][k]; lane l = 16g + i
// holds D[4g + r][i].
//
// Tiles of 64 tokens x 32 channels are staged in LDS as [token][channel]
// images.  bf16 images are unpadded 64-B rows whose four 16-B chunks are
// XOR-swizzled by sw(row) = ((row>>2)&1)<<1 | ((row>>3)&1): the ds_read_b128
// row read (16 consecutive rows, one chunk) and the ds_read_b64_tr_b16
// transposed read (rows 4g + q of two groups, two adjacent chunks) are both
// bank-conflict free on it.  fp32 images are padded rows of 36 floats.
//
// Score tiles never pass through LDS: an accumulator v4f s[b] (b = 0..3) holds
// S[key 16b + 4g + r][i] (or S[q 16b + 4g + r][key i] in dK/dV), and the MFMA's
// k-slot order is free as long as both operands agree, so pfrag() hands the
// accumulators (as bf16) straight to the next product as the operand whose
// k-slot j of lane group g is token 16(2h + j/4) + 4g + j%4; vtfrag() reads the
// other operand (a [token][channel] image, channel on the lane) in that order.
template <typename T> struct FA;
template <> struct FA<bf16> {
  static constexpr int KS = 32, IMG = kTileRows * 32;
  typedef v8bf F;
  __device__ static __forceinline__ int sw(int row) { return (((row >> 2) & 1) << 1) | ((row >> 3) & 1); }
  __device__ static __forceinline__ int at(int row, int col) {
    return row * 32 + ((((col >> 3) ^ sw(row)) << 3) | (col & 7));
  }
  // rows r0 + i, k = k0 + 8g .. +7 of an image (k0 = 0: one k-step spans the 32 channels)
  __device__ static __forceinline__ F kfrag(const bf16* img, int r0, int k0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    return *reinterpret_cast<const v8bf*>(img + at(r0 + i, k0 + 8 * g));
  }
  // channels c0 + i (lane row), k-slots = tokens t0 + 16(j/4) + 4g + j%4
  __device__ static __forceinline__ F vtfrag(const bf16* img, int t0, int c0) {
    const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int r = t0 + 4 * g + q, c = c0 + 4 * p;
    v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(img + at(r, c)));
    v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(img + at(r + 16, c)));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
  // accumulators s[2h], s[2h+1] as the operand of k-step h
  __device__ static __forceinline__ F pfrag(const v4f* s, int h) {
    F f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      f[r] = (bf16)s[2 * h][r];
      f[4 + r] = (bf16)s[2 * h + 1][r];
    }
    return f;
  }
  __device__ static __forceinline__ F ones() {
    F f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (bf16)1.f;
    return f;
  }
  // a fragment straight from global memory (rows r0.., k contiguous)
  __device__ static __forceinline__ F gfrag(const bf16* p, size_t ld, int r0, int k0, bool ok) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    if (!ok) return F{};
    return *reinterpret_cast<const v8bf*>(p + (size_t)(r0 + i) * ld + k0 + 8 * g);
  }
  __device__ static __forceinline__ void mma(v4f& acc, const F& x, const F& y) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc, 0, 0, 0);
  }
};
template <> struct FA<float> {
  static constexpr int KS = 16, LD = 36, IMG = kTileRows * LD;
  typedef v4f F;
  __device__ static __forceinline__ int at(int row, int col) { return row * LD + col; }
  __device__ static __forceinline__ F kfrag(const float* img, int r0, int k0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    return *reinterpret_cast<const v4f*>(img + at(r0 + i, k0 + 4 * g));
  }
  // element j of lane (g, i): image[t0 + 4g + j][c0 + i]  (mma j: k-slot g)
  __device__ static __forceinline__ F vtfrag(const float* img, int t0, int c0) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    F f;
#pragma unroll
    for (int j = 0; j < 4; ++j) f[j] = img[at(t0 + 4 * g + j, c0 + i)];
    return f;
  }
  __device__ static __forceinline__ F pfrag(const v4f* s, int h) { return s[h]; }
  __device__ static __forceinline__ F ones() { return F{1.f, 1.f, 1.f, 1.f}; }
  __device__ static __forceinline__ F gfrag(const float* p, size_t ld, int r0, int k0, bool ok) {
    const int l = threadIdx.x & 63, i = l & 15, g = l >> 4;
    if (!ok) return F{0.f, 0.f, 0.f, 0.f};
    return *reinterpret_cast<const v4f*>(p + (size_t)(r0 + i) * ld + k0 + 4 * g);
  }
  __device__ static __forceinline__ void mma(v4f& acc, const F& x, const F& y) {
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[j], y[j], acc, 0, 0, 0);
  }
};

// single-instruction maxima (fmaxf on MFMA results otherwise gets a
// canonicalising v_max per operand)
__device__ __forceinline__ float max2_(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float max3_(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
// maximum of the 16 scores a lane holds
__device__ __forceinline__ float max16(const v4f* s) {
  float m = max3_(s[0][0], s[0][1], s[0][2]);
  m = max3_(m, s[0][3], s[1][0]);
  m = max3_(m, s[1][1], s[1][2]);
  m = max3_(m, s[1][3], s[2][0]);
  m = max3_(m, s[2][1], s[2][2]);
  m = max3_(m, s[2][3], s[3][0]);
  m = max3_(m, s[3][1], s[3][2]);
  return max2_(m, s[3][3]);
}
__device__ __forceinline__ float q4max(float v) {
  v = max2_(v, __shfl_xor(v, 16, 64));
  return max2_(v, __shfl_xor(v, 32, 64));
}
__device__ __forceinline__ float q4sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}
// v_exp_f32: 2^x without OCML's denormal-range fix-up (results below 2^-126
// flush to 0, far below what a bf16/fp32 softmax weight resolves)
__device__ __forceinline__ float exp2_hw(float x) { return __builtin_amdgcn_exp2f(x); }

// four consecutive values of one row -> memory (8 B bf16 / 16 B fp32)
template <typename T>
__device__ __forceinline__ void st4(T* p, float a, float b, float c, float d);
template <> __device__ __forceinline__ void st4<bf16>(bf16* p, float a, float b, float c, float d) {
  v4bf v;
  v[0] = (bf16)a; v[1] = (bf16)b; v[2] = (bf16)c; v[3] = (bf16)d;
  *reinterpret_cast<v4bf*>(p) = v;
}
template <> __device__ __forceinline__ void st4<float>(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<v4f*>(p) = v4f{a, b, c, d};
}

// Register-staged tile copy (issue the global loads early, write the LDS
// image after the barrier): rows [t0, t0+64) x 32 channels at column `col` of a
// [rows][ld] tensor; rows >= N are zero in the image.  The loads are
// unconditional (row index clamped to N-1); the store applies the row mask.
// 256 threads.  The loads are inline asm, waited for by hand at the bottom of the
// tile loop (vmcnt 0, tied to the loaded registers, so no copy of them can be
// placed before the data lands -- waiting at the top let the loop's back-edge
// copies read registers still in flight): as plain loads the compiler sank the
// next tile's loads below the tile's MFMAs, to the loop header right in front of
// their store, so every tile of the dK/dV kernel waited out a full global-load
// round trip twice (r4 PMC: half of its wave cycles waiting).
#ifndef VLP_ATTN_ASMLOAD   // 0: plain loads (the compiler places them), for A/B
#define VLP_ATTN_ASMLOAD 1
#endif
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// early-clobber outputs: the destination must not share registers with the
// address (the compiler would otherwise reuse them and copy the "result" early)
__device__ __forceinline__ u32x4 ldg16_issue(const void* p) {
  u32x4 r;
#if VLP_ATTN_ASMLOAD
  asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(r) : "v"(p) : "memory");
#else
  r = *reinterpret_cast<const u32x4*>(p);
#endif
  return r;
}
__device__ __forceinline__ float ldg4_issue(const float* p) {
#if VLP_ATTN_ASMLOAD
  float r;
  asm volatile("global_load_dword %0, %1, off" : "=&v"(r) : "v"(p) : "memory");
  return r;
#else
  return *p;
#endif
}
// make a value loaded by an ordinary (compiler-tracked) load opaque: the
// compiler waits for the load once here instead of at its first use inside the
// tile loop, where its waitcnt pass would put a vmcnt(0) on every iteration and
// drain the hand-issued tile prefetch
template <class X>
__device__ __forceinline__ void launder(X& x) {
  asm volatile("" : "+v"(x));
}
template <typename T>
struct TileStage {
  static constexpr int EPC = 16 / (int)sizeof(T), CPR = kDh / EPC, CPT = kTileRows * CPR / 256;
  u32x4 v[CPT];
  __device__ __forceinline__ void load(const T* src, size_t ld, int col, int t0, int N) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int q = threadIdx.x + 256 * c, r = q / CPR, ch = q % CPR;
      v[c] = ldg16_issue(src + (size_t)min(t0 + r, N - 1) * ld + col + ch * EPC);
    }
  }
  // every vector-memory load of this thread retired (the staged registers tied in)
  __device__ __forceinline__ void wait() {
#pragma unroll
    for (int c = 0; c < CPT; ++c)
      if (VLP_ATTN_ASMLOAD) asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[c])::"memory");
  }
  __device__ __forceinline__ void store(T* img, int t0, int N) const {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int q = threadIdx.x + 256 * c, r = q / CPR, ch = q % CPR;
      const u32x4 z = {0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(img + FA<T>::at(r, ch * EPC)) = t0 + r < N ? v[c] : z;
    }
  }
};

// ---------------- grid ----------------
// The attention kernels run a 1-D grid of nx tiles x H heads x BT blocks.
// VLP_ATTN_XCD = 1: the block id is remapped so that each XCD owns a contiguous
// run of (tile, head, block) ids -- the nx tiles of one (block, head), which all
// re-read that pair's 64 KB K/V (Q/dO) slices, then sit on one XCD together and
// hit its L2 (with the plain round-robin dispatch they spread over all 8 XCDs).
// 0: the id is used as is (neighbouring tiles on different XCDs).
#ifndef VLP_ATTN_XCD
#define VLP_ATTN_XCD 1
#endif
__device__ __forceinline__ void attn_tile(int nx, int H, int& x, int& h, int& bt) {
  const int total = (int)gridDim.x;
  int id = (int)blockIdx.x;
#if VLP_ATTN_XCD
  if (total >= 16) {
    const int xcd = id & 7, idx = id >> 3, q = total >> 3, rr = total & 7;
    id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
#endif
  x = id % nx;
  const int r = id / nx;
  h = r % H;
  bt = r / H;
}

// ---------------- forward ----------------
// grid (ceil(N/128), H, BT); 4 waves, wave w owns queries qt*128 + 32w .. +31
// as two 16-query subtiles that share every K / V fragment read.
// out[bt*N + q][h*32 + d]; lse[(bt*H + h)*N + q] = log2-sum-exp of the scaled
// (x log2 e) scores.  Per key tile: S^T = K Q^T, the online softmax in
// registers (lane = query, 16 keys per lane), O^T += V^T P^T with P fed from
// the accumulators; the row sums come out of the same product with a ones
// operand (1^T P^T), i.e. they sum exactly the weights O accumulates.
template <typename T>
__global__ void __launch_bounds__(256)
nest_attn_fwd_kernel(int BT, int H, int N, const T* __restrict__ qkv, T* __restrict__ out,
                     float* __restrict__ lse, float sl2) {
  using M = FA<T>;
  constexpr int QW = 2, KSN = kDh / M::KS;
  __shared__ __attribute__((aligned(16))) T sK[M::IMG];
  __shared__ __attribute__((aligned(16))) T sV[M::IMG];
  int qt, h, bt;
  attn_tile((N + kQBlock - 1) / kQBlock, H, qt, h, bt);
  const int C = H * kDh;
  const size_t ld3 = 3 * (size_t)C;
  const T* base = qkv + (size_t)bt * N * ld3;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  const int q0 = qt * kQBlock + 32 * w;
  typename M::F qf[QW][KSN];
#pragma unroll
  for (int u = 0; u < QW; ++u)
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks)
      qf[u][ks] = M::gfrag(base + h * kDh, ld3, q0 + 16 * u, ks * M::KS, q0 + 16 * u + li < N);
  const typename M::F one = M::ones();
  float mi[QW];
  v4f o[QW][2], lsum[QW];
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    mi[u] = -INFINITY;
    lsum[u] = o[u][0] = o[u][1] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  const int nt = (N + kTileRows - 1) / kTileRows;
#pragma unroll
  for (int u = 0; u < QW; ++u)
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) launder(qf[u][ks]);
  TileStage<T> stk, stv;
  stk.load(base, ld3, C + h * kDh, 0, N);
  stv.load(base, ld3, 2 * C + h * kDh, 0, N);
  stk.wait();
  stv.wait();
  for (int t = 0; t < nt; ++t) {
    __syncthreads();   // every wave is done with the previous tile
    stk.store(sK, t * kTileRows, N);
    stv.store(sV, t * kTileRows, N);
    __syncthreads();
    // next tile's loads fly under this tile's MFMAs (unconditional: past the
    // end they re-read row N-1, which keeps the loaded registers phi-free so
    // nothing waits on them before the next store)
    stk.load(base, ld3, C + h * kDh, (t + 1) * kTileRows, N);
    stv.load(base, ld3, 2 * C + h * kDh, (t + 1) * kTileRows, N);
    v4f s[QW][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
#pragma unroll
      for (int u = 0; u < QW; ++u) s[u][b] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        const typename M::F kf = M::kfrag(sK, 16 * b, ks * M::KS);
#pragma unroll
        for (int u = 0; u < QW; ++u) M::mma(s[u][b], kf, qf[u][ks]);
      }
    }
    if (t * kTileRows + kTileRows > N) {   // partial last tile: keys >= N take no weight
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (t * kTileRows + 16 * b + 4 * lg + r >= N)
#pragma unroll
            for (int u = 0; u < QW; ++u) s[u][b][r] = -INFINITY;
    }
#pragma unroll
    for (int u = 0; u < QW; ++u) {
      const float mn = max2_(mi[u], q4max(max16(s[u])) * sl2);   // running max of the scaled scores
      const float alpha = exp2_hw(mi[u] - mn);                   // 0 on the first tile (mi = -inf)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) s[u][b][r] = exp2_hw(fmaf(s[u][b][r], sl2, -mn));
      mi[u] = mn;
      o[u][0] *= alpha;
      o[u][1] *= alpha;
      lsum[u] *= alpha;
    }
    // O^T[d][q] += sum_key V^T[d][key] P[q][key];  l[q] += sum_key P[q][key]
#pragma unroll
    for (int hs = 0; hs < kTileRows / M::KS; ++hs) {
      const typename M::F v0 = M::vtfrag(sV, hs * M::KS, 0), v1 = M::vtfrag(sV, hs * M::KS, 16);
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const typename M::F pf = M::pfrag(s[u], hs);
        M::mma(o[u][0], v0, pf);
        M::mma(o[u][1], v1, pf);
        M::mma(lsum[u], one, pf);
      }
    }
    stk.wait();   // the next tile's rows landed (issued before this tile's MFMAs)
    stv.wait();
  }
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    const int q = q0 + 16 * u + li;
    if (q < N) {
      const float inv = 1.f / lsum[u][0];
      T* dst = out + ((size_t)bt * N + q) * C + h * kDh;
#pragma unroll
      for (int db = 0; db < 2; ++db)
        st4<T>(dst + 16 * db + 4 * lg, o[u][db][0] * inv, o[u][db][1] * inv, o[u][db][2] * inv,
               o[u][db][3] * inv);
      if (lg == 0) lse[((size_t)bt * H + h) * N + q] = mi[u] + log2f(lsum[u][0]);
    }
  }
}

// delta[(bt*H + h)*N + q] = sum_d dout[row][h*32 + d] * out[row][h*32 + d]
template <typename T>
__global__ void nest_attn_delta_kernel(int BT, int H, int N, const T* __restrict__ out,
                                       const T* __restrict__ dout, float* __restrict__ delta) {
  constexpr int EPC = 16 / (int)sizeof(T);
  const size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x;   // (row, h)
  const size_t total = (size_t)BT * N * H;
  if (idx >= total) return;
  const size_t row = idx / H;
  const int h = (int)(idx - row * H);
  const int C = H * kDh;
  const T* a = out + row * C + h * kDh;
  const T* b = dout + row * C + h * kDh;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kDh; c += EPC) {
    float x[EPC], y[EPC];
    Chunk<T>::unpack(ldg16(a + c), x);
    Chunk<T>::unpack(ldg16(b + c), y);
#pragma unroll
    for (int j = 0; j < EPC; ++j) s += x[j] * y[j];
  }
  const size_t bt = row / N, q = row - bt * N;
  delta[(bt * H + h) * N + q] = s;
}

// ---------------- backward: dQ over key tiles ----------------
// grid (ceil(N/128), H, BT); wave w owns queries qt*128 + 32w .. +31 as two
// 16-query subtiles (lane = query) sharing the K / V fragment reads.
//   P = exp2(S*sl2 - lse), dP' = dO V^T - delta (the accumulator starts at
//   -delta), dS = P dP', dQ^T += K^T dS^T with dS fed from the accumulators.
template <typename T>
__global__ void __launch_bounds__(256)
nest_attn_bwd_dq_kernel(int BT, int H, int N, const T* __restrict__ qkv, const T* __restrict__ dout,
                        const float* __restrict__ lse, const float* __restrict__ delta, T* __restrict__ dqkv,
                        float sl2, float scale) {
  using M = FA<T>;
  constexpr int QW = 2, KSN = kDh / M::KS;
  __shared__ __attribute__((aligned(16))) T sK[M::IMG];
  __shared__ __attribute__((aligned(16))) T sV[M::IMG];
  int qt, h, bt;
  attn_tile((N + kQBlock - 1) / kQBlock, H, qt, h, bt);
  const int C = H * kDh;
  const size_t ld3 = 3 * (size_t)C;
  const T* base = qkv + (size_t)bt * N * ld3;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  const int q0 = qt * kQBlock + 32 * w;
  typename M::F qf[QW][KSN], df[QW][KSN];
  float lq[QW], ndl[QW];
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    const int q = q0 + 16 * u;
    const bool ok = q + li < N;
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      qf[u][ks] = M::gfrag(base + h * kDh, ld3, q, ks * M::KS, ok);
      df[u][ks] = M::gfrag(dout + (size_t)bt * N * C + h * kDh, C, q, ks * M::KS, ok);
    }
    const size_t so = ((size_t)bt * H + h) * N + q + li;
    lq[u] = ok ? lse[so] : INFINITY;
    ndl[u] = ok ? -delta[so] : 0.f;
  }
  v4f acc[QW][2];
#pragma unroll
  for (int u = 0; u < QW; ++u) acc[u][0] = acc[u][1] = v4f{0.f, 0.f, 0.f, 0.f};
  const int nt = (N + kTileRows - 1) / kTileRows;
#pragma unroll
  for (int u = 0; u < QW; ++u) {
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      launder(qf[u][ks]);
      launder(df[u][ks]);
    }
    launder(lq[u]);
    launder(ndl[u]);
  }
  TileStage<T> stk, stv;
  stk.load(base, ld3, C + h * kDh, 0, N);
  stv.load(base, ld3, 2 * C + h * kDh, 0, N);
  stk.wait();
  stv.wait();
  for (int t = 0; t < nt; ++t) {
    __syncthreads();
    stk.store(sK, t * kTileRows, N);
    stv.store(sV, t * kTileRows, N);
    __syncthreads();
    stk.load(base, ld3, C + h * kDh, (t + 1) * kTileRows, N);
    stv.load(base, ld3, 2 * C + h * kDh, (t + 1) * kTileRows, N);
    v4f ds[QW][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      v4f sc[QW], dp[QW];
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        sc[u] = v4f{0.f, 0.f, 0.f, 0.f};
        dp[u] = v4f{ndl[u], ndl[u], ndl[u], ndl[u]};
      }
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        const typename M::F kf = M::kfrag(sK, 16 * b, ks * M::KS), vf = M::kfrag(sV, 16 * b, ks * M::KS);
#pragma unroll
        for (int u = 0; u < QW; ++u) {
          M::mma(sc[u], kf, qf[u][ks]);
          M::mma(dp[u], vf, df[u][ks]);
        }
      }
#pragma unroll
      for (int u = 0; u < QW; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) ds[u][b][r] = exp2_hw(fmaf(sc[u][r], sl2, -lq[u])) * dp[u][r];
    }
    if (t * kTileRows + kTileRows > N) {   // keys >= N (zero rows) carry no probability
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (t * kTileRows + 16 * b + 4 * lg + r >= N)
#pragma unroll
            for (int u = 0; u < QW; ++u) ds[u][b][r] = 0.f;
    }
    // dQ^T[d][q] += sum_key K^T[d][key] dS[q][key]
#pragma unroll
    for (int hs = 0; hs < kTileRows / M::KS; ++hs) {
      const typename M::F k0 = M::vtfrag(sK, hs * M::KS, 0), k1 = M::vtfrag(sK, hs * M::KS, 16);
#pragma unroll
      for (int u = 0; u < QW; ++u) {
        const typename M::F pf = M::pfrag(ds[u], hs);
        M::mma(acc[u][0], k0, pf);
        M::mma(acc[u][1], k1, pf);
      }
    }
    stk.wait();
    stv.wait();
  }
#pragma unroll
  for (int u = 0; u < QW; ++u) {
    const int q = q0 + 16 * u + li;
    if (q < N) {
      T* dst = dqkv + ((size_t)bt * N + q) * ld3 + h * kDh;
#pragma unroll
      for (int db = 0; db < 2; ++db)
        st4<T>(dst + 16 * db + 4 * lg, acc[u][db][0] * scale, acc[u][db][1] * scale, acc[u][db][2] * scale,
               acc[u][db][3] * scale);
    }
  }
}

// ---------------- backward: dK, dV over query tiles ----------------
// grid (ceil(N/64), H, BT); wave w owns keys kt*64 + 16w .. +15 (lane = key;
// two key subtiles per wave measured slower: 188 VGPRs halve the occupancy).
//   S[q][key] = Q K^T and dP[q][key] - delta[q] as accumulators (row q =
//   16b + 4g + r), P and dS from them, then dV^T += dO^T P and dK^T += Q^T dS
//   with P / dS fed from the accumulators.  Query rows >= N are zero in the
//   images with lse = +inf, so they carry no probability.
template <typename T>
__global__ void __launch_bounds__(256)
nest_attn_bwd_dkdv_kernel(int BT, int H, int N, const T* __restrict__ qkv, const T* __restrict__ dout,
                          const float* __restrict__ lse, const float* __restrict__ delta,
                          T* __restrict__ dqkv, float sl2, float scale) {
  using M = FA<T>;
  constexpr int KW = 1, KSN = kDh / M::KS;
  __shared__ __attribute__((aligned(16))) T sQ[M::IMG];
  __shared__ __attribute__((aligned(16))) T sD[M::IMG];
  __shared__ __attribute__((aligned(16))) float sL[kTileRows], sDl[kTileRows];
  int kt, h, bt;
  attn_tile((N + 63) / 64, H, kt, h, bt);
  const int C = H * kDh;
  const size_t ld3 = 3 * (size_t)C;
  const T* base = qkv + (size_t)bt * N * ld3;
  const T* dbase = dout + (size_t)bt * N * C;
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, li = l & 15, lg = l >> 4;
  const int k0 = kt * 64 * KW + 16 * KW * w;
  typename M::F kf[KW][KSN], vf[KW][KSN];
#pragma unroll
  for (int u = 0; u < KW; ++u)
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      const bool ok = k0 + 16 * u + li < N;
      kf[u][ks] = M::gfrag(base + C + h * kDh, ld3, k0 + 16 * u, ks * M::KS, ok);
      vf[u][ks] = M::gfrag(base + 2 * C + h * kDh, ld3, k0 + 16 * u, ks * M::KS, ok);
    }
  v4f dk[KW][2], dv[KW][2];
#pragma unroll
  for (int u = 0; u < KW; ++u) dk[u][0] = dk[u][1] = dv[u][0] = dv[u][1] = v4f{0.f, 0.f, 0.f, 0.f};
  const size_t sb = ((size_t)bt * H + h) * N;
  const int nt = (N + kTileRows - 1) / kTileRows;
#pragma unroll
  for (int u = 0; u < KW; ++u)
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      launder(kf[u][ks]);
      launder(vf[u][ks]);
    }
  TileStage<T> stq, std_;
  float pl = 0.f, pd = 0.f;
  auto load_rows = [&](int t0) {
    stq.load(base, ld3, h * kDh, t0, N);
    std_.load(dbase, C, h * kDh, t0, N);
    const int q = min(t0 + (int)(threadIdx.x & (kTileRows - 1)), N - 1);   // every thread: no phi
    pl = ldg4_issue(lse + sb + q);
    pd = ldg4_issue(delta + sb + q);
  };
  auto wait_rows = [&]() {
    stq.wait();
    std_.wait();
    if (VLP_ATTN_ASMLOAD) asm volatile("s_waitcnt vmcnt(0)" : "+v"(pl), "+v"(pd)::"memory");
  };
  load_rows(0);
  wait_rows();
  for (int t = 0; t < nt; ++t) {
    __syncthreads();
    stq.store(sQ, t * kTileRows, N);
    std_.store(sD, t * kTileRows, N);
    if (threadIdx.x < kTileRows) {
      const bool ok = t * kTileRows + (int)threadIdx.x < N;
      sL[threadIdx.x] = ok ? pl : INFINITY;
      sDl[threadIdx.x] = ok ? -pd : 0.f;
    }
    __syncthreads();
    load_rows((t + 1) * kTileRows);
    v4f p[KW][4], ds[KW][4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const v4f lq = *reinterpret_cast<const v4f*>(sL + 16 * b + 4 * lg);
      const v4f ndl = *reinterpret_cast<const v4f*>(sDl + 16 * b + 4 * lg);
      v4f sc[KW], dp[KW];
#pragma unroll
      for (int u = 0; u < KW; ++u) {
        sc[u] = v4f{0.f, 0.f, 0.f, 0.f};
        dp[u] = ndl;
      }
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        const typename M::F qa = M::kfrag(sQ, 16 * b, ks * M::KS), da = M::kfrag(sD, 16 * b, ks * M::KS);
#pragma unroll
        for (int u = 0; u < KW; ++u) {
          M::mma(sc[u], qa, kf[u][ks]);
          M::mma(dp[u], da, vf[u][ks]);
        }
      }
#pragma unroll
      for (int u = 0; u < KW; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[u][b][r] = exp2_hw(fmaf(sc[u][r], sl2, -lq[r]));
          ds[u][b][r] = p[u][b][r] * dp[u][r];
        }
    }
    // dV^T[d][key] += sum_q dO^T[d][q] P[q][key];  dK^T[d][key] += sum_q Q^T[d][q] dS[q][key]
#pragma unroll
    for (int hs = 0; hs < kTileRows / M::KS; ++hs)
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        const typename M::F dt = M::vtfrag(sD, hs * M::KS, 16 * db), qt_ = M::vtfrag(sQ, hs * M::KS, 16 * db);
#pragma unroll
        for (int u = 0; u < KW; ++u) {
          M::mma(dv[u][db], dt, M::pfrag(p[u], hs));
          M::mma(dk[u][db], qt_, M::pfrag(ds[u], hs));
        }
      }
    wait_rows();   // the next tile's rows landed (issued before this tile's MFMAs)
  }
#pragma unroll
  for (int u = 0; u < KW; ++u) {
    const int key = k0 + 16 * u + li;
    if (key < N) {
      T* dst = dqkv + ((size_t)bt * N + key) * ld3 + h * kDh;
#pragma unroll
      for (int db = 0; db < 2; ++db) {
        st4<T>(dst + C + 16 * db + 4 * lg, dk[u][db][0] * scale, dk[u][db][1] * scale, dk[u][db][2] * scale,
               dk[u][db][3] * scale);
        st4<T>(dst + 2 * C + 16 * db + 4 * lg, dv[u][db][0], dv[u][db][1], dv[u][db][2], dv[u][db][3]);
      }
    }
  }
}

// ---------------- blockify / deblockify ----------------
// image x[B][Hg*bs][Wg*bs][C] (NHWC) <-> blocked tokens y[B][Hg*Wg][bs*bs][C]
// (timm nest blockify: block index gh*Wg + gw, token bh*bs + bw).  Forward adds
// the level's positional embedding pos[Hg*Wg][bs*bs][C] (fp32) when given.
template <typename T>
__global__ void nest_blockify_kernel(int B, int Hg, int Wg, int bs, int C, const T* __restrict__ x,
                                     const float* __restrict__ pos, T* __restrict__ y, int inverse) {
  constexpr int EPC = 16 / (int)sizeof(T);
  const int cpr = C / EPC;
  const size_t total = (size_t)B * Hg * bs * Wg * bs * cpr;
  for (size_t q = blockIdx.x * (size_t)blockDim.x + threadIdx.x; q < total; q += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(q % cpr);
    size_t pix = q / cpr;                       // image pixel index (b, h, w)
    const int W = Wg * bs, Hh = Hg * bs;
    const int wq = (int)(pix % W);
    const size_t r = pix / W;
    const int hq = (int)(r % Hh);
    const int b = (int)(r / Hh);
    const int gh = hq / bs, bh = hq - gh * bs, gw = wq / bs, bw = wq - gw * bs;
    const size_t blk = (size_t)gh * Wg + gw, tok = (size_t)bh * bs + bw;
    const size_t trow = ((size_t)b * Hg * Wg + blk) * bs * bs + tok;
    if (!inverse) {
      uint4 v = ldg16(x + pix * C + c * EPC);
      if (pos) {
        float f[EPC];
        Chunk<T>::unpack(v, f);
        const float* pp = pos + (blk * bs * bs + tok) * C + c * EPC;
#pragma unroll
        for (int j = 0; j < EPC; ++j) f[j] += pp[j];
        v = Chunk<T>::pack(f);
      }
      stg16(y + trow * C + c * EPC, v);
    } else {
      stg16(y + pix * C + c * EPC, ldg16(x + trow * C + c * EPC));
    }
  }
}

// positional-embedding gradient: dpos[t][c] = sum_b dy[b][t][c] (fp32 out)
template <typename T>
__global__ void nest_pos_grad_kernel(int B, int TN, int C, const T* __restrict__ dy, float* __restrict__ dpos) {
  const size_t total = (size_t)TN * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += to_f(dy[(size_t)b * total + e]);
    dpos[e] = s;
  }
}

// ---------------- 3x3 / 2 max pool, padding 1 (ConvPool) ----------------
// x[B][H][W][C] -> y[B][Ho][Wo][C], idx = window tap (0..8) of the maximum
// (first maximum in row-major tap order, as torch's max_pool2d).
template <typename T>
__global__ void nest_maxpool_fwd_kernel(int B, int H, int W, int C, const T* __restrict__ x, T* __restrict__ y,
                                        uint8_t* __restrict__ idx) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const size_t total = (size_t)B * Ho * Wo * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    size_t r = e / C;
    const int wo = (int)(r % Wo);
    r /= Wo;
    const int ho = (int)(r % Ho);
    const int b = (int)(r / Ho);
    float best = 0.f;
    int bi = -1;
    for (int kh = 0; kh < 3; ++kh) {
      const int hi = 2 * ho - 1 + kh;
      if ((unsigned)hi >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int wi = 2 * wo - 1 + kw;
        if ((unsigned)wi >= (unsigned)W) continue;
        const float v = to_f(x[(((size_t)b * H + hi) * W + wi) * C + c]);
        if (bi < 0 || v > best) { best = v; bi = kh * 3 + kw; }
      }
    }
    y[e] = from_f<T>(best);
    idx[e] = (uint8_t)bi;
  }
}
// dx[b][h][w][c] = sum of dy over the pooled outputs whose window's maximum is (h, w)
template <typename T>
__global__ void nest_maxpool_bwd_kernel(int B, int H, int W, int C, const T* __restrict__ dy,
                                        const uint8_t* __restrict__ idx, T* __restrict__ dx) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const size_t total = (size_t)B * H * W * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    size_t r = e / C;
    const int wi = (int)(r % W);
    r /= W;
    const int hi = (int)(r % H);
    const int b = (int)(r / H);
    float s = 0.f;
    // the pooled rows whose window 2ho-1 .. 2ho+1 holds hi: (hi+1)/2 and the one above
    for (int a = 0; a < 2; ++a) {
      const int ho = (hi + 1) / 2 - a;
      if (ho < 0 || ho >= Ho || 2 * ho - 1 > hi || 2 * ho + 1 < hi) continue;
      for (int bb = 0; bb < 2; ++bb) {
        const int wo = (wi + 1) / 2 - bb;
        if (wo < 0 || wo >= Wo || 2 * wo - 1 > wi || 2 * wo + 1 < wi) continue;
        const size_t o = (((size_t)b * Ho + ho) * Wo + wo) * C + c;
        const int tap = (hi - (2 * ho - 1)) * 3 + (wi - (2 * wo - 1));
        if (idx[o] == tap) s += to_f(dy[o]);
      }
    }
    dx[e] = from_f<T>(s);
  }
}

// ---------------- patch embedding im2col ----------------
// 4x4 / 4 patches of the normalised image, rows in BLOCKED token order of
// level 0 (block (gh, gw) of the Hp x Wp patch grid, token (bh, bw)), so the
// patch GEMM writes level 0's input directly.  K = 48 = (c, kh, kw) as the
// conv weight [96][3][4][4] flattens; from the uint8 1-channel upload the
// three channels are the same normalised pixel (PretrainDataModule.py:167-171).
template <typename T>
__global__ void nest_patch_prep_kernel(int B, int Himg, int Wimg, int bs, const float* __restrict__ x,
                                       const uint8_t* __restrict__ xu8, float mean, float inv_std,
                                       T* __restrict__ out) {
  const int Hp = Himg / 4, Wp = Wimg / 4;
  const int Hg = Hp / bs, Wg = Wp / bs;
  const size_t total = (size_t)B * Hp * Wp * 48;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int k = (int)(e % 48);
    const size_t trow = e / 48;                               // blocked token row
    const int tok = (int)(trow % ((size_t)bs * bs));
    size_t r = trow / ((size_t)bs * bs);
    const int blk = (int)(r % ((size_t)Hg * Wg));
    const int b = (int)(r / ((size_t)Hg * Wg));
    const int gh = blk / Wg, gw = blk - gh * Wg, bh = tok / bs, bw = tok - bh * bs;
    const int ph = gh * bs + bh, pw = gw * bs + bw;           // patch coordinates
    const int c = k / 16, kh = (k >> 2) & 3, kw = k & 3;
    const int hi = 4 * ph + kh, wi = 4 * pw + kw;
    float v;
    if (xu8) v = ((float)xu8[((size_t)b * Himg + hi) * Wimg + wi] - mean) * inv_std;
    else v = x[(((size_t)b * 3 + c) * Himg + hi) * Wimg + wi];
    out[e] = from_f<T>(v);
  }
}

// ---------------- small helpers ----------------
// y[m][n] += bias[n]
template <typename T>
__global__ void nest_add_bias_kernel(size_t M, int N, T* __restrict__ y, const float* __restrict__ bias) {
  const size_t total = M * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x)
    y[e] = from_f<T>(to_f(y[e]) + bias[e % N]);
}
// dst[n][d*H + h] <-> dst[n][h*Dh + d]: the proj weight's input columns (fp32
// master -> compute dtype), or (inverse) its gradient back to timm's order
template <typename TI, typename TO>
__global__ void nest_permute_cols_kernel(int Nr, int H, int Dh, const TI* __restrict__ src, TO* __restrict__ dst,
                                         int inverse) {
  const int C = H * Dh;
  const size_t total = (size_t)Nr * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const size_t n = e / C;
    const int j = (int)(e - n * C);      // head-major column h*Dh + d
    const int h = j / Dh, d = j - h * Dh;
    const int t = d * H + h;             // timm column
    if (!inverse) dst[e] = from_f<TO>(to_f(src[n * C + t]));
    else dst[n * C + t] = from_f<TO>(to_f(src[e]));
  }
}
// DropPath on a residual branch: x[m][n] += s[m / rows] * y[m][n] (s = 0 or 1/(1-p))
// mode 1 (backward): y[m][n] = s[m / rows] * x[m][n]
template <typename T>
__global__ void nest_rowscale_kernel(size_t M, int N, int rows, const float* __restrict__ s, T* __restrict__ x,
                                     T* __restrict__ y, int mode) {
  const size_t total = M * N;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const float k = s[(e / N) / rows];
    if (mode == 0) x[e] = from_f<T>(to_f(x[e]) + k * to_f(y[e]));
    else y[e] = from_f<T>(k * to_f(x[e]));
  }
}
// dy[b*HW + p][c] = dfeat[b][c] * inv (global average pool backward)
template <typename T>
__global__ void nest_bcast_kernel(int B, int HW, int C, const float* __restrict__ dfeat, float inv,
                                  T* __restrict__ dy) {
  const size_t total = (size_t)B * HW * C;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(e % C);
    const size_t b = e / ((size_t)HW * C);
    dy[e] = from_f<T>(dfeat[b * C + c] * inv);
  }
}

static inline dim3 ew(size_t n) {
  size_t b = (n + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

}  // namespace vlp

using namespace vlp;

#define NEST_DT(dtype, F, ...)                  \
  do {                                          \
    if ((dtype) == VLP_BF16) F<bf16>(__VA_ARGS__); \
    else F<float>(__VA_ARGS__);                 \
  } while (0)

template <typename T>
static void attn_fwd_t(int BT, int H, int N, const void* qkv, void* out, float* lse, float scale, hipStream_t st) {
  hipLaunchKernelGGL(nest_attn_fwd_kernel<T>, dim3(((N + kQBlock - 1) / kQBlock) * H * BT), dim3(256), 0, st, BT, H, N,
                     (const T*)qkv, (T*)out, lse, scale * 1.4426950408889634f);
}
VLP_EXPORT int vlp_nest_attn_fwd(int dtype, int BT, int H, int N, int dh, const void* qkv, void* out, float* lse,
                                 float scale, void* stream) {
  if (dh != kDh || BT < 1 || H < 1 || N < 1 || (long long)((N + 63) / 64) * H * BT >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  NEST_DT(dtype, attn_fwd_t, BT, H, N, qkv, out, lse, scale, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void attn_bwd_t(int BT, int H, int N, const void* qkv, const void* out, const void* dout, const float* lse,
                       float* delta, void* dqkv, float scale, hipStream_t st) {
  const size_t rows = (size_t)BT * N * H;
  hipLaunchKernelGGL(nest_attn_delta_kernel<T>, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, st, BT, H, N,
                     (const T*)out, (const T*)dout, delta);
  const dim3 gq(((N + kQBlock - 1) / kQBlock) * H * BT), gk(((N + 63) / 64) * H * BT);
  const float sl2 = scale * 1.4426950408889634f;
  hipLaunchKernelGGL(nest_attn_bwd_dq_kernel<T>, gq, dim3(256), 0, st, BT, H, N, (const T*)qkv, (const T*)dout, lse,
                     (const float*)delta, (T*)dqkv, sl2, scale);
  hipLaunchKernelGGL(nest_attn_bwd_dkdv_kernel<T>, gk, dim3(256), 0, st, BT, H, N, (const T*)qkv, (const T*)dout, lse,
                     (const float*)delta, (T*)dqkv, sl2, scale);
}
VLP_EXPORT int vlp_nest_attn_bwd(int dtype, int BT, int H, int N, int dh, const void* qkv, const void* out,
                                 const void* dout, const float* lse, float* delta, void* dqkv, float scale,
                                 void* stream) {
  if (dh != kDh || BT < 1 || H < 1 || N < 1 || (long long)((N + 63) / 64) * H * BT >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  NEST_DT(dtype, attn_bwd_t, BT, H, N, qkv, out, dout, lse, delta, dqkv, scale, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void blockify_t(int B, int Hg, int Wg, int bs, int C, const void* x, const float* pos, void* y, int inv,
                       hipStream_t st) {
  const size_t n = (size_t)B * Hg * bs * Wg * bs * (C / (16 / (int)sizeof(T)));
  hipLaunchKernelGGL(nest_blockify_kernel<T>, ew(n), dim3(256), 0, st, B, Hg, Wg, bs, C, (const T*)x, pos, (T*)y,
                     inv);
}
VLP_EXPORT int vlp_nest_blockify(int dtype, int B, int Hg, int Wg, int bs, int C, const void* x, const float* pos,
                                 void* y, int inverse, void* stream) {
  if (C % (dtype == VLP_BF16 ? 8 : 4) || (inverse && pos)) return (int)hipErrorInvalidValue;
  NEST_DT(dtype, blockify_t, B, Hg, Wg, bs, C, x, pos, y, inverse, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void pos_grad_t(int B, int TN, int C, const void* dy, float* dpos, hipStream_t st) {
  hipLaunchKernelGGL(nest_pos_grad_kernel<T>, ew((size_t)TN * C), dim3(256), 0, st, B, TN, C, (const T*)dy, dpos);
}
VLP_EXPORT int vlp_nest_pos_grad(int dtype, int B, int TN, int C, const void* dy, float* dpos, void* stream) {
  NEST_DT(dtype, pos_grad_t, B, TN, C, dy, dpos, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void mp_fwd_t(int B, int H, int W, int C, const void* x, void* y, uint8_t* idx, hipStream_t st) {
  const size_t n = (size_t)B * ((H + 1) / 2) * ((W + 1) / 2) * C;
  hipLaunchKernelGGL(nest_maxpool_fwd_kernel<T>, ew(n), dim3(256), 0, st, B, H, W, C, (const T*)x, (T*)y, idx);
}
VLP_EXPORT int vlp_nest_maxpool_fwd(int dtype, int B, int H, int W, int C, const void* x, void* y, uint8_t* idx,
                                    void* stream) {
  NEST_DT(dtype, mp_fwd_t, B, H, W, C, x, y, idx, (hipStream_t)stream);
  return (int)hipGetLastError();
}
template <typename T>
static void mp_bwd_t(int B, int H, int W, int C, const void* dy, const uint8_t* idx, void* dx, hipStream_t st) {
  hipLaunchKernelGGL(nest_maxpool_bwd_kernel<T>, ew((size_t)B * H * W * C), dim3(256), 0, st, B, H, W, C,
                     (const T*)dy, idx, (T*)dx);
}
VLP_EXPORT int vlp_nest_maxpool_bwd(int dtype, int B, int H, int W, int C, const void* dy, const uint8_t* idx,
                                    void* dx, void* stream) {
  NEST_DT(dtype, mp_bwd_t, B, H, W, C, dy, idx, dx, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void patch_t(int B, int H, int W, int bs, const float* x, const uint8_t* xu8, float mean, float std_,
                    void* out, hipStream_t st) {
  hipLaunchKernelGGL(nest_patch_prep_kernel<T>, ew((size_t)B * (H / 4) * (W / 4) * 48), dim3(256), 0, st, B, H, W,
                     bs, x, xu8, mean, 1.f / std_, (T*)out);
}
VLP_EXPORT int vlp_nest_patch_prep(int dtype, int B, int H, int W, int bs, const float* x, const uint8_t* x_u8,
                                   float mean, float std_, void* out, void* stream) {
  if (H % 4 || W % 4 || (H / 4) % bs || (W / 4) % bs || (!x) == (!x_u8)) return (int)hipErrorInvalidValue;
  NEST_DT(dtype, patch_t, B, H, W, bs, x, x_u8, mean, std_, out, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void bias_t(long long M, int N, void* y, const float* b, hipStream_t st) {
  hipLaunchKernelGGL(nest_add_bias_kernel<T>, ew((size_t)M * N), dim3(256), 0, st, (size_t)M, N, (T*)y, b);
}
VLP_EXPORT int vlp_nest_add_bias(int dtype, long long M, int N, void* y, const float* bias, void* stream) {
  NEST_DT(dtype, bias_t, M, N, y, bias, (hipStream_t)stream);
  return (int)hipGetLastError();
}

VLP_EXPORT int vlp_nest_permute_cols(int dtype_out, int Nr, int H, int Dh, const float* src, void* dst,
                                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const dim3 g = ew((size_t)Nr * H * Dh);
  if (dtype_out == VLP_BF16)
    hipLaunchKernelGGL((nest_permute_cols_kernel<float, bf16>), g, dim3(256), 0, st, Nr, H, Dh, src, (bf16*)dst, 0);
  else
    hipLaunchKernelGGL((nest_permute_cols_kernel<float, float>), g, dim3(256), 0, st, Nr, H, Dh, src, (float*)dst,
                       0);
  return (int)hipGetLastError();
}
VLP_EXPORT int vlp_nest_unpermute_cols(int Nr, int H, int Dh, const float* src, float* dst, void* stream) {
  hipLaunchKernelGGL((nest_permute_cols_kernel<float, float>), ew((size_t)Nr * H * Dh), dim3(256), 0,
                     (hipStream_t)stream, Nr, H, Dh, src, dst, 1);
  return (int)hipGetLastError();
}

template <typename T>
static void rowscale_t(long long M, int N, int rows, const float* s, void* x, void* y, int mode, hipStream_t st) {
  hipLaunchKernelGGL(nest_rowscale_kernel<T>, ew((size_t)M * N), dim3(256), 0, st, (size_t)M, N, rows, s, (T*)x,
                     (T*)y, mode);
}
VLP_EXPORT int vlp_nest_rowscale(int dtype, long long M, int N, int rows, const float* s, void* x, void* y, int mode,
                                 void* stream) {
  NEST_DT(dtype, rowscale_t, M, N, rows, s, x, y, mode, (hipStream_t)stream);
  return (int)hipGetLastError();
}

template <typename T>
static void bcast_t(int B, int HW, int C, const float* dfeat, float inv, void* dy, hipStream_t st) {
  hipLaunchKernelGGL(nest_bcast_kernel<T>, ew((size_t)B * HW * C), dim3(256), 0, st, B, HW, C, dfeat, inv, (T*)dy);
}
VLP_EXPORT int vlp_nest_bcast(int dtype, int B, int HW, int C, const float* dfeat, float inv, void* dy,
                              void* stream) {
  NEST_DT(dtype, bcast_t, B, HW, C, dfeat, inv, dy, (hipStream_t)stream);
  return (int)hipGetLastError();
}
