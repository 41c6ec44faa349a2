// MFMA GEMM engine for gfx950 (CDNA4), shared by every contraction on the
// hot path: implicit-GEMM convolutions (fwd / dgrad / wgrad), TinyBERT linear
// layers, and the CLIP projections.
//
//   C[m][n] = sum_k A(m, k) * B(n, k)
//
// A and B are supplied by *loader* functors that return 16-byte chunks
// (8 bf16 / 4 fp32 values).  A loader is either
//   K-contiguous  (kKContig = true):  chunk = A(m, k .. k+EPC-1)
//   MN-contiguous (kKContig = false): chunk = A(m .. m+EPC-1, k)
// so NHWC activations, torch [out][in] weights, and "transposed" operands
// (wgrad / weight-gradient products) all stream with 16-B coalesced loads and
// no explicit transpose pass.  Chunks are staged through a double-buffered,
// XOR-swizzled LDS image; MN-contiguous bf16 images are read with the gfx950
// ds_read_b64_tr_b16 transposing read.
//
// bf16: v_mfma_f32_16x16x32_bf16, BK = 64.  fp32 (parity mode):
// v_mfma_f32_16x16x4_f32 (exact fp32 fma chain), BK = 32.  In both cases one
// LDS row is 128 bytes, so the LDS geometry and swizzles are identical.
//
// The MFMA is issued "swapped" (MFMA-A = B tile, MFMA-B = A tile) so each lane
// owns four consecutive output COLUMNS of one row: epilogues store 8/16-byte
// vectors along the NHWC channel dimension.
//
// 4 waves (256 threads) per workgroup in a WGM x WGN wave grid; the grid is
// remapped so that consecutive tile ids share an XCD (L2 reuse of the A panel).
// Split-K over grid.y for reductions over pixels (weight gradients).
#pragma once
#include <mutex>
#include <type_traits>
#include <utility>
#include <vector>
#include "common.h"

#ifndef VLP_BIG_SCHED   // gemm_big_kernel instruction interleaving (0: compiler order)
#define VLP_BIG_SCHED 0
#endif
#ifndef VLP_BIG_PRIO    // gemm_big_kernel: s_setprio 1 for waves 4-7
#define VLP_BIG_PRIO 0
#endif

namespace vlp {

typedef __attribute__((address_space(3))) v4bf lds_v4bf;

struct GemmShape {
  int M, N, K;
  int kchunk;   // K range per split (multiple of BK); == K rounded up when no split
  int tiles_m, tiles_n;
  int xsplit;   // 1: split-K grid is 1-D and every split's tiles share one XCD
  int dbg;      // reserved (0)
  int nsplit;   // K-splits (bk / big kernels: 1-D grid of nsplit * tiles)
};

// ---------------- LDS image addressing (bytes) ----------------
// K-contig image: [rows][128 B]; 16-B chunk c of row r -> c ^ ((r>>1)&7).
__device__ __forceinline__ int kc_off(int r, int c) {
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}
// MN-contig image: [k-rows][RB bytes]; 32-B blocks XOR-swizzled by k.
template <int RB>
__device__ __forceinline__ int mn_off(int k, int byte_in_row) {
  const int sw = (RB >= 256) ? (k & 7) : ((k >> 1) & 3);
  return k * RB + ((((byte_in_row >> 5) ^ sw) << 5) | (byte_in_row & 31));
}

// Blocked MN-contig image (direct staging): 1-KiB blocks of 8 k-rows x 8
// 16-B chunks, block (k>>3, c>>3) at ((k>>3)*CPB + (c>>3)) KiB (CPB = chunk
// blocks per k-row = MN/64); inside a block, chunk c&7 of row k&7 sits at
// 16*((c&7) ^ h(k)), h = bit1(k)<<1 | bit3(k)<<2: the two 32-lane halves of a
// ds_read_b64_tr_b16 fragment read (rows 32s+8g+q, chunk pair c0, c0+1)
// land on 32 distinct 8-B bank slots.  Each 1-KiB block is ONE wave-wide
// LDS-DMA of 8 rows x 128 B: 8 full cache lines per load instruction.
__device__ __forceinline__ int mn8_h(int k) { return (((k >> 1) & 1) << 1) | (((k >> 3) & 1) << 2); }
template <int CPB>
__device__ __forceinline__ int mn8_off(int k, int mn) {
  const int c = mn >> 3;
  return ((k >> 3) * CPB + (c >> 3)) * 1024 + (k & 7) * 128 + (((c & 7) ^ mn8_h(k)) << 4) +
         ((mn & 4) << 1);
}

// Sum over each 16-lane DPP row (the 16 rows of an MFMA output block);
// lane 15 of the row receives the total.  Four row_shr DPP adds: VALU only,
// where __shfl_xor would issue ds_bpermute LDS traffic.
__device__ __forceinline__ float row16_sum(float x) {
  int v = __builtin_bit_cast(int, x);
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
  v = __builtin_bit_cast(int, x);
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
  v = __builtin_bit_cast(int, x);
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
  v = __builtin_bit_cast(int, x);
  x += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
  return x;
}

template <typename T, int BM, bool KC>
struct TileGeom {
  static constexpr int EPC = Elem<T>::EPC;
  static constexpr int BK = Elem<T>::BK;
  static constexpr int BYTES = BM * 128;            // one stage of this operand
  static constexpr int NCH = BYTES / 16 / 256;      // chunks per thread
  static constexpr int RB = BM * (int)sizeof(T);    // MN image row bytes
  static constexpr int CPR = RB / 16;               // MN chunks per k-row
  static_assert(NCH >= 1, "tile too small");
  static_assert(KC || (256 % CPR == 0), "MN tile geometry");
};

// Per-thread staging of one operand tile into registers and then LDS.
template <typename T, int BM, class L>
struct Stager {
  using G = TileGeom<T, BM, L::kKContig>;
  typename L::State st[L::kKContig ? G::NCH : 1];
  uint4 r[G::NCH];

  __device__ __forceinline__ void init(const L& ld, int row0) {
    const int t = threadIdx.x;
    if constexpr (L::kKContig) {
#pragma unroll
      for (int i = 0; i < G::NCH; ++i) st[i] = ld.fixed(row0 + (t >> 3) + 32 * i);
    } else {
      st[0] = ld.fixed(row0 + (t % G::CPR) * G::EPC);
    }
  }
  __device__ __forceinline__ void load(const L& ld, int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < G::NCH; ++i) {
      if constexpr (L::kKContig) {
        r[i] = ld.load(st[i], k0 + (t & 7) * G::EPC);
      } else {
        r[i] = ld.load(st[0], k0 + t / G::CPR + (256 / G::CPR) * i);
      }
    }
  }
  __device__ __forceinline__ void store(char* lds) const {
    const int t = threadIdx.x;
#pragma unroll
    for (int i = 0; i < G::NCH; ++i) {
      int off;
      if constexpr (L::kKContig) {
        off = kc_off((t >> 3) + 32 * i, t & 7);
      } else {
        off = mn_off<G::RB>(t / G::CPR + (256 / G::CPR) * i, (t % G::CPR) * 16);
      }
      *reinterpret_cast<uint4*>(lds + off) = r[i];
    }
  }
};

// ---------------- direct-to-LDS staging (bf16) ----------------
// Loaders that can name the global address of a chunk (kDirect = true) are
// staged with global_load_lds_dwordx4: each wave-instruction writes 1 KiB of
// LDS lane-linearly, so lane L of instruction i fills PHYSICAL chunk
// q = (wave*NI + i)*64 + L and fetches the LOGICAL chunk that the XOR swizzle
// places there (the swizzles are involutions).  No staging registers, no
// ds_write pass; the loads of tile t+1 fly while tile t is multiplied.
//
// Direct loaders are INCREMENTAL (profiling showed ~8 VALU per MFMA when every
// chunk address was rebuilt from scratch each K-step):
//   DState start(int coord, int koff, int kb)  once per chunk: coord = the
//        operand row (K-contig) or first row of the chunk (MN-contig), koff = the
//        chunk's k offset inside a K-step, kb = the first K-step's base
//   Step step(int k0)                           once per K-step per wave: the
//        k0-only context (conv tap, channel offset, K bound) -- wave-uniform,
//        so it lives in scalar registers and is shared by all NI chunks
//   const void* next(DState&, const Step&)     per chunk per K-step: the
//        chunk's address or the zero page (branch-free select); advances state
static __device__ uint4 g_zero16;
__device__ __forceinline__ const void* zero_page() { return &g_zero16; }

template <class L, class = void> struct DirectTrait { static constexpr bool value = false; };
template <class E, class = void> struct StageTrait { static constexpr bool value = false; };
template <class E> struct StageTrait<E, std::void_t<decltype(E::kStage)>> {
  static constexpr bool value = E::kStage;
};
// operands a row-chunk epilogue fetches ahead of its row8() call (16-B chunks)
struct RowPre { uint4 u[3]; };
// row-chunk epilogues may declare their own prefetch record (E::Pre) and a third
// per-column statistic (E::kStats3, E::stat3, row8r3 instead of row8r)
template <class E, class = void> struct PreTypeTrait { using type = RowPre; };
template <class E> struct PreTypeTrait<E, std::void_t<typename E::Pre>> { using type = typename E::Pre; };
template <class E, class = void> struct Stat3Trait { static constexpr bool value = false; };
template <class E> struct Stat3Trait<E, std::void_t<decltype(E::kStats3)>> { static constexpr bool value = E::kStats3; };
// split-K epilogues that write their own partial slab (no atomics): the kernel
// hands the epilogue its split index via at_split(split)
template <class E, class = void> struct SplitTrait { static constexpr bool value = false; };
template <class E> struct SplitTrait<E, std::void_t<decltype(E::kSplitOut)>> {
  static constexpr bool value = E::kSplitOut;
};
// A loader's per-chunk byte offset, computed once per tile, made opaque to the
// compiler: otherwise it re-associates offset + per-K-step delta back into the
// pixel coordinates and recomputes (v_mul_lo_u32 + v_mad_u64_u32 per chunk and
// K-step) instead of keeping one VGPR per chunk (VLP_OPAQUE_BASE = 0: as before)
#ifndef VLP_OPAQUE_BASE
#define VLP_OPAQUE_BASE 1
#endif
__device__ __forceinline__ unsigned opaque_base(unsigned v) {
#if VLP_OPAQUE_BASE
  asm volatile("" : "+v"(v));
#endif
  return v;
}
// K-step order: a loader with kKPerm maps the logical K offset of a 64-deep
// step to the physical one (kperm); the buffer-protocol kernels apply the SAME
// map to both operands, so the product is unchanged up to fp32 summation order
template <class L, class = void> struct KPermTrait { static constexpr bool value = false; };
template <class L> struct KPermTrait<L, std::void_t<decltype(L::kKPerm)>> { static constexpr bool value = L::kKPerm; };
template <class L>
__device__ __forceinline__ int kperm_of(const L& l, int k) {
  if constexpr (KPermTrait<L>::value) return l.kperm(k);
  else return k;
}
template <class E, class = void> struct RowTrait { static constexpr bool value = false; };
template <class E> struct RowTrait<E, std::void_t<decltype(E::kRow)>> {
  static constexpr bool value = E::kRow;
};
template <class L> struct DirectTrait<L, std::void_t<decltype(L::kDirect)>> {
  static constexpr bool value = L::kDirect;
};
// row-chunk epilogues: per-channel coefficient arrays (E::kCoefs, E::coef(k))
// and how many row chunks of operands to keep in flight (E::kPreDepth)
// row-chunk epilogues that add a per-column bias (E::bias, may be null) to the raw
// accumulators before they are staged as bf16 (one rounding of acc + bias)
template <class E, class = void> struct StageBiasTrait { static constexpr bool value = false; };
template <class E> struct StageBiasTrait<E, std::void_t<decltype(E::kStageBias)>> {
  static constexpr bool value = E::kStageBias;
};
template <class E, class = void> struct CoefTrait { static constexpr int value = 0; };
template <class E> struct CoefTrait<E, std::void_t<decltype(E::kCoefs)>> { static constexpr int value = E::kCoefs; };
// row epilogues whose operand u[E::kLdsSlot] (a [rows][C] bf16 tensor, E::lds_operand())
// a kernel may stage into LDS as the tile's [BM][BN] image ahead of the epilogue
template <class E, class = void> struct LdsSlotTrait { static constexpr int value = -1; };
template <class E> struct LdsSlotTrait<E, std::void_t<decltype(E::kLdsSlot)>> {
  static constexpr int value = E::kLdsSlot;
};
template <class E, class = void> struct PreDepthTrait { static constexpr int value = 8; };
template <class E> struct PreDepthTrait<E, std::void_t<decltype(E::kPreDepth)>> {
  static constexpr int value = E::kPreDepth;
};
// a thread's 8 coefficients held in registers, indexed by global column
// (c[col + j] = p[j]) like the global / LDS coefficient pointers
struct RegCoef {
  const float* p; int base;
  __device__ __forceinline__ float operator[](int i) const { return p[i - base]; }
};

template <typename T, int BM, class L>
struct GStager {
  using G = TileGeom<T, BM, L::kKContig>;
  static constexpr int NI = G::NCH;
  typename L::DState st[NI];

  __device__ __forceinline__ void init(const L& ld, int row0, int kb) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (w * NI + i) * 64 + lane;
      const int r = q >> 3, p = q & 7;
      const int c = p ^ ((r >> 1) & 7);
      st[i] = ld.start(row0 + r, c * G::EPC, kb);
    }
  }
  __device__ __forceinline__ void issue(const L& ld, int k0, char* lds) {
    const int w = threadIdx.x >> 6;
    const auto stp = ld.step(k0);   // K-step-uniform context (scalar registers)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const void* p = ld.next(st[i], stp);
      __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)(lds + (w * NI + i) * 1024),
                                       16, 0, 0);
    }
  }
};

// Uniform staging interface: register staging (any loader, fp32 parity mode,
// transforming loaders) or direct-to-LDS (bf16 + kDirect loaders).
// (the 2-stage kernel stages MN-contig operands through registers; direct
// MN staging lives in the multi-stage kernel)
template <typename T, int BM, class L,
          bool DIRECT = (sizeof(T) == 2) && DirectTrait<L>::value && L::kKContig>
struct OpStager;
template <typename T, int BM, class L>
struct OpStager<T, BM, L, false> {
  Stager<T, BM, L> s;
  __device__ __forceinline__ void init(const L& ld, int row0, int) { s.init(ld, row0); }
  __device__ __forceinline__ void prefetch(const L& ld, int k0, char*) { s.load(ld, k0); }
  __device__ __forceinline__ void commit(char* lds) const { s.store(lds); }
};
template <typename T, int BM, class L>
struct OpStager<T, BM, L, true> {
  GStager<T, BM, L> s;
  __device__ __forceinline__ void init(const L& ld, int row0, int kb) { s.init(ld, row0, kb); }
  __device__ __forceinline__ void prefetch(const L& ld, int k0, char* lds) { s.issue(ld, k0, lds); }
  __device__ __forceinline__ void commit(char*) const {}
};

// ---------------- fragment reads ----------------
// bf16 fragment for MFMA 16x16x32, k-step s (0/1) within a BK=64 stage.
// Lane l = 16g + i holds operand row (rb + i) at k = 32s + 8g + (0..7): a
// k-permutation shared by both operands, chosen so a K-contig fragment is ONE
// 16-B chunk (ds_read_b128, conflict-free under the kc_off swizzle) and an
// MN-contig fragment is two ds_read_b64_tr_b16 (k-rows 32s+8g+q, +4).
// MNCOL: MN-contig image in the blocked layout of the direct MN stager
// (GStagerN<..., false>, mn8_off): 1-KiB blocks of 8 k-rows x 8 chunks.
template <bool KC, int RB, bool MNCOL = false>
__device__ __forceinline__ v8bf frag_bf16(const char* lds, int rb, int s) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, g = l >> 4;
  if constexpr (KC) {
    return *reinterpret_cast<const v8bf*>(lds + kc_off(rb + i, 4 * s + g));
  } else {
    v4bf lo, hi;
    const int q = i >> 2, p = i & 3;
    const int k1 = 32 * s + 8 * g + q;
    if constexpr (MNCOL) {
      const int mn = rb + 4 * p;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(lds + mn8_off<RB / 128>(k1, mn)));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(lds + mn8_off<RB / 128>(k1 + 4, mn)));
    } else {
      const int by = (rb + 4 * p) * 2;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(lds + mn_off<RB>(k1, by)));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(lds + mn_off<RB>(k1 + 4, by)));
    }
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// MN-contig (blocked image) fragment through inline-asm transposing reads.
// hipcc treats ds_read_b64_tr_b16 as possibly aliasing an in-flight LDS-DMA
// and drains vmcnt(0) in front of it, which would empty a multi-tile
// prefetch ring every K-step; asm reads are invisible to that analysis, so
// the caller owns the wait: asm_lds_wait() before the first consumer.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(unsigned long long)(const __attribute__((address_space(3))) char*)p;
}
template <int RB>
__device__ __forceinline__ v8bf frag_tr_asm(const char* lds, int rb, int s) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, g = l >> 4;
  const int q = i >> 2, p = i & 3;
  const int k1 = 32 * s + 8 * g + q;
  const int mn = rb + 4 * p;
  v4bf lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(lds_addr(lds + mn8_off<RB / 128>(k1, mn))));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(lds_addr(lds + mn8_off<RB / 128>(k1 + 4, mn))));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ void asm_lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// The same fragment from a per-(slot, fragment) lane address: the k-substep
// (+4*CPB KiB) and the upper k-half (+512 B) are immediate offsets of the
// instruction, so a wave keeps one address VGPR per fragment and slot instead
// of one per read (mn8_off is additive in both: neither changes the swizzle).
template <int RB>
__device__ __forceinline__ unsigned mn_frag_base(const char* lds, int rb) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, g = l >> 4;
  const int q = i >> 2, p = i & 3;
  return lds_addr(lds + mn8_off<RB / 128>(8 * g + q, rb + 4 * p));
}
template <int OFF>
__device__ __forceinline__ v8bf frag_tr_at(unsigned base) {
  v4bf lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(base), "n"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(base), "n"(OFF + 512));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// fragment j of a wave's column of 16-row fragments: fragments j and j + 4 are
// 1 KiB apart (the next 64-row block, same swizzle), so 4 base addresses serve
// any number of fragments
template <int RB, int J>
__device__ __forceinline__ v8bf frag_tr_sub(unsigned base, int s) {
  constexpr int S1 = 4 * (RB / 128) * 1024;
  constexpr int OJ = (J >> 2) * 1024;
  return s == 0 ? frag_tr_at<OJ>(base) : frag_tr_at<S1 + OJ>(base);
}
template <int I, int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (I < N) {
    fn(std::integral_constant<int, I>{});
    static_for<I + 1, N>(fn);
  }
}
template <bool KC, int RB>
__device__ __forceinline__ v8bf frag_big(const char* lds, int rb, int s) {
  if constexpr (KC) return frag_bf16<true, RB, true>(lds, rb, s);
  else return frag_tr_asm<RB>(lds, rb, s);
}

// fp32 fragment for 4 x MFMA 16x16x4f32 over a 16-k sub-step s (0/1) of BK=32.
// Lane l = 16g + i holds row (rb + i) at k = 16s + 4g + j in element j (MFMA j).
template <bool KC, int RB>
__device__ __forceinline__ v4f frag_f32(const char* lds, int rb, int s) {
  const int l = threadIdx.x & 63;
  const int i = l & 15, g = l >> 4;
  if constexpr (KC) {
    return *reinterpret_cast<const v4f*>(lds + kc_off(rb + i, 4 * s + g));
  } else {
    v4f v;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      v[j] = *reinterpret_cast<const float*>(lds + mn_off<RB>(16 * s + 4 * g + j, (rb + i) * 4));
    return v;
  }
}

// ---------------- the kernel ----------------
// Epilogue contract:
//   static constexpr bool kStats;  // accumulate two per-column sums
//   __device__ void operator()(int row, int col, v4f v, v4f& s1, v4f& s2) const;
//      called only for row < M (col < N, N % 4 == 0); s1/s2 start at 0.
//   double* stat1, *stat2;          // per-column sums (only when kStats)
template <typename T, int BM, int BN, int WGM, class LA, class LB, class EP>
__global__ void __launch_bounds__(256)
gemm_kernel(GemmShape sh, LA la, LB lb, EP ep) {
  constexpr int WGN = 4 / WGM;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;   // wave tile
  constexpr int MB = WTM / 16, NB = WTN / 16;
  constexpr int BK = Elem<T>::BK;
  using GA = TileGeom<T, BM, LA::kKContig>;
  using GB = TileGeom<T, BN, LB::kKContig>;
  constexpr int STAGE = GA::BYTES + GB::BYTES;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  // XCD-aware bijective remap of the tile id (consecutive ids -> same XCD).
  const int nwg = sh.tiles_m * sh.tiles_n;
  const int bid = blockIdx.x;
  int wid = bid;
  if (nwg >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = nwg >> 3, rr = nwg & 7;
    wid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int tm = wid / sh.tiles_n, tn = wid - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;

  const int kb = blockIdx.y * sh.kchunk;
  int ke = kb + sh.kchunk;
  if (ke > sh.K) ke = sh.K;
  const int nk = (ke - kb + BK - 1) / BK;

  const int wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave - wm * WGN;

  OpStager<T, BM, LA> sa;
  OpStager<T, BN, LB> sb;
  sa.init(la, row0, kb);
  sb.init(lb, col0, kb);

  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    sa.prefetch(la, kb, smem);
    sb.prefetch(lb, kb, smem + GA::BYTES);
    sa.commit(smem);
    sb.commit(smem + GA::BYTES);
  }
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const bool more = (t + 1) < nk;
    char* nxt = smem + ((t + 1) & 1) * STAGE;
    if (more) {
      sa.prefetch(la, kb + (t + 1) * BK, nxt);
      sb.prefetch(lb, kb + (t + 1) * BK, nxt + GA::BYTES);
    }
    const char* ia = smem + (t & 1) * STAGE;
    const char* ib = ia + GA::BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (sizeof(T) == 2) {
        v8bf fa[MB], fb[NB];
#pragma unroll
        for (int a = 0; a < MB; ++a) fa[a] = frag_bf16<LA::kKContig, GA::RB>(ia, wm * WTM + a * 16, s);
#pragma unroll
        for (int b = 0; b < NB; ++b) fb[b] = frag_bf16<LB::kKContig, GB::RB>(ib, wn * WTN + b * 16, s);
#pragma unroll
        for (int a = 0; a < MB; ++a)
#pragma unroll
          for (int b = 0; b < NB; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
      } else {
        v4f fa[MB], fb[NB];
#pragma unroll
        for (int a = 0; a < MB; ++a) fa[a] = frag_f32<LA::kKContig, GA::RB>(ia, wm * WTM + a * 16, s);
#pragma unroll
        for (int b = 0; b < NB; ++b) fb[b] = frag_f32<LB::kKContig, GB::RB>(ib, wn * WTN + b * 16, s);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int a = 0; a < MB; ++a)
#pragma unroll
            for (int b = 0; b < NB; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(fb[b][j], fa[a][j], acc[a][b], 0, 0, 0);
      }
    }
    if (more) {
      sa.commit(nxt);
      sb.commit(nxt + GA::BYTES);
    }
    __syncthreads();
  }

  // ---------------- epilogue ----------------
  // lane l = 16g + i owns C[row = rbase + i][col = cbase + 4g .. 4g+3].
  // Column blocks are finished one at a time so the statistic partials have a
  // short live range (the whole-tile form cost ~140 VGPRs and 2 waves/SIMD).
  const int l = threadIdx.x & 63;
  const int li = l & 15, lg = l >> 4;
  float* red = reinterpret_cast<float*>(smem);   // [WGM][BN][2]; LDS is free after the K loop
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int col = col0 + wn * WTN + b * 16 + 4 * lg;
    v4f s1 = v4f{0.f, 0.f, 0.f, 0.f}, s2 = s1;
#pragma unroll
    for (int a = 0; a < MB; ++a) {
      const int row = row0 + wm * WTM + a * 16 + li;
      if (row < sh.M && col < sh.N) {
        v4f c1 = v4f{0.f, 0.f, 0.f, 0.f}, c2 = c1;
        ep(row, col, acc[a][b], c1, c2);
        if constexpr (EP::kStats) { s1 += c1; s2 += c2; }
      }
    }
    if constexpr (EP::kStats) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = row16_sum(s1[j]), y = row16_sum(s2[j]);
        if (li == 15) {
          const int cl = wn * WTN + b * 16 + 4 * lg + j;
          red[(wm * BN + cl) * 2 + 0] = x;
          red[(wm * BN + cl) * 2 + 1] = y;
        }
      }
    }
  }
  if constexpr (EP::kStats) {
    // per-wave partials -> one fp64 atomic per column per workgroup, spread
    // over `stat_rep` replicas (replica = tile id % stat_rep) so ~1e5
    // workgroups do not serialise on the same C addresses; vlp_stat_reduce
    // folds the replicas afterwards.
    __syncthreads();
    const int rep = ep.stat_rep > 1 ? (wid % ep.stat_rep) : 0;
    for (int cl = threadIdx.x; cl < BN; cl += 256) {
      const int col = col0 + cl;
      if (col < sh.N) {
        float x = 0.f, y = 0.f;
#pragma unroll
        for (int w = 0; w < WGM; ++w) { x += red[(w * BN + cl) * 2]; y += red[(w * BN + cl) * 2 + 1]; }
        atomicAdd(ep.stat1 + (size_t)rep * sh.N + col, (double)x);
        atomicAdd(ep.stat2 + (size_t)rep * sh.N + col, (double)y);
      }
    }
  }
}

// ---------------- multi-stage direct-to-LDS kernel (bf16) ----------------
// S-slot LDS ring: tiles t+1 .. t+S-2 stay in flight while tile t is
// multiplied.  Per K-step: wait (counted vmcnt: this wave's loads of tile t
// have landed), raw s_barrier (every wave's have; every wave finished tile
// t-1, whose slot is refilled next), issue tile t+S-1, compute tile t.  A
// __syncthreads() would drain the ring (an LDS-DMA is a pending VM op), so
// the wait and barrier are explicit.
template <typename T, int BM, class L, int NT, bool KC = L::kKContig>
struct GStagerN;
// K-contig operand: [BM rows][128 B] image, 16-B chunks XOR-swizzled by row.
template <typename T, int BM, class L, int NT>
struct GStagerN<T, BM, L, NT, true> {
  static constexpr int NI = BM * 8 / NT;   // 16-B chunks (= 1 KiB wave-instructions) per thread
  static_assert(NI >= 1 && (BM * 8) % NT == 0, "tile / thread geometry");
  typename L::DState st[NI];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (w * NI + i) * 64 + lane;
      const int r = q >> 3, p = q & 7;
      st[i] = ld.start(row0 + r, (p ^ ((r >> 1) & 7)) * Elem<T>::EPC, kb);
    }
  }
  __device__ __forceinline__ void issue(const L& ld, int k0, char* lds, bool = false) {
    const int w = threadIdx.x >> 6;
    const auto stp = ld.step(k0);   // K-step-uniform context (scalar registers)
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const void* p = ld.next(st[i], stp);
      __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)(lds + (w * NI + i) * 1024),
                                       16, 0, 0);
    }
  }
};
// MN-contig operand, blocked image (mn8_off): wave w's instruction i fills
// 1-KiB block b = w*NI + i = (k-row block b / CPB, chunk block b % CPB), lane
// L row k = 8*(b / CPB) + L/8 -- 8 full 128-B lines per instruction.  The
// loader's per-k state (e.g. the output pixel of a weight-gradient
// reduction) is walked once per distinct row of the thread (NI / CPB rows)
// and combined with a fixed offset per chunk column:
//   RState rstart(int k, int kb); void radvance(RState&)      per k-row
//   CState cstart(int mn)                                      per column
//   const void* addr(const RState&, const CState&)             address / zero page
template <typename T, int BM, class L, int NT>
struct GStagerN<T, BM, L, NT, false> {
  static constexpr int NW = NT / 64;
  static constexpr int CPB = BM / 64;              // chunk blocks per k-row block
  static constexpr int NI = 8 * CPB / NW;          // 1-KiB blocks per thread
  static constexpr int NR = NI >= CPB ? NI / CPB : 1;   // distinct k-rows per thread
  static_assert(NI >= 1 && (8 * CPB) % NW == 0 && (NI % CPB == 0 || CPB % NI == 0), "tile / thread geometry");
  static_assert(sizeof(T) == 2, "MN direct staging is bf16 (BK = 64 rows)");
  typename L::RState rs[NR];
  typename L::CState cs[NI];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int b = w * NI + i;
      const int k = 8 * (b / CPB) + (lane >> 3);
      const int c = 8 * (b % CPB) + ((lane & 7) ^ mn8_h(k));
      cs[i] = ld.cstart(row0 + c * 8);
      if (i % CPB == 0 || NI < CPB) {
        if (i / CPB < NR) rs[i / CPB] = ld.rstart(k, kb);
      }
    }
  }
  __device__ __forceinline__ void issue(const L& ld, int, char* lds, bool freeze = false) {
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const void* p = ld.addr(rs[NI >= CPB ? i / CPB : 0], cs[i]);
      __builtin_amdgcn_global_load_lds(p, (__attribute__((address_space(3))) void*)(lds + (w * NI + i) * 1024),
                                       16, 0, 0);
    }
    if (!freeze) {
#pragma unroll
      for (int r = 0; r < NR; ++r) ld.radvance(rs[r]);
    }
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void raw_barrier() { asm volatile("s_barrier" ::: "memory"); }

template <class EP>
__device__ __forceinline__ double* stat3_of(const EP& ep) {
  if constexpr (Stat3Trait<EP>::value) return ep.stat3;
  else return nullptr;
}

// timing experiments only (wrong results): 1 = staged epilogues skip their
// global stores, 2 = staged epilogues skip the statistics reduction + atomics,
// 3 = row epilogues skip their operand loads (pre8)
#ifndef VLP_EPI_EXP
#define VLP_EPI_EXP 0
#endif
// Epilogue shared by the multi-stage kernels: lane l = 16g + i owns
// C[row = rbase + i][col = cbase + 4g .. 4g+3] of each 16x16 block.
// LP: the row epilogue's operand slot kLdsSlot comes from the LDS image lds_pre.
// RAW (staged epilogues): the workgroup syncs are LDS-only (lgkmcnt + s_barrier,
// no vmcnt drain), so the epilogue's own stores stay in flight past it, and the
// statistics scratch is red_ovr with the staging tile at smem (persistent kernels
// keep the next tile's loads in the rest of LDS).
template <int BM, int BN, int WGM, int WGN, class EP, bool LP = false, bool RAW = false, int MB, int NB>
__device__ __forceinline__ void ms_epilogue(const GemmShape& sh, const EP& ep, v4f (&acc)[MB][NB], int row0,
                                            int col0, int wid, int wm, int wn, char* smem,
                                            const char* lds_pre = nullptr, float* red_ovr = nullptr) {
  auto epi_sync = [&]() __attribute__((always_inline)) {
    if constexpr (RAW) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    } else {
      __syncthreads();
    }
  };
  constexpr int NT = WGM * WGN * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  const int l = threadIdx.x & 63;
  const int li = l & 15, lg = l >> 4;
  if constexpr (RowTrait<EP>::value) {
    // row-chunk epilogue: the raw accumulators are staged as a bf16 tile, then
    // every thread walks 16-B row chunks of ONE fixed 8-column group, so the
    // epilogue's own operand loads (residual, ReLU mask, BN input) are
    // row-contiguous 16-B loads like its stores, and the per-column statistic
    // partials stay in 16 registers per thread until one LDS reduction.
    constexpr int CPR = BN / 8;
    static_assert(NT % CPR == 0, "row-chunk geometry");
    bf16* stg = reinterpret_cast<bf16*>(smem);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int coll = wn * WTN + b * 16 + 4 * lg;
      v4f bb = v4f{0.f, 0.f, 0.f, 0.f};
      if constexpr (StageBiasTrait<EP>::value) {
        if (ep.bias != nullptr && col0 + coll < sh.N) bb = *reinterpret_cast<const v4f*>(ep.bias + col0 + coll);
      }
#pragma unroll
      for (int a = 0; a < MB; ++a) {
        const int rowl = wm * WTM + a * 16 + li;
        v4bf ob;
        if constexpr (StageBiasTrait<EP>::value) {
          ob[0] = (bf16)(acc[a][b][0] + bb[0]); ob[1] = (bf16)(acc[a][b][1] + bb[1]);
          ob[2] = (bf16)(acc[a][b][2] + bb[2]); ob[3] = (bf16)(acc[a][b][3] + bb[3]);
        } else {
          ob[0] = (bf16)acc[a][b][0]; ob[1] = (bf16)acc[a][b][1];
          ob[2] = (bf16)acc[a][b][2]; ob[3] = (bf16)acc[a][b][3];
        }
        *reinterpret_cast<v4bf*>(stg + rowl * BN + (((coll >> 3) ^ (rowl & (CPR - 1))) << 3) + (coll & 4)) = ob;
      }
    }
    // the thread's operand rows (D chunks ahead) and its 8 columns' per-channel
    // coefficients are requested while the staged tile settles: the loads of
    // the row loop overlap each other instead of one round trip per row
    constexpr int RS = NT / CPR;
    constexpr int NIT = (BM + RS - 1) / RS;
    constexpr int D = PreDepthTrait<EP>::value < NIT ? PreDepthTrait<EP>::value : NIT;
    constexpr int NCF = CoefTrait<EP>::value;
    const int c = threadIdx.x % CPR;
    const int col = col0 + c * 8;
    const int r0 = threadIdx.x / CPR;
    const bool cok = col < sh.N;
    using PreT = typename PreTypeTrait<EP>::type;
    constexpr bool S3 = Stat3Trait<EP>::value;
    constexpr int NS = S3 ? 3 : 2;
    PreT pre[D];
    // lds_pre: operand slot LS of every row is the caller's LDS image [BM rows][BN * 2 B]
    // (all rows and columns of the tile valid), read at use; the other slots load here
    constexpr int LS = LP ? LdsSlotTrait<EP>::value : -1;
    static_assert(!LP || LS >= 0, "LDS operand staging needs E::kLdsSlot");
    auto pre_load = [&](int row, PreT& p) __attribute__((always_inline)) {
      if constexpr (LS >= 0) ep.pre8_rest(row, col, p);
      else ep.pre8(row, col, p);
    };
#pragma unroll
    for (int i = 0; i < D; ++i) {
      const int r = r0 + i * RS;
      if (VLP_EPI_EXP != 3 && cok && r < BM && row0 + r < sh.M) pre_load(row0 + r, pre[i]);
    }
    float cf[NCF > 0 ? NCF : 1][8];
    if constexpr (NCF > 0) {
      if (cok) {
#pragma unroll
        for (int k = 0; k < NCF; ++k) {
          const v4f a = *reinterpret_cast<const v4f*>(ep.coef(k) + col);
          const v4f b = *reinterpret_cast<const v4f*>(ep.coef(k) + col + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { cf[k][j] = a[j]; cf[k][4 + j] = b[j]; }
        }
      }
    }
    __syncthreads();
    float s1[8], s2[8], s3[S3 ? 8 : 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) s1[j] = s2[j] = 0.f;
#pragma unroll
    for (int j = 0; j < (S3 ? 8 : 1); ++j) s3[j] = 0.f;
#pragma unroll
    for (int i = 0; i < NIT; ++i) {
      const int r = r0 + i * RS;
      const int row = row0 + r;
      PreT cur = pre[i % D];
      if constexpr (LS >= 0) cur.u[LS] = *reinterpret_cast<const uint4*>(lds_pre + r * (BN * 2) + c * 16);
      if (i + D < NIT) {
        const int rn = r + D * RS;
        if (VLP_EPI_EXP != 3 && cok && rn < BM && row0 + rn < sh.M) pre_load(row0 + rn, pre[i % D]);
      }
      if (cok && r < BM && row < sh.M) {
        float v[8];
        Chunk<bf16>::unpack(*reinterpret_cast<const uint4*>(stg + r * BN + ((c ^ (r & (CPR - 1))) << 3)), v);
        if constexpr (S3) ep.row8r3(row, col, v, cur, s1, s2, s3, cf);
        else if constexpr (NCF > 0) ep.row8r(row, col, v, cur, s1, s2, cf);
        else ep.row8(row, col, v, cur, s1, s2);
      }
    }
    if constexpr (EP::kStats) {
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem);   // [NT][8 * NS]
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[threadIdx.x * 8 * NS + j] = s1[j];
        red[threadIdx.x * 8 * NS + 8 + j] = s2[j];
        if constexpr (S3) red[threadIdx.x * 8 * NS + 16 + j] = s3[j];
      }
      __syncthreads();
      const int rep = ep.stat_rep > 1 ? (wid % ep.stat_rep) : 0;
      for (int q = threadIdx.x; q < NS * BN; q += NT) {
        const int cl = q / NS, stt = q - cl * NS;
        const int cc = cl >> 3, j = cl & 7;
        float x = 0.f;
        for (int k = cc; k < NT; k += CPR) x += red[k * 8 * NS + stt * 8 + j];
        double* dst = stt == 0 ? ep.stat1 : stt == 1 ? ep.stat2 : stat3_of(ep);
        if (col0 + cl < sh.N) atomicAdd(dst + (size_t)rep * sh.N + col0 + cl, (double)x);
      }
    }
    return;
  }
  float* red = RAW ? red_ovr : reinterpret_cast<float*>(smem);
  // staged epilogues: outputs go through a bf16 LDS tile (16-B chunks XOR-
  // swizzled by row) and leave as full 16-B row segments, 4..8 rows per wave
  // store instead of 32-B pieces of 16 rows
  constexpr bool kStage = StageTrait<EP>::value;
  static_assert(!RAW || kStage, "raw-sync epilogues are the staged ones");
  constexpr int CPR = BN / 8;
  bf16* stg = reinterpret_cast<bf16*>(smem + (RAW ? 0 : 4096));
  
  static_assert(!EP::kStats || WGM * BN * 2 * 4 <= 4096, "stats scratch");
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const int coll = wn * WTN + b * 16 + 4 * lg;
    const int col = col0 + coll;
    v4f s1 = v4f{0.f, 0.f, 0.f, 0.f}, s2 = s1;
#pragma unroll
    for (int a = 0; a < MB; ++a) {
      const int rowl = wm * WTM + a * 16 + li;
      const int row = row0 + rowl;
      if (row < sh.M && col < sh.N) {
        v4f c1 = v4f{0.f, 0.f, 0.f, 0.f}, c2 = c1;
        if constexpr (kStage) {
          const v4f o = ep.value(row, col, acc[a][b], c1, c2);
          v4bf ob;
          ob[0] = (bf16)o[0]; ob[1] = (bf16)o[1]; ob[2] = (bf16)o[2]; ob[3] = (bf16)o[3];
          *reinterpret_cast<v4bf*>(stg + rowl * BN + (((coll >> 3) ^ (rowl & (CPR - 1))) << 3) +
                                   (coll & 4)) = ob;
        } else {
          ep(row, col, acc[a][b], c1, c2);
        }
        if constexpr (EP::kStats) { s1 += c1; s2 += c2; }
      }
    }
    if constexpr (EP::kStats) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float x = row16_sum(s1[j]), y = row16_sum(s2[j]);
        if (li == 15) {
          const int cl = wn * WTN + b * 16 + 4 * lg + j;
          red[(wm * BN + cl) * 2 + 0] = x;
          red[(wm * BN + cl) * 2 + 1] = y;
        }
      }
    }
  }
  if constexpr (kStage) {
    epi_sync();
#pragma unroll 4
    for (int q = threadIdx.x; q < BM * CPR; q += NT) {
      const int r = q / CPR, c = q - r * CPR;
      const int row = row0 + r, col = col0 + c * 8;
      if (VLP_EPI_EXP != 1 && row < sh.M && col < sh.N)
        ep.store8(row, col, *reinterpret_cast<const uint4*>(stg + r * BN + ((c ^ (r & (CPR - 1))) << 3)));
    }
  }
  if constexpr (EP::kStats && VLP_EPI_EXP != 2) {
    epi_sync();
    const int rep = ep.stat_rep > 1 ? (wid % ep.stat_rep) : 0;
    for (int cl = threadIdx.x; cl < BN; cl += NT) {
      const int col = col0 + cl;
      if (col < sh.N) {
        float x = 0.f, y = 0.f;
#pragma unroll
        for (int w = 0; w < WGM; ++w) { x += red[(w * BN + cl) * 2]; y += red[(w * BN + cl) * 2 + 1]; }
        atomicAdd(ep.stat1 + (size_t)rep * sh.N + col, (double)x);
        atomicAdd(ep.stat2 + (size_t)rep * sh.N + col, (double)y);
      }
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int S, class LA, class LB, class EP>
__global__ void __launch_bounds__(WGM * WGN * 64)
gemm_ms_kernel(GemmShape sh, LA la, LB lb, EP ep) {
  using T = bf16;
  constexpr int NT = WGM * WGN * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MB = WTM / 16, NB = WTN / 16;
  constexpr int BK = 64;
  using GA = TileGeom<T, BM, LA::kKContig>;
  using GB = TileGeom<T, BN, LB::kKContig>;
  constexpr int ABYTES = BM * 128;
  constexpr int STAGE = (BM + BN) * 128;
  using SA = GStagerN<T, BM, LA, NT>;
  using SB = GStagerN<T, BN, LB, NT>;
  constexpr int NI = SA::NI + SB::NI;   // VM ops per thread per tile

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = sh.tiles_m * sh.tiles_n;
  const int bid = blockIdx.x;
  int wid = bid, split = blockIdx.y;
  if (sh.xsplit) {
    // split-K reductions re-read their K slice once per tile: keep all tiles of
    // a split on one XCD (dispatch is round-robin over XCDs) so the slice is
    // fetched into ONE L2 instead of eight
    const int xcd = bid & 7, j = bid >> 3, jt = j / nwg;
    split = xcd + 8 * jt;
    wid = j - jt * nwg;
  } else if (nwg >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = nwg >> 3, rr = nwg & 7;
    wid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int tm = wid / sh.tiles_n, tn = wid - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * sh.kchunk;
  int ke = kb + sh.kchunk;
  if (ke > sh.K) ke = sh.K;
  const int nk = (ke - kb + BK - 1) / BK;
  const int wave = threadIdx.x >> 6;
  const int wm = wave / WGN, wn = wave - wm * WGN;

  SA sa;
  SB sb;
  sa.init(la, row0, kb);
  sb.init(lb, col0, kb);
  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    if (s < nk) {
      sa.issue(la, kb + s * BK, smem + s * STAGE);
      sb.issue(lb, kb + s * BK, smem + s * STAGE + ABYTES);
    }
  }
  int slot = 0;                 // slot of tile t
  int fill = S - 1;             // slot receiving tile t + S - 1
  for (int t = 0; t < nk; ++t) {
    // tiles issued after t so far: min(t + S - 2, nk - 1) - t
    const int ahead = (t + S - 2 < nk - 1 ? S - 2 : nk - 1 - t);
    if constexpr (S >= 4) {
      if (ahead >= 2) wait_vmcnt<2 * NI>();
      else if (ahead == 1) wait_vmcnt<NI>();
      else wait_vmcnt<0>();
    } else if constexpr (S == 3) {
      if (ahead >= 1) wait_vmcnt<NI>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    raw_barrier();
    // All fragments of tile t are read BEFORE tile t+S-1 is issued: hipcc
    // cannot tell a ds_read_b64_tr_b16 from a read of the DMA target and
    // would otherwise drain the just-issued loads (s_waitcnt vmcnt(0)) in
    // front of the first transposed read, serialising load and compute.
    const char* ia = smem + slot * STAGE;
    const char* ib = ia + ABYTES;
    v8bf fa[2][MB], fb[2][NB];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int a = 0; a < MB; ++a) fa[s][a] = frag_bf16<LA::kKContig, GA::RB, true>(ia, wm * WTM + a * 16, s);
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[s][b] = frag_bf16<LB::kKContig, GB::RB, true>(ib, wn * WTN + b * 16, s);
    }
    if (t + S - 1 < nk) {
      char* f = smem + fill * STAGE;
      sa.issue(la, kb + (t + S - 1) * BK, f, false);
      sb.issue(lb, kb + (t + S - 1) * BK, f + ABYTES, false);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][b], fa[s][a], acc[a][b], 0, 0, 0);
    }
    slot = (slot + 1 == S) ? 0 : slot + 1;
    fill = (fill + 1 == S) ? 0 : fill + 1;
  }
  __syncthreads();   // all waves done with the ring before the epilogue reuses LDS

  static_assert(!StageTrait<EP>::value || 4096 + BM * BN * 2 <= S * STAGE, "staging tile fits the ring");
  ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep, acc, row0, col0, wid, wm, wn, smem);
}

// ---------------- buffer-DMA two-slot kernel (bf16) ----------------
// The same engine as gemm_ms_kernel with S = 2, restated for a lower VALU
// cost per K-step (profiling: 4-8 VALU per MFMA in the direct kernels, more
// than the two-waves-per-SIMD issue budget of ~2):
//  * operands are fetched with buffer_load ... lds through a buffer resource
//    (base + 32-bit byte offset): an out-of-range chunk is an offset past
//    num_records (kOOB), which the hardware returns as zeros, so no zero-page
//    pointer select and no 64-bit address arithmetic;
//  * the K loop is unrolled by the two ring slots, so every LDS address
//    (fragment reads, DMA destinations) is a compile-time offset from a
//    wave-uniform base held in SGPRs;
//  * a K-step past the end issues through a null resource (num_records = 0)
//    instead of branching, so the loop body stays one basic block.
// Loader protocol (kBuf = true):
//   rsrc_t rsrc() const                                     whole-operand resource
//   K-contig: BState bstart(int row, int koff, int kb); BStep bstep(int k0);
//             unsigned boff(BState&, const BStep&)          byte offset | kOOB
//   MN-contig: BRow brstart(int k, int kb); BCol bcstart(int mn);
//             unsigned boff(const BRow&, const BCol&); void bradvance(BRow&)
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr unsigned kOOB = 0x80000000u;   // every operand is < 2 GiB (checked on the host)

__device__ __forceinline__ rsrc_t buf_rsrc(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  void* q = (void*)(((unsigned long long)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ rsrc_t null_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0, 0x00020000);
}
__device__ __forceinline__ void dma16(rsrc_t r, unsigned voff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, 0, 0, 0);
}

// A operand loaders that ask the ping-pong kernel to apply relu(sc[c]*a + sh[c])
// to the A fragments in registers (BN-apply + ReLU on load; padding taps and
// rows past M masked to zero from the loader's tap-validity mask)
template <class L, class = void> struct XformTrait { static constexpr bool value = false; };
template <class L> struct XformTrait<L, std::void_t<decltype(L::kXformA)>> { static constexpr bool value = L::kXformA; };
__device__ __forceinline__ v8bf bn_relu_frag(v8bf v, v4f s0, v4f s1, v4f h0, v4f h1, bool ok) {
  v8bf r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    r[j] = (bf16)fmaxf(fmaf((float)v[j], s0[j], h0[j]), 0.f);
    r[4 + j] = (bf16)fmaxf(fmaf((float)v[4 + j], s1[j], h1[j]), 0.f);
  }
  return ok ? r : v8bf{};
}
template <class L, class = void> struct BufTrait { static constexpr bool value = false; };
template <class L> struct BufTrait<L, std::void_t<decltype(L::kBuf)>> { static constexpr bool value = L::kBuf; };

template <int BM, class L, int NT, bool KC = L::kKContig>
struct BStager;
// K-contig operand: [BM rows][128 B] image, chunk p of row r at p ^ ((r>>1)&7).
template <int BM, class L, int NT>
struct BStager<BM, L, NT, true> {
  static constexpr int NI = BM * 8 / NT;
  static_assert(NI >= 1 && (BM * 8) % NT == 0, "tile / thread geometry");
  typename L::BState st[NI];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb, int wv) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int q = (wv * NI + i) * 64 + lane;
      const int r = q >> 3, p = q & 7;
      st[i] = ld.bstart(row0 + r, (p ^ ((r >> 1) & 7)) * 8, kb);
    }
  }
  __device__ __forceinline__ void issue(const L& ld, rsrc_t rs, int k0, char* lds, int wv) {
    const auto stp = ld.bstep(k0);
#pragma unroll
    for (int i = 0; i < NI; ++i) dma16(rs, ld.boff(st[i], stp), lds + (wv * NI + i) * 1024);
  }
};
// MN-contig operand, blocked image (mn8_off), as GStagerN.
template <int BM, class L, int NT>
struct BStager<BM, L, NT, false> {
  static constexpr int NW = NT / 64;
  static constexpr int CPB = BM / 64;
  static constexpr int NI = 8 * CPB / NW;
  static constexpr int NR = NI >= CPB ? NI / CPB : 1;
  static_assert(NI >= 1 && (8 * CPB) % NW == 0 && (NI % CPB == 0 || CPB % NI == 0), "tile / thread geometry");
  typename L::BRow rs[NR];
  typename L::BCol cs[NI];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb, int wv) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int b = wv * NI + i;
      const int k = 8 * (b / CPB) + (lane >> 3);
      const int c = 8 * (b % CPB) + ((lane & 7) ^ mn8_h(k));
      cs[i] = ld.bcstart(row0 + c * 8);
      if (i % CPB == 0 || NI < CPB) {
        if (i / CPB < NR) rs[i / CPB] = ld.brstart(k, kb);
      }
    }
  }
  __device__ __forceinline__ void issue(const L& ld, rsrc_t r, int, char* lds, int wv) {
#pragma unroll
    for (int i = 0; i < NI; ++i) dma16(r, ld.boff(rs[NI >= CPB ? i / CPB : 0], cs[i]), lds + (wv * NI + i) * 1024);
#pragma unroll
    for (int j = 0; j < NR; ++j) ld.bradvance(rs[j]);
  }
};

// at least two waves per SIMD: the 4-wave tiles (128x128, 256x64) then fit in
// 256 registers, so two workgroups share a CU (their LDS rings allow it) and
// one's epilogue overlaps the other's main loop; the 8-wave tiles have two
// waves per SIMD anyway
#ifndef VLP_WAVES_PER_EU
#define VLP_WAVES_PER_EU 2
#endif
template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP>
__global__ void __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_waves_per_eu(VLP_WAVES_PER_EU)))
gemm_bk_kernel(GemmShape sh, LA la, LB lb, EP ep) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MB = WTM / 16, NB = WTN / 16;
  constexpr int BK = 64;
  constexpr int ABYTES = BM * 128;
  constexpr int STAGE = (BM + BN) * 128;
  using SA = BStager<BM, LA, NT>;
  using SB = BStager<BN, LB, NT>;
  static_assert(!StageTrait<EP>::value || 4096 + BM * BN * 2 <= 2 * STAGE, "staging tile fits the ring");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  // 1-D grid over (split, tile), split-major, bijectively remapped so each
  // XCD owns a contiguous run: the tiles of one K-split (which share its
  // operand slab) sit on one or two XCDs and hit one L2
  const int nwg = sh.tiles_m * sh.tiles_n;
  const int ntot = nwg * sh.nsplit;
  const int bid = blockIdx.x;
  int g = bid;
  if (ntot >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = ntot >> 3, rr = ntot & 7;
    g = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int split = g / nwg;
  const int wid = g - split * nwg;
  const int tm = wid / sh.tiles_n, tn = wid - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * sh.kchunk;
  int ke = kb + sh.kchunk;
  if (ke > sh.K) ke = sh.K;
  const int nk = (ke - kb + BK - 1) / BK;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wm = wv / WGN, wn = wv - wm * WGN;

  SA sa;
  SB sb;
  sa.init(la, row0, kb, wv);
  sb.init(lb, col0, kb, wv);
  const rsrc_t ra = la.rsrc(), rb = lb.rsrc();
  const rsrc_t rz = null_rsrc(zero_page());
  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};

  // odd nk: tile 0 goes to slot 1 so the main loop always runs slot pairs
  const int s0 = (nk & 1) * STAGE;
  sa.issue(la, nk > 0 ? ra : rz, kperm_of(la, kb), smem + s0, wv);
  sb.issue(lb, nk > 0 ? rb : rz, kperm_of(la, kb), smem + s0 + ABYTES, wv);

  // one K-step: tile t sits in ring slot SL; tile t+1 is fetched into 1-SL
  auto body = [&](auto slc, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slc)::value;
    wait_vmcnt<0>();
    raw_barrier();
    const char* ia = smem + SL * STAGE;
    const char* ib = ia + ABYTES;
    v8bf fa[2][MB], fb[2][NB];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int a = 0; a < MB; ++a) fa[s][a] = frag_bf16<LA::kKContig, BM * 2, true>(ia, wm * WTM + a * 16, s);
#pragma unroll
      for (int b = 0; b < NB; ++b) fb[s][b] = frag_bf16<LB::kKContig, BN * 2, true>(ib, wn * WTN + b * 16, s);
    }
    const bool live = t + 1 < nk;
    char* f = smem + (1 - SL) * STAGE;
    const int kn = kperm_of(la, kb + (t + 1) * BK);
    sa.issue(la, live ? ra : rz, kn, f, wv);
    sb.issue(lb, live ? rb : rz, kn, f + ABYTES, wv);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[s][b], fa[s][a], acc[a][b], 0, 0, 0);
  };
  int t = 0;
  if (nk & 1) {
    body(std::integral_constant<int, 1>{}, 0);
    t = 1;
  }
  for (; t < nk; t += 2) {
    body(std::integral_constant<int, 0>{}, t);
    body(std::integral_constant<int, 1>{}, t + 1);
  }
  __syncthreads();   // ring drained (incl. the null-resource tail fetch) before LDS is reused
  if constexpr (SplitTrait<EP>::value) {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep.at_split(split), acc, row0, col0, wid, wm, wn, smem);
  } else {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep, acc, row0, col0, wid, wm, wn, smem);
  }
}

// ---------------- 8-wave large-tile kernel (bf16) ----------------
// The 128x128 / two-barrier / one-tile-in-flight structure tops out near
// 900 TF/s (its per-K-step vmcnt(0) drains the prefetch; measured: halving
// the VALU per MFMA did not move it).  This kernel runs one 512-thread
// workgroup per CU on a 256-row tile, with TWO K-tiles in flight:
//   iteration t (tile t in ring slot t&1):
//     vmcnt(NI) + barrier          tile t landed (tile t+1 still in flight)
//     read all fragments of tile t (k-substeps 0 and 1) into registers
//     MFMAs of k-substep 0         (overlap the substep-1 reads)
//     lgkmcnt(0) + barrier         every wave is done with slot t&1
//     fetch tile t+2 into slot t&1 (null resource past the end)
//     MFMAs of k-substep 1
// so each fetch has ~two iterations of MFMA work to land in, and the
// operand traffic per FLOP halves against 128x128 (256x256: 128 FLOP/B).
template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP, int WPE = VLP_WAVES_PER_EU>
__global__ void __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_waves_per_eu(WPE)))
gemm_big_kernel(GemmShape sh, LA la, LB lb, EP ep) {
  constexpr int NT = WGM * WGN * 64;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MB = WTM / 16, NB = WTN / 16;
  constexpr int BK = 64;
  constexpr int ABYTES = BM * 128;
  constexpr int STAGE = (BM + BN) * 128;
  using SA = BStager<BM, LA, NT>;
  using SB = BStager<BN, LB, NT>;
  constexpr int NI = SA::NI + SB::NI;   // LDS-DMA ops per thread per K-tile

  extern __shared__ __attribute__((aligned(16))) char smem[];

  // 1-D grid over (split, tile), split-major, bijectively remapped so each
  // XCD owns a contiguous run: the tiles of one K-split (which share its
  // operand slab) sit on one or two XCDs and hit one L2
  const int nwg = sh.tiles_m * sh.tiles_n;
  const int ntot = nwg * sh.nsplit;
  const int bid = blockIdx.x;
  int g = bid;
  if (ntot >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = ntot >> 3, rr = ntot & 7;
    g = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int split = g / nwg;
  const int wid = g - split * nwg;
  const int tm = wid / sh.tiles_n, tn = wid - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  const int kb = split * sh.kchunk;
  int ke = kb + sh.kchunk;
  if (ke > sh.K) ke = sh.K;
  const int nk = (ke - kb + BK - 1) / BK;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wm = wv / WGN, wn = wv - wm * WGN;

  SA sa;
  SB sb;
  sa.init(la, row0, kb, wv);
  sb.init(lb, col0, kb, wv);
  const rsrc_t ra = la.rsrc(), rb = lb.rsrc();
  const rsrc_t rz = null_rsrc(zero_page());
  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};

  // odd nk: tile 0 goes to slot 1 so the main loop always runs slot pairs
  const int s0 = (nk & 1) * STAGE;
  sa.issue(la, nk > 0 ? ra : rz, kperm_of(la, kb), smem + s0, wv);
  sb.issue(lb, nk > 0 ? rb : rz, kperm_of(la, kb), smem + s0 + ABYTES, wv);
  sa.issue(la, nk > 1 ? ra : rz, kperm_of(la, kb + BK), smem + (STAGE - s0), wv);
  sb.issue(lb, nk > 1 ? rb : rz, kperm_of(la, kb + BK), smem + (STAGE - s0) + ABYTES, wv);
  // MN-contig operands: one LDS address per (ring slot, fragment)
  constexpr int QA = MB < 4 ? MB : 4, QB = NB < 4 ? NB : 4;
  unsigned abase[2][LA::kKContig ? 1 : QA], bbase[2][LB::kKContig ? 1 : QB];
  if constexpr (!LA::kKContig) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
      for (int a = 0; a < QA; ++a) abase[sl][a] = mn_frag_base<BM * 2>(smem + sl * STAGE, wm * WTM + a * 16);
  }
  if constexpr (!LB::kKContig) {
#pragma unroll
    for (int sl = 0; sl < 2; ++sl)
#pragma unroll
      for (int b = 0; b < QB; ++b)
        bbase[sl][b] = mn_frag_base<BN * 2>(smem + sl * STAGE + ABYTES, wn * WTN + b * 16);
  }
  auto fragA = [&](auto slc, const char* ia, auto ac, int s) __attribute__((always_inline)) {
    constexpr int a = decltype(ac)::value;
    if constexpr (LA::kKContig) return frag_big<true, BM * 2>(ia, wm * WTM + a * 16, s);
    else return frag_tr_sub<BM * 2, a>(abase[decltype(slc)::value][a & 3], s);
  };
  auto fragB = [&](auto slc, const char* ib, auto bc, int s) __attribute__((always_inline)) {
    constexpr int b = decltype(bc)::value;
    if constexpr (LB::kKContig) return frag_big<true, BN * 2>(ib, wn * WTN + b * 16, s);
    else return frag_tr_sub<BN * 2, b>(bbase[decltype(slc)::value][b & 3], s);
  };

#if VLP_BIG_PRIO
  // static priority for the second-dispatched half (MI355X_MICROARCH.md, "Two waves
  // per SIMD" item 4): waves 4-7 are the arbitration losers on every segment
  if (wv >= (WGM * WGN) / 2) __builtin_amdgcn_s_setprio(1);
#endif
  auto body = [&](auto slc, int t) __attribute__((always_inline)) {
    constexpr int SL = decltype(slc)::value;
    wait_vmcnt<NI>();
    raw_barrier();
    const char* ia = smem + SL * STAGE;
    const char* ib = ia + ABYTES;
    v8bf fa[2][MB], fb[2][NB];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      static_for<0, MB>([&](auto ac) { fa[s][decltype(ac)::value] = fragA(slc, ia, ac, s); });
      static_for<0, NB>([&](auto bc) { fb[s][decltype(bc)::value] = fragB(slc, ib, bc, s); });
    }
    if constexpr (!LA::kKContig || !LB::kKContig) asm_lds_wait();
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[0][b], fa[0][a], acc[a][b], 0, 0, 0);
#if VLP_BIG_SCHED >= 2
    // K-contig operands: the substep-1 fragment reads trail the substep-0 MFMAs
    // (one ds_read_b128 per two MFMAs) instead of bursting before them
    if constexpr (LA::kKContig && LB::kKContig) {
#pragma unroll
      for (int q = 0; q < MB + NB; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x0100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x0008, 2, 0);
      }
    }
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    const bool live = t + 2 < nk;
    char* f = smem + SL * STAGE;
    const int kn = kperm_of(la, kb + (t + 2) * BK);
    sa.issue(la, live ? ra : rz, kn, f, wv);
    sb.issue(lb, live ? rb : rz, kn, f + ABYTES, wv);
#pragma unroll
    for (int a = 0; a < MB; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[1][b], fa[1][a], acc[a][b], 0, 0, 0);
#if VLP_BIG_SCHED >= 1
    // the next tile's LDS-DMA pieces spread over the substep-1 MFMAs (one per
    // MB*NB/NI MFMAs) instead of a burst in which the SIMD's matrix pipe idles
    {
      constexpr int PER = (MB * NB) / NI > 0 ? (MB * NB) / NI : 1;
#pragma unroll
      for (int q = 0; q < NI; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x0010, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x0008, PER, 1);
      }
    }
#endif
  };
  int t = 0;
  if (nk & 1) {
    body(std::integral_constant<int, 1>{}, 0);
    t = 1;
  }
  for (; t < nk; t += 2) {
    body(std::integral_constant<int, 0>{}, t);
    body(std::integral_constant<int, 1>{}, t + 1);
  }
  __syncthreads();   // ring drained (incl. the null-resource tail fetches) before LDS is reused
  if constexpr (SplitTrait<EP>::value) {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep.at_split(split), acc, row0, col0, wid, wm, wn, smem);
  } else {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep, acc, row0, col0, wid, wm, wn, smem);
  }
}

template <int BM, int BN, class EP>
constexpr int big_lds_bytes() {
  constexpr int ring = 2 * (BM + BN) * 128;
  constexpr int stg = StageTrait<EP>::value ? 4096 + BM * BN * 2 : 4096;
  return ring > stg ? ring : stg;
}

// ---------------- ping-pong large-tile kernel (bf16, K-contig operands) ----------------
// The two wave groups of a 2 x WGN workgroup (M halves; one wave of each per
// SIMD) run one barrier interval apart, so that on every SIMD one wave issues
// its MFMAs while its partner issues the next phase's fragment reads and
// LDS-DMA pieces (MI355X_MICROARCH "two waves per SIMD"; the 256x256
// 8-phase schedule of cdna_hip_programming.md §5).  The ring holds four
// 32-deep half-tiles ([rows][64 B] images, 16-B chunk c of row r at
// c ^ (bit3(r) << 1): conflict-free ds_read_b128 fragment reads); the loaders
// still step 64-deep (half h = the chunks 4h..4h+3 of a step, +64 B).
// Phase q (half-tile q in slot q % 4), per wave:
//   L_q: fragment reads of half-tile q; group 0 fetches A of half-tile q+2,
//        group 1 B of half-tile q+3 (then waits until B of q+1 has landed);
//        barrier
//   M_q: lgkmcnt(0); MFMAs; group 0 waits until A of q+1 has landed; barrier
// Group 1 enters one barrier late, so its L_q shares an interval with group
// 0's M_q.  A slot is refetched only after both groups' reads of its previous
// half-tile retired behind a barrier (q+2 / q+3 land in slots last read in
// phases q-2 / q-1), and half-tile q+1 is read only after both issuers'
// counted waits and a barrier.
// MFMA issue of a phase at raised wave priority (the partner wave's loads then
// issue in the MFMA gaps, MI355X guide 8-phase template)
#ifndef VLP_PP_PRIO
#define VLP_PP_PRIO 1
#endif
// timing experiments only (wrong results): 1 = no LDS-DMA issue, 2 = no fragment
// reads, 3 = no MFMAs (tools/build_variant.sh; never in the product library)
#ifndef VLP_PP_EXP
#define VLP_PP_EXP 0
#endif
__device__ __forceinline__ int pp_chunk(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }
template <int BM, class L, int NTG, bool KC = L::kKContig>
struct HStager;
// K-contig operand: [BM rows][64 B] half image, 16 rows per wave-wide piece
template <int BM, class L, int NTG>
struct HStager<BM, L, NTG, true> {
  static constexpr int P = BM * 4 / NTG;   // 16-B pieces per thread per half-tile
  static_assert(P >= 1 && (BM * 4) % NTG == 0, "tile / thread geometry");
  typename L::BState st[P];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb, int wg) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int q = (wg * P + i) * 64 + lane;
      const int r = q >> 2;
      st[i] = ld.bstart(row0 + r, pp_chunk(r, q & 3) * 8, kb);
    }
  }
  template <int H>
  __device__ __forceinline__ void issue(const L& ld, rsrc_t rs, int k0, char* lds, int wg) {
    const auto stp = ld.bstep(k0);
#pragma unroll
    for (int i = 0; i < P; ++i) dma16(rs, ld.boff(st[i], stp) + (unsigned)H * 64u, lds + (wg * P + i) * 1024);
  }
};
// MN-contig operand: the blocked image (mn8_off) of 32 k-rows; each wave owns
// one 8-row k-group, so a thread keeps one pixel-row walk per half
template <int BM, class L, int NTG>
struct HStager<BM, L, NTG, false> {
  static constexpr int CPB = BM / 64;
  static constexpr int P = BM * 4 / NTG;
  static_assert(P == CPB && NTG == 256, "one k-group per wave");
  typename L::BRow rs[2];
  typename L::BCol cs[P];
  __device__ __forceinline__ void init(const L& ld, int row0, int kb, int wg) {
    const int lane = threadIdx.x & 63;
    const int k = 8 * wg + (lane >> 3);
#pragma unroll
    for (int i = 0; i < P; ++i) cs[i] = ld.bcstart(row0 + (8 * i + ((lane & 7) ^ mn8_h(k))) * 8);
    rs[0] = ld.brstart(k, kb);
    rs[1] = ld.brstart(k + 32, kb);
  }
  template <int H>
  __device__ __forceinline__ void issue(const L& ld, rsrc_t r, int, char* lds, int wg) {
#pragma unroll
    for (int i = 0; i < P; ++i) dma16(r, ld.boff(rs[H], cs[i]), lds + (wg * P + i) * 1024);
    ld.bradvance(rs[H]);
  }
};

template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP>
__global__ void __launch_bounds__(WGM * WGN * 64) __attribute__((amdgpu_waves_per_eu(2)))
gemm_pp_kernel(GemmShape sh, LA la, LB lb, EP ep) {
  static_assert(WGM % 2 == 0, "two M-half wave groups");
  constexpr int NT = WGM * WGN * 64, NTG = NT / 2;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MB = WTM / 16, NB = WTN / 16;
  constexpr int BK = 64;
  constexpr int HA = BM * 64, SLOT = (BM + BN) * 64;
  using SA = HStager<BM, LA, NTG>;
  using SB = HStager<BN, LB, NTG>;

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int nwg = sh.tiles_m * sh.tiles_n;
  const int ntot = nwg * sh.nsplit;
  const int bid = blockIdx.x;
  int g = bid;
  if (ntot >= 16) {
    const int xcd = bid & 7, idx = bid >> 3, q = ntot >> 3, rr = ntot & 7;
    g = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  }
  const int split = g / nwg;
  const int wid = g - split * nwg;
  const int kb = split * sh.kchunk;
  int ke = kb + sh.kchunk;
  const int tm = wid / sh.tiles_n, tn = wid - tm * sh.tiles_n;
  const int row0 = tm * BM, col0 = tn * BN;
  if (ke > sh.K) ke = sh.K;
  const int nk = (ke - kb + BK - 1) / BK;
  const int nh = 2 * (nk > 0 ? nk : 0);
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int wm = wv / WGN, wn = wv - wm * WGN;
  const int grp = wm / (WGM / 2), wg = wv - grp * (WGM / 2) * WGN;

  const rsrc_t ra = la.rsrc(), rb = lb.rsrc();
  const rsrc_t rz = null_rsrc(zero_page());
  v4f acc[MB][NB];
#pragma unroll
  for (int a = 0; a < MB; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[a][b] = v4f{0.f, 0.f, 0.f, 0.f};

  // half-tile u sits in slot (u + off) % 4 (off even, so u and its slot share
  // parity = the half of its 64-deep step); nh % 4 == 2 starts at slot 2 so
  // the 4-phase unrolled loop ends on slot 3
  const int off = nh & 2;
  const int lane = threadIdx.x & 63;
  const int fi = lane & 15, fg = lane >> 4;
  const char* fbase = smem + fi * 64 + (pp_chunk(fi, fg) << 4);
  // BN-apply on the A fragments: per-channel (scale, shift) table in LDS past
  // the ring / epilogue staging, one tap-validity mask per fragment row
  constexpr bool XA = XformTrait<LA>::value;
  float* const xtab = reinterpret_cast<float*>(smem + big_lds_bytes<BM, BN, EP>());
  unsigned xm[XA ? (MB + 2) / 3 : 1];   // three 9-bit row masks per register
  if constexpr (XA) {
    const int C = la.xchannels();
    for (int i = threadIdx.x; i < C; i += NT) {
      xtab[i] = la.sc[i];
      xtab[512 + i] = la.sh[i];
    }
#pragma unroll
    for (int a = 0; a < (MB + 2) / 3; ++a) xm[a] = 0;
#pragma unroll
    for (int a = 0; a < MB; ++a) xm[a / 3] |= la.xrow_mask(row0 + wm * WTM + a * 16 + fi) << (9 * (a % 3));
    __syncthreads();
  }
  // MN-contig operands: one transposing-read address per (slot pair, fragment column)
  constexpr int QA = MB < 4 ? MB : 4, QB = NB < 4 ? NB : 4;
  unsigned abase[2][LA::kKContig ? 1 : QA], bbase[2][LB::kKContig ? 1 : QB];
  if constexpr (!LA::kKContig) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int a = 0; a < QA; ++a) abase[p][a] = mn_frag_base<BM * 2>(smem + 2 * p * SLOT, wm * WTM + a * 16);
  }
  if constexpr (!LB::kKContig) {
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int b = 0; b < QB; ++b) bbase[p][b] = mn_frag_base<BN * 2>(smem + 2 * p * SLOT + HA, wn * WTN + b * 16);
  }

  // the main loop of one wave group: group 0 holds only A's loader state,
  // group 1 only B's (the two paths share the register allocation)
  auto run = [&](auto gc) __attribute__((always_inline)) {
    constexpr int G = decltype(gc)::value;
    using S = std::conditional_t<G == 0, SA, SB>;
    S ss;
    if constexpr (G == 0) ss.init(la, row0, kb, wg);
    else ss.init(lb, col0, kb, wg);
    auto fetch = [&](auto hc, int u, char* slot) __attribute__((always_inline)) {
      if constexpr (VLP_PP_EXP == 1) return;
      if constexpr (VLP_PP_EXP == 6 && G == 0) if (((u >> 1) % 9) != 0) return;   // A bytes / 9
      if constexpr (VLP_PP_EXP == 7 && G == 1) if (((u >> 1) % 9) != 0) return;   // B bytes / 9
      const int k0 = VLP_PP_EXP == 5 ? kb + (u >> 1) * BK : kperm_of(la, kb + (u >> 1) * BK);
      if constexpr (G == 0) ss.template issue<decltype(hc)::value>(la, u < nh ? ra : rz, k0, slot, wg);
      else ss.template issue<decltype(hc)::value>(lb, u < nh ? rb : rz, k0, slot + HA, wg);
    };
    using H0 = std::integral_constant<int, 0>;
    using H1 = std::integral_constant<int, 1>;
    if constexpr (G == 0) {
      fetch(H0{}, 0, smem + off * SLOT);
      fetch(H1{}, 1, smem + ((off + 1) & 3) * SLOT);
      wait_vmcnt<S::P>();
    } else {
      fetch(H0{}, 0, smem + off * SLOT);
      fetch(H1{}, 1, smem + ((off + 1) & 3) * SLOT);
      fetch(H0{}, 2, smem + ((off + 2) & 3) * SLOT);
      wait_vmcnt<2 * S::P>();
    }
    raw_barrier();
    if constexpr (G == 1) raw_barrier();   // the stagger
    __builtin_amdgcn_sched_barrier(0);

    auto phase = [&](auto slc, int q) __attribute__((always_inline)) {
      constexpr int SL = decltype(slc)::value;
      constexpr int SO = (SL & 1) * SLOT;   // offset inside the slot pair
      v8bf fa[MB], fb[NB];
      if constexpr (VLP_PP_EXP == 2) {
#pragma unroll
        for (int a = 0; a < MB; ++a) fa[a] = v8bf{};
#pragma unroll
        for (int b = 0; b < NB; ++b) fb[b] = v8bf{};
      } else {
      static_for<0, MB>([&](auto ac) {
        constexpr int a = decltype(ac)::value;
        if constexpr (LA::kKContig)
          fa[a] = *reinterpret_cast<const v8bf*>(fbase + SL * SLOT + (wm * WTM + a * 16) * 64);
        else
          fa[a] = frag_tr_at<SO + (a >> 2) * 1024>(abase[SL >> 1][a & 3]);
      });
      static_for<0, NB>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        if constexpr (LB::kKContig)
          fb[b] = *reinterpret_cast<const v8bf*>(fbase + SL * SLOT + HA + (wn * WTN + b * 16) * 64);
        else
          fb[b] = frag_tr_at<SO + (b >> 2) * 1024>(bbase[SL >> 1][b & 3]);
      });
      }
      v4f xs0, xs1, xh0, xh1;
      unsigned xtap = 0;
      if constexpr (XA) {
        int ci0;
        xtap = la.xtap(kperm_of(la, kb + (q >> 1) * BK), ci0);
        const float* t = xtab + ci0 + (SL & 1) * 32 + fg * 8;
        xs0 = *reinterpret_cast<const v4f*>(t);
        xs1 = *reinterpret_cast<const v4f*>(t + 4);
        xh0 = *reinterpret_cast<const v4f*>(t + 512);
        xh1 = *reinterpret_cast<const v4f*>(t + 516);
      }
      if constexpr (G == 0) {
        fetch(std::integral_constant<int, SL & 1>{}, q + 2, smem + ((SL + 2) & 3) * SLOT);
      } else {
        fetch(std::integral_constant<int, 1 - (SL & 1)>{}, q + 3, smem + ((SL + 3) & 3) * SLOT);
        wait_vmcnt<2 * S::P>();
      }
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#if VLP_PP_PRIO
      __builtin_amdgcn_s_setprio(1);
#endif
      if constexpr (XA) {
#pragma unroll
        for (int a = 0; a < MB; ++a) fa[a] = bn_relu_frag(fa[a], xs0, xs1, xh0, xh1, (xm[a / 3] >> (xtap + 9 * (a % 3))) & 1u);
      }
      if constexpr (VLP_PP_EXP == 4 && NB == 4) {   // 32x32x16 issue pattern (wrong layout)
        typedef float v16f_ __attribute__((ext_vector_type(16)));
#pragma unroll
        for (int a = 0; a < MB; ++a) {
          v16f_ t = *reinterpret_cast<v16f_*>(&acc[a][0]);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[a & 3], fa[a], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[(a + 1) & 3], fa[a], t, 0, 0, 0);
          *reinterpret_cast<v16f_*>(&acc[a][0]) = t;
        }
      } else if constexpr (VLP_PP_EXP != 3) {
#pragma unroll
      for (int a = 0; a < MB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[b], fa[a], acc[a][b], 0, 0, 0);
      } else {
#pragma unroll
      for (int a = 0; a < MB; ++a)
        acc[a][0][0] += (float)fa[a][0] + (float)fb[0][0];
      }
#if VLP_PP_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      if constexpr (G == 0) wait_vmcnt<S::P>();
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
      __builtin_amdgcn_sched_barrier(0);
    };
    int q = 0;
    if (off) {
      phase(std::integral_constant<int, 2>{}, 0);
      phase(std::integral_constant<int, 3>{}, 1);
      q = 2;
    }
    for (; q < nh; q += 4) {
      phase(std::integral_constant<int, 0>{}, q);
      phase(std::integral_constant<int, 1>{}, q + 1);
      phase(std::integral_constant<int, 2>{}, q + 2);
      phase(std::integral_constant<int, 3>{}, q + 3);
    }
    if constexpr (G == 0) raw_barrier();   // matches group 1's stagger barrier
  };
  if (grp == 0) run(std::integral_constant<int, 0>{});
  else run(std::integral_constant<int, 1>{});
  __syncthreads();   // ring drained (incl. the null-resource tail fetches) before LDS is reused
  if constexpr (SplitTrait<EP>::value) {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep.at_split(split), acc, row0, col0, wid, wm, wn, smem);
  } else {
    ms_epilogue<BM, BN, WGM, WGN, EP>(sh, ep, acc, row0, col0, wid, wm, wn, smem);
  }
}

// Split-K count for a reduction of K over `tiles` output tiles, given the
// number of workgroups the chip holds at once (`slots`).  Workgroups of one
// launch all cost about the same, so the launch takes ceil(WG / slots)
// rounds: pick the split (1..4 rounds' worth) with the best slot fill, each
// split still >= min_k deep (epilogue atomics amortised).
// split count of the last launch_gemm_bk / launch_gemm_big call on this host
// thread (callers of split-store epilogues size their fold pass with it)
inline int& last_ksplit() {
  static thread_local int v = 1;
  return v;
}
// fraction of the chip's workgroup slots an auto-split launch is sized for
// (1: all; the weight gradients on their side stream may take fewer, see
// conv_wgrad_ws_t)
inline int& ksplit_slot_div() {
  static thread_local int v = 1;
  return v;
}
inline int balanced_ksplit(int tiles, int K, int slots, int min_k) {
  slots = slots / ksplit_slot_div() > 0 ? slots / ksplit_slot_div() : 1;
  if (tiles >= slots) return 1;
  int best = 1;
  double best_eff = 0.0;
  for (int r = 1; r <= 4; ++r) {
    int ks = r * slots / tiles;
    if (ks < 1) continue;
    if (ks > 1 && K / ks < min_k) {   // too shallow: the deepest split that keeps min_k
      ks = K / min_k > 1 ? K / min_k : 1;
      const long long wg = (long long)ks * tiles;
      const double eff = (double)wg / (double)(((wg + slots - 1) / slots) * slots);
      if (ks > best && (eff > best_eff + 0.01 || best == 1)) best = ks;
      break;
    }
    const long long wg = (long long)ks * tiles;
    const double eff = (double)wg / (double)(((wg + slots - 1) / slots) * slots);
    if (eff > best_eff + 0.01) { best_eff = eff; best = ks; }
  }
  return best;
}
// current device index (per-device caches of per-function launch state)
inline int cur_dev() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d & 31;
}
inline int device_cus() {
  static int n[32] = {};
  const int d = cur_dev();
  if (!n[d]) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0) v = 256;
    n[d] = v;
  }
  return n[d];
}
// Launch state of one kernel instantiation, per device: the dynamic-LDS limit is
// raised once per device (its error returned, not dropped), and the resident
// workgroups per CU are queried once per device (the split-K choice uses them)
struct KernelDevState {
  unsigned attr_set = 0;
  int occ[32] = {};
};
inline int prepare_kernel(KernelDevState& s, const void* fn, int lds, int threads, int* occ) {
  const int d = cur_dev();
  if (lds > 65536 && !(s.attr_set & (1u << d))) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return (int)e;
    s.attr_set |= 1u << d;
  }
  if (occ) {
    if (!s.occ[d]) {
      int o = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, threads, lds) != hipSuccess || o <= 0) o = 1;
      s.occ[d] = o;
    }
    *occ = s.occ[d];
  }
  return 0;
}

template <int BM, int BN, int WGM, int WGN, int S, class LA, class LB, class EP>
inline int launch_gemm_ms(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                          hipStream_t stream) {
  constexpr int BK = 64;
  if (M <= 0 || N <= 0) return 0;
  GemmShape sh;
  sh.xsplit = 0;
  sh.nsplit = 1;
  sh.dbg = 0;
  sh.M = M; sh.N = N; sh.K = K;
  sh.tiles_m = (M + BM - 1) / BM;
  sh.tiles_n = (N + BN - 1) / BN;
  constexpr int lds = S * (BM + BN) * 128;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static KernelDevState kst;
  if (ksplit <= 0) {   // auto: fill whole rounds of resident workgroups
    int occ = 1;
    const int e = prepare_kernel(kst, (const void*)&gemm_ms_kernel<BM, BN, WGM, WGN, S, LA, LB, EP>, lds, WGM * WGN * 64, &occ);
    if (e) return e;
    ksplit = balanced_ksplit(sh.tiles_m * sh.tiles_n, K, occ * device_cus(), -ksplit > 0 ? -ksplit : 2048);
  }
  if (ksplit < 1) ksplit = 1;
  int kc = (K + ksplit - 1) / ksplit;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc < BK) kc = BK;
  ksplit = (K + kc - 1) / kc;
  if (ksplit < 1) ksplit = 1;
  sh.kchunk = kc;
  sh.xsplit = (ksplit >= 8 && ksplit % 8 == 0) ? 1 : 0;
  dim3 grid = sh.xsplit ? dim3(sh.tiles_m * sh.tiles_n * ksplit, 1, 1)
                        : dim3(sh.tiles_m * sh.tiles_n, ksplit, 1);
  {
    const int e = prepare_kernel(kst, (const void*)&gemm_ms_kernel<BM, BN, WGM, WGN, S, LA, LB, EP>, lds, 0, nullptr);
    if (e) return e;
  }
  hipLaunchKernelGGL((gemm_ms_kernel<BM, BN, WGM, WGN, S, LA, LB, EP>), grid, dim3(WGM * WGN * 64), lds,
                     stream, sh, la, lb, ep);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP>
inline int launch_gemm_bk(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                          hipStream_t stream) {
  constexpr int BK = 64;
  constexpr int S = 2;
  if (M <= 0 || N <= 0) return 0;
  GemmShape sh;
  sh.xsplit = 0;
  sh.nsplit = 1;
  sh.dbg = 0;
  sh.M = M; sh.N = N; sh.K = K;
  sh.tiles_m = (M + BM - 1) / BM;
  sh.tiles_n = (N + BN - 1) / BN;
  constexpr int lds = S * (BM + BN) * 128;
  static_assert(lds <= 160 * 1024, "LDS budget");
  static KernelDevState kst;
  if (ksplit <= 0) {   // auto: fill whole rounds of resident workgroups
    int occ = 1;
    const int e = prepare_kernel(kst, (const void*)&gemm_bk_kernel<BM, BN, WGM, WGN, LA, LB, EP>, lds, WGM * WGN * 64, &occ);
    if (e) return e;
    ksplit = balanced_ksplit(sh.tiles_m * sh.tiles_n, K, occ * device_cus(), -ksplit > 0 ? -ksplit : 2048);
  }
  if (ksplit < 1) ksplit = 1;
  int kc = (K + ksplit - 1) / ksplit;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc < BK) kc = BK;
  ksplit = (K + kc - 1) / kc;
  if (ksplit < 1) ksplit = 1;
  sh.kchunk = kc;
  sh.xsplit = 0;
  sh.nsplit = ksplit;
  last_ksplit() = ksplit;
  dim3 grid(sh.tiles_m * sh.tiles_n * ksplit, 1, 1);
  {
    const int e = prepare_kernel(kst, (const void*)&gemm_bk_kernel<BM, BN, WGM, WGN, LA, LB, EP>, lds, 0, nullptr);
    if (e) return e;
  }
  hipLaunchKernelGGL((gemm_bk_kernel<BM, BN, WGM, WGN, LA, LB, EP>), grid, dim3(WGM * WGN * 64), lds,
                     stream, sh, la, lb, ep);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP, int WPE = VLP_WAVES_PER_EU>
inline int launch_gemm_big(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                          hipStream_t stream) {
  constexpr int BK = 64;
  constexpr int S = 2;
  if (M <= 0 || N <= 0) return 0;
  GemmShape sh;
  sh.xsplit = 0;
  sh.nsplit = 1;
  sh.dbg = 0;
  sh.M = M; sh.N = N; sh.K = K;
  sh.tiles_m = (M + BM - 1) / BM;
  sh.tiles_n = (N + BN - 1) / BN;
  constexpr int lds = big_lds_bytes<BM, BN, EP>();
  static_assert(lds <= 160 * 1024, "LDS budget");
  static KernelDevState kst;
  if (ksplit <= 0) {   // auto: fill whole rounds of resident workgroups
    int occ = 1;
    const int e = prepare_kernel(kst, (const void*)&gemm_big_kernel<BM, BN, WGM, WGN, LA, LB, EP, WPE>, lds, WGM * WGN * 64, &occ);
    if (e) return e;
    ksplit = balanced_ksplit(sh.tiles_m * sh.tiles_n, K, occ * device_cus(), -ksplit > 0 ? -ksplit : 2048);
  }
  if (ksplit < 1) ksplit = 1;
  int kc = (K + ksplit - 1) / ksplit;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc < BK) kc = BK;
  ksplit = (K + kc - 1) / kc;
  if (ksplit < 1) ksplit = 1;
  sh.kchunk = kc;
  sh.xsplit = 0;
  sh.nsplit = ksplit;
  last_ksplit() = ksplit;
  dim3 grid(sh.tiles_m * sh.tiles_n * ksplit, 1, 1);
  {
    const int e = prepare_kernel(kst, (const void*)&gemm_big_kernel<BM, BN, WGM, WGN, LA, LB, EP, WPE>, lds, 0, nullptr);
    if (e) return e;
  }
  hipLaunchKernelGGL((gemm_big_kernel<BM, BN, WGM, WGN, LA, LB, EP, WPE>), grid, dim3(WGM * WGN * 64), lds,
                     stream, sh, la, lb, ep);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WGM, int WGN, class LA, class LB, class EP>
inline int launch_gemm_pp(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                          hipStream_t stream) {
  constexpr int BK = 64;
  if (M <= 0 || N <= 0) return 0;
  GemmShape sh;
  sh.xsplit = 0;
  sh.dbg = 0;
  sh.M = M; sh.N = N; sh.K = K;
  sh.tiles_m = (M + BM - 1) / BM;
  sh.tiles_n = (N + BN - 1) / BN;
  constexpr int lds = big_lds_bytes<BM, BN, EP>() + (XformTrait<LA>::value ? 4096 : 0);
  static_assert(lds <= 160 * 1024, "LDS budget");
  static KernelDevState kst;
  if (ksplit <= 0) {   // auto: fill whole rounds of resident workgroups
    int occ = 1;
    const int e = prepare_kernel(kst, (const void*)&gemm_pp_kernel<BM, BN, WGM, WGN, LA, LB, EP>, lds, WGM * WGN * 64, &occ);
    if (e) return e;
    ksplit = balanced_ksplit(sh.tiles_m * sh.tiles_n, K, occ * device_cus(), -ksplit > 0 ? -ksplit : 2048);
  }
  if (ksplit < 1) ksplit = 1;
  int kc = (K + ksplit - 1) / ksplit;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc < BK) kc = BK;
  ksplit = (K + kc - 1) / kc;
  if (ksplit < 1) ksplit = 1;
  sh.kchunk = kc;
  sh.nsplit = ksplit;
  last_ksplit() = ksplit;
  dim3 grid(sh.tiles_m * sh.tiles_n * ksplit, 1, 1);
  {
    const int e = prepare_kernel(kst, (const void*)&gemm_pp_kernel<BM, BN, WGM, WGN, LA, LB, EP>, lds, 0, nullptr);
    if (e) return e;
  }
  hipLaunchKernelGGL((gemm_pp_kernel<BM, BN, WGM, WGN, LA, LB, EP>), grid, dim3(WGM * WGN * 64), lds, stream, sh,
                     la, lb, ep);
  return (int)hipGetLastError();
}

template <typename T, int BM, int BN>
constexpr int gemm_lds_bytes() { return 2 * (BM + BN) * 128; }

// ---------------- variant dispatch ----------------
// bf16 + direct loaders -> multi-stage kernels; everything else -> the
// register-staged 2-stage kernel.  VLP_GEMM_DEFAULT_VARIANT (compile time) selects among tile /
// stage configurations (tools/build_variant.sh builds A/B libraries; the default is the measured best).
#ifndef VLP_GEMM_DEFAULT_VARIANT
#define VLP_GEMM_DEFAULT_VARIANT 5
#endif
inline int gemm_variant() {
  return VLP_GEMM_DEFAULT_VARIANT;
}
template <typename T, class LA, class LB>
constexpr bool use_ms() {
  return std::is_same<T, bf16>::value && DirectTrait<LA>::value && DirectTrait<LB>::value;
}
template <typename T, class LA, class LB>
constexpr bool use_bk() {
  return std::is_same<T, bf16>::value && BufTrait<LA>::value && BufTrait<LB>::value;
}
// large-tile shape choice: 256x256 (8 waves, one workgroup per CU) when both
// dimensions allow it, else 128x256, and 128x128 (4 waves) for N = 128
template <class LA, class LB, class EP>
inline int gemm_big_auto(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep, hipStream_t st) {
  // (256x256 keeps 128x64 fragments per wave live: only the all-K-contig case
  // fits the 256-VGPR budget without spilling)
  // ping-pong schedule (gemm_pp_kernel): 1 = K-contig x K-contig, 2 = also MN x MN
  // (default 2, measured per step: K-contig +0.4-0.8 % (the 256x256 forward /
  // data-gradient GEMMs +3 %), MN x MN weight gradients another +2.4 % (layers
  // 3-4 +10-19 %); the 128x256 MN tiles of layer 2 lose (-10 %) and stay on
  // gemm_big_kernel, as do 256x128 K-contig tiles)
  constexpr int pp = 2;   // ping-pong kernel for K-contig 256x256 and MNxMN weight gradients
  constexpr bool kk = LA::kKContig && LB::kKContig;
  constexpr bool mm = !LA::kKContig && !LB::kKContig;
  if constexpr (kk || mm) {
    if (pp >= (kk ? 1 : 2) && M >= 256 && N >= 256 && K % 64 == 0)
      return launch_gemm_pp<256, 256, 2, 4>(M, N, K, ksplit, la, lb, ep, st);
  }
  if constexpr (mm) {
    // Co = 128 weight gradients (layer 2, N = 9 * 128 = 3 * 384): 128x384 tiles,
    // a 64x96 per-wave tile (20 transposing reads per 24 MFMAs)
    if (pp >= 2 && pp != 7 && M > 64 && M <= 128 && N % 384 == 0 && K % 64 == 0)
      return launch_gemm_pp<128, 384, 2, 4>(M, N, K, ksplit, la, lb, ep, st);
  }
  if constexpr (kk) {
    if (M >= 256 && N >= 256) return launch_gemm_big<256, 256, 2, 4>(M, N, K, ksplit, la, lb, ep, st);
  }
  if (N >= 256) return launch_gemm_big<128, 256, 2, 4>(M, N, K, ksplit, la, lb, ep, st);
  // N = 128: 128x128 tiles (4 waves, 64 KB ring) run two workgroups per CU, so
  // one tile's epilogue overlaps the other's main loop (layer 2, K = 1152 is
  // only 18 K-steps per tile); measured +1 % per step over 256x128
  constexpr int n128 = 1;
  if (n128 == 1) return launch_gemm_big<128, 128, 2, 2>(M, N, K, ksplit, la, lb, ep, st);
  return launch_gemm_big<256, 128, 4, 2>(M, N, K, ksplit, la, lb, ep, st);
}
// N >= 128 columns
template <typename T, class LA, class LB, class EP>
inline int gemm_wide(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                     hipStream_t st) {
  if constexpr (use_bk<T, LA, LB>()) {
    if (gemm_variant() >= 4) return launch_gemm_bk<128, 128, 2, 2>(M, N, K, ksplit, la, lb, ep, st);
  }
  if constexpr (use_ms<T, LA, LB>()) {
    switch (gemm_variant()) {
      case 0: return launch_gemm<T, 128, 128, 2>(M, N, K, ksplit, la, lb, ep, st);
      case 3: return launch_gemm_ms<128, 128, 2, 2, 2>(M, N, K, ksplit, la, lb, ep, st);
      default: return launch_gemm_ms<256, 128, 4, 2, 2>(M, N, K, ksplit, la, lb, ep, st);
    }
  } else {
    return launch_gemm<T, 128, 128, 2>(M, N, K, ksplit, la, lb, ep, st);
  }
}
// convolution GEMMs with N >= 128 (and M >= 128): the 8-wave large-tile
// kernel where both loaders speak the buffer protocol (VLP_GEMM_VARIANT >= 5)
template <typename T, class LA, class LB, class EP>
inline int gemm_conv_wide(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                          hipStream_t st) {
  if constexpr (use_bk<T, LA, LB>()) {
    if (gemm_variant() >= 5) return gemm_big_auto(M, N, K, ksplit, la, lb, ep, st);
  }
  return gemm_wide<T>(M, N, K, ksplit, la, lb, ep, st);
}
// N <= 64 columns (Co = 64 convs)
template <typename T, class LA, class LB, class EP>
inline int gemm_narrow(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                       hipStream_t st) {
  if constexpr (use_bk<T, LA, LB>()) {
    if (gemm_variant() >= 6 && M >= 512) return launch_gemm_big<512, 64, 8, 1>(M, N, K, ksplit, la, lb, ep, st);
    if (gemm_variant() >= 4) return launch_gemm_bk<256, 64, 4, 1>(M, N, K, ksplit, la, lb, ep, st);
  }
  if constexpr (use_ms<T, LA, LB>()) {
    switch (gemm_variant()) {
      case 0: return launch_gemm<T, 256, 64, 4>(M, N, K, ksplit, la, lb, ep, st);
      case 3: return launch_gemm_ms<256, 64, 4, 1, 2>(M, N, K, ksplit, la, lb, ep, st);
      default: return launch_gemm_ms<256, 64, 4, 1, 4>(M, N, K, ksplit, la, lb, ep, st);
    }
  } else {
    return launch_gemm<T, 256, 64, 4>(M, N, K, ksplit, la, lb, ep, st);
  }
}
// M <= 64 rows (weight gradients of Co = 64 convs)
template <typename T, class LA, class LB, class EP>
inline int gemm_short(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                      hipStream_t st) {
  if constexpr (use_bk<T, LA, LB>()) {
    // 64 x 192 tiles (3 taps of 64 channels) on the two-K-tiles-in-flight engine:
    // the 4-wave 64 x 128 ring kept one K-tile in flight and was latency-bound
    constexpr int short_big = 1;
    if (gemm_variant() >= 5 && short_big && N % 192 == 0)
      return launch_gemm_big<64, 192, 1, 4>(M, N, K, ksplit, la, lb, ep, st);
    if (gemm_variant() >= 4) return launch_gemm_bk<64, 128, 1, 4>(M, N, K, ksplit, la, lb, ep, st);
  }
  if constexpr (use_ms<T, LA, LB>()) {
    switch (gemm_variant()) {
      case 0: return launch_gemm<T, 64, 128, 1>(M, N, K, ksplit, la, lb, ep, st);
      default: return launch_gemm_ms<64, 128, 1, 4, 2>(M, N, K, ksplit, la, lb, ep, st);
    }
  } else {
    return launch_gemm<T, 64, 128, 1>(M, N, K, ksplit, la, lb, ep, st);
  }
}

// Host-side launcher.  ksplit > 1 splits the reduction over grid.y (the
// epilogue must then accumulate atomically).
template <typename T, int BM, int BN, int WGM, class LA, class LB, class EP>
inline int launch_gemm(int M, int N, int K, int ksplit, const LA& la, const LB& lb, const EP& ep,
                       hipStream_t stream) {
  constexpr int BK = Elem<T>::BK;
  if (M <= 0 || N <= 0) return 0;
  GemmShape sh;
  sh.xsplit = 0;
  sh.nsplit = 1;
  sh.dbg = 0;
  sh.M = M; sh.N = N; sh.K = K;
  sh.tiles_m = (M + BM - 1) / BM;
  sh.tiles_n = (N + BN - 1) / BN;
  if (ksplit <= 0) {   // auto: ~1024 workgroups, >= 4096-deep splits
    const int tiles = sh.tiles_m * sh.tiles_n;
    ksplit = (1024 + tiles - 1) / tiles;
    const int maxsplit = (K + 4095) / 4096;
    if (ksplit > maxsplit) ksplit = maxsplit;
  }
  if (ksplit < 1) ksplit = 1;
  int kc = (K + ksplit - 1) / ksplit;
  kc = ((kc + BK - 1) / BK) * BK;
  if (kc < BK) kc = BK;
  ksplit = (K + kc - 1) / kc;
  if (ksplit < 1) ksplit = 1;
  sh.kchunk = kc;
  dim3 grid(sh.tiles_m * sh.tiles_n, ksplit, 1);
  constexpr int lds = gemm_lds_bytes<T, BM, BN>();
  static KernelDevState kst;
  {
    const int e = prepare_kernel(kst, (const void*)&gemm_kernel<T, BM, BN, WGM, LA, LB, EP>, lds, 0, nullptr);
    if (e) return e;
  }
  hipLaunchKernelGGL((gemm_kernel<T, BM, BN, WGM, LA, LB, EP>), grid, dim3(256), lds, stream, sh, la, lb, ep);
  return (int)hipGetLastError();
}

// ---------------- generic loaders ----------------
// Row-major matrix, K contiguous: A(m,k) = p[m*ld + k].  Zero outside [M) x [K).
template <typename T>
struct KMat {
  static constexpr bool kKContig = true;
  static constexpr bool kDirect = true;
  struct State { const T* p; bool ok; };
  const T* p; int ld, M, K;
  __device__ State fixed(int m) const { return State{p + (size_t)m * ld, m < M}; }
  __device__ uint4 load(const State& s, int k) const {
    return (s.ok && k < K) ? ldg16(s.p + k) : zero4();
  }
  struct DState { const T* p; int kk; bool ok; };
  struct Step {};
  __device__ Step step(int) const { return Step{}; }
  __device__ DState start(int m, int koff, int kb) const {
    return DState{p + (size_t)(m < M ? m : 0) * ld + kb + koff, kb + koff, m < M};
  }
  __device__ const void* next(DState& s, const Step&) const {
    const void* r = (s.ok & (s.kk < K)) ? (const void*)s.p : zero_page();
    s.p += Elem<T>::BK;
    s.kk += Elem<T>::BK;
    return r;
  }
  // buffer protocol (gemm_bk_kernel): o = chunk byte offset at k = 0
  static constexpr bool kBuf = true;
  struct BState { unsigned o; int koff; };
  struct BStep { unsigned kbytes; int klim; };
  __device__ rsrc_t rsrc() const { return buf_rsrc(p, (unsigned)(((size_t)(M - 1) * ld + K) * sizeof(T))); }
  __device__ BState bstart(int m, int koff, int) const {
    return BState{m < M ? (unsigned)(((size_t)m * ld + koff) * sizeof(T)) : kOOB, koff};
  }
  __device__ BStep bstep(int k0) const { return BStep{(unsigned)(k0 * sizeof(T)), K - k0}; }
  __device__ unsigned boff(BState& s, const BStep& st) const { return s.koff < st.klim ? s.o + st.kbytes : kOOB; }
};
// MN contiguous: A(m,k) = p[k*ld + m].  Requires M % EPC == 0.
template <typename T>
struct MNMat {
  static constexpr bool kKContig = false;
  static constexpr bool kDirect = true;
  struct State { const T* p; bool ok; };
  const T* p; int ld, M, K;
  __device__ State fixed(int m) const { return State{p + m, m < M}; }
  __device__ uint4 load(const State& s, int k) const {
    return (s.ok && k < K) ? ldg16(s.p + (size_t)k * ld) : zero4();
  }
  struct RState { const T* p; int kk; };   // row k of this thread
  struct CState { int m; bool ok; };
  __device__ RState rstart(int k, int kb) const { return RState{p + (size_t)(kb + k) * ld, kb + k}; }
  __device__ CState cstart(int m) const { return CState{m < M ? m : 0, m < M}; }
  __device__ const void* addr(const RState& r, const CState& c) const {
    return (c.ok & (r.kk < K)) ? (const void*)(r.p + c.m) : zero_page();
  }
  __device__ void radvance(RState& r) const {
    r.p += (size_t)Elem<T>::BK * ld;
    r.kk += Elem<T>::BK;
  }
  // buffer protocol (gemm_bk_kernel)
  static constexpr bool kBuf = true;
  __device__ rsrc_t rsrc() const { return buf_rsrc(p, (unsigned)(((size_t)(K - 1) * ld + M) * sizeof(T))); }
  struct BRow { unsigned o; int kk; };
  typedef unsigned BCol;
  __device__ BRow brstart(int k, int kb) const { return BRow{(unsigned)((size_t)(kb + k) * ld * sizeof(T)), kb + k}; }
  __device__ unsigned bcstart(int m) const { return m < M ? (unsigned)(m * sizeof(T)) : kOOB; }
  __device__ unsigned boff(const BRow& r, unsigned c) const { return r.kk < K ? r.o + c : kOOB; }
  __device__ void bradvance(BRow& r) const {
    r.o += (unsigned)(Elem<T>::BK * ld * sizeof(T));
    r.kk += Elem<T>::BK;
  }
};

// ---------------- generic epilogues ----------------
// out[row*ldo + col] = alpha*v (+ bias[col]) (+ res[row*ldr+col]); optional GELU(erf).
template <typename TO>
struct EpiStore {
  static constexpr bool kStats = false;
  double* stat1 = nullptr; double* stat2 = nullptr;
  TO* out; int ldo;
  const float* bias;      // may be null
  float alpha;
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    v = v * alpha;
    if (bias) v += *reinterpret_cast<const v4f*>(bias + col);
    store4(out + (size_t)row * ldo + col, v);
  }
};
// split-K partial of a weight gradient: split s writes slab s of
// out[ks][rows][ldo] with plain stores, folded by a separate pass (fp32
// atomics of many splits onto the same small dW were the bound:
// ~50 G atomics/s, 80-170 us per conv weight gradient)
struct EpiSplitStore {
  static constexpr bool kStats = false;
  static constexpr bool kSplitOut = true;
  double* stat1 = nullptr; double* stat2 = nullptr;
  float* out; int ldo; size_t slab;
  __device__ EpiSplitStore at_split(int s) const {
    EpiSplitStore e = *this;
    e.out += (size_t)s * slab;
    return e;
  }
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    *reinterpret_cast<v4f*>(out + (size_t)row * ldo + col) = v;
  }
};
// fp32 atomic accumulation (split-K / weight gradients)
struct EpiAtomic {
  static constexpr bool kStats = false;
  double* stat1 = nullptr; double* stat2 = nullptr;
  float* out; int ldo; float alpha;
  __device__ void operator()(int row, int col, v4f v, v4f&, v4f&) const {
    float* p = out + (size_t)row * ldo + col;
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(p + j, v[j] * alpha);
  }
};

}  // namespace vlp
