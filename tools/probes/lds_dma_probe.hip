// Probe: (1) global_load_lds_dwordx4 from a 2-byte-misaligned address,
// (2) raw buffer_load ... lds with an out-of-range offset (zero fill?).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef __attribute__((address_space(3))) void lds_t;
__global__ void probe(const uint16_t* src, uint16_t* out, int shift_elems, int n_bytes) {
  __shared__ __attribute__((aligned(16))) uint16_t s[2][64 * 8];
  const int l = threadIdx.x;
  for (int i = l; i < 2 * 64 * 8; i += 64) (&s[0][0])[i] = 0xBEEF;
  __syncthreads();
  const uint16_t* p = src + l * 8 + shift_elems;
  __builtin_amdgcn_global_load_lds(p, (lds_t*)&s[0][0], 16, 0, 0);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, n_bytes, 0x00020000);
  // lanes >= 32 read out of range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_t*)&s[1][0], 16, l * 16 + (l >= 32 ? 0x40000000 : 0), 0, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = l; i < 2 * 64 * 8; i += 64) out[i] = (&s[0][0])[i];
}
int main() {
  const int N = 64 * 8 + 64;
  uint16_t h[N];
  for (int i = 0; i < N; ++i) h[i] = (uint16_t)i;
  uint16_t *d, *o;
  hipMalloc(&d, N * 2); hipMalloc(&o, 2 * 64 * 8 * 2);
  hipMemcpy(d, h, N * 2, hipMemcpyHostToDevice);
  uint16_t ho[2 * 64 * 8];
  for (int shift = 0; shift < 3; ++shift) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, shift, N * 2);
    hipError_t e = hipDeviceSynchronize();
    hipMemcpy(ho, o, sizeof(ho), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 64 * 8; ++i) bad += ho[i] != (uint16_t)(i + shift);
    int zero_ok = 0, in_ok = 0;
    for (int i = 0; i < 32 * 8; ++i) in_ok += ho[512 + i] == (uint16_t)i;
    for (int i = 32 * 8; i < 64 * 8; ++i) zero_ok += ho[512 + i] == 0;
    printf("shift %d: err=%d misaligned-glds mismatches=%d | buffer-lds in-range ok=%d/256 oob zero=%d/256 (first oob val 0x%04x)\n",
           shift, (int)e, bad, in_ok, zero_ok, ho[512 + 256]);
  }
  return 0;
}
