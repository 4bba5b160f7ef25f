// Micro-probe (tools only): what LDS stores in MFMA shadows cost the issuing wave.  A chain of 48
// v_mfma_f32_32x32x16_bf16 (AGPR accumulator, one wave per SIMD, 4 waves per CU), with S stores
// after every MFMA (S = 0..4), or one store after every second MFMA, of ds_write2_b64 / ds_write_b128 /
// ds_write_b64, conflict-free lane addresses.  Variant W: only SIMD 0's wave stores (the other
// three run the bare chain).
// build: hipcc --offload-arch=gfx950 -O3 -o lds_store_mfma lds_store_mfma.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int N = 48;

// KIND: 0 ds_write2_b64, 1 ds_write_b128, 2 ds_write_b64;  S stores per MFMA (S < 0: one per -S MFMAs)
template <int KIND, int S, bool ONE>
__global__ void __launch_bounds__(256) k(const float *in, float *out, long long *cyc) {
  extern __shared__ char lds[];
  const int t = threadIdx.x, w = t >> 6, l = t & 63;
  bf16x8 a, b;
  for (int i = 0; i < 8; i++) {
    a[i] = (__bf16)in[t * 8 + i];
    b[i] = (__bf16)in[t * 8 + i + 1];
  }
  f32x16 c0 = {};
  uint2 d0 = make_uint2(t, t + 1), d1 = make_uint2(t + 2, t + 3);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 d4 = {(unsigned)t, (unsigned)t + 1, (unsigned)t + 2, (unsigned)t + 3};
  // per wave 16 KiB; store q of a region at (q % 8) KiB, lane 16 l
  const uint32_t base = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)(lds + w * 16384 + 16 * l);
  const bool st = !ONE || w == 0;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  long long t0 = __builtin_readcyclecounter();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; i++) {
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
    const int ns = S >= 0 ? S : (i % (-S) == 0 ? 1 : 0);
    if (st) {
#pragma unroll
      for (int q = 0; q < ns; q++) {
        const int off = ((i * 4 + q) % 8) * 1024;
        if constexpr (KIND == 0)  // (8-bit offsets in 8-byte units: every store to the same KiB)
          asm volatile("ds_write2_b64 %0, %1, %2 offset1:1" ::"v"(base), "v"(d0), "v"(d1) : "memory");
        if constexpr (KIND == 1)
          asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(base), "v"(d4), "i"(off) : "memory");
        if constexpr (KIND == 2)
          asm volatile("ds_write_b64 %0, %1 offset:%2" ::"v"(base), "v"(d0), "i"(off) : "memory");
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  long long t1 = __builtin_readcyclecounter();
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0);
  float s = 0;
  for (int i = 0; i < 16; i++) s += c0[i];
  out[blockIdx.x * 256 + t] = s;
  if (l == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;
}

template <int KIND, int S, bool ONE>
void run(const char *name, float *in, float *out, long long *cyc) {
  (void)hipFuncSetAttribute((const void *)k<KIND, S, ONE>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  for (int rep = 0; rep < 3; rep++) hipLaunchKernelGGL((k<KIND, S, ONE>), dim3(256), dim3(256), 65536, 0, in, out, cyc);
  static long long h[1024];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  double s0 = 0, s1 = 0;
  for (int i = 0; i < 256; i++) {
    s0 += h[4 * i];
    s1 += h[4 * i + 1] + h[4 * i + 2] + h[4 * i + 3];
  }
  printf("%-34s wave0 %6.1f  others %6.1f cycles per MFMA\n", name, s0 / 256 / N, s1 / 768 / N);
}

int main() {
  float *in, *out;
  long long *cyc;
  (void)hipMalloc(&in, 1 << 20);
  (void)hipMalloc(&out, 1 << 22);
  (void)hipMalloc(&cyc, 8 * 1024);
  (void)hipMemset(in, 0, 1 << 20);
  run<0, 0, false>("chain only", in, out, cyc);
  run<0, -2, false>("write2_b64 1 per 2 MFMA, 4 waves", in, out, cyc);
  run<0, 1, false>("write2_b64 1 per MFMA, 4 waves", in, out, cyc);
  run<0, 2, false>("write2_b64 2 per MFMA, 4 waves", in, out, cyc);
  run<0, 3, false>("write2_b64 3 per MFMA, 4 waves", in, out, cyc);
  run<0, 4, false>("write2_b64 4 per MFMA, 4 waves", in, out, cyc);
  run<0, 1, true>("write2_b64 1 per MFMA, wave 0", in, out, cyc);
  run<0, 2, true>("write2_b64 2 per MFMA, wave 0", in, out, cyc);
  run<0, 4, true>("write2_b64 4 per MFMA, wave 0", in, out, cyc);
  run<1, 1, false>("write_b128 1 per MFMA, 4 waves", in, out, cyc);
  run<1, 2, false>("write_b128 2 per MFMA, 4 waves", in, out, cyc);
  run<2, 2, false>("write_b64 2 per MFMA, 4 waves", in, out, cyc);
  run<2, 4, false>("write_b64 4 per MFMA, 4 waves", in, out, cyc);
  return 0;
}
