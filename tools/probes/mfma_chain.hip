// Micro-probe (tools only): cycles per v_mfma_f32_32x32x16_bf16 in a dependent accumulation chain,
// accumulator in VGPRs (builtin, -amdgpu-mfma-vgpr-form=1) vs AGPRs (inline asm "+a"), one or two
// interleaved chains, with 0 or 5 independent VALU per MFMA.  One wave per SIMD (1 024 waves).
// build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form=1 -o mfma_chain mfma_chain.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int N = 48;

template <int MODE>
__global__ void __launch_bounds__(256) k(const float *in, float *out, long long *cyc) {
  const int t = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; i++) {
    a[i] = (__bf16)in[t * 8 + i];
    b[i] = (__bf16)in[t * 8 + i + 1];
  }
  f32x16 c0 = {}, c1 = {};
  float v0 = in[t], v1 = in[t + 1], v2 = in[t + 2], v3 = in[t + 3], v4 = in[t + 4];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  long long t0 = __builtin_readcyclecounter();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < N; i++) {
    if constexpr (MODE == 0 || MODE == 4) c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    if constexpr (MODE == 1 || MODE == 5) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
    if constexpr (MODE == 2 || MODE == 6) {
      if (i & 1) c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
      else c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    }
    if constexpr (MODE == 3 || MODE == 7) {
      if (i & 1) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c1) : "v"(a), "v"(b));
      else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
    }
    if constexpr (MODE >= 4) {  // five independent VALU
      v0 = v0 * 1.0001f + 0.5f;
      v1 = v1 * 1.0001f + 0.5f;
      v2 = v2 * 1.0001f + 0.5f;
      v3 = v3 * 1.0001f + 0.5f;
      v4 = v4 * 1.0001f + 0.5f;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  long long t1 = __builtin_readcyclecounter();
  __builtin_amdgcn_sched_barrier(0);
  float s = v0 + v1 + v2 + v3 + v4;
  for (int i = 0; i < 16; i++) s += c0[i] + c1[i];
  out[blockIdx.x * 256 + t] = s;
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *in, *out;
  long long *cyc;
  hipMalloc(&in, 1 << 20);
  hipMalloc(&out, 1 << 22);
  hipMalloc(&cyc, 8 * 1024);
  hipMemset(in, 0, 1 << 20);
  const char *names[8] = {"VGPR acc, 1 chain", "AGPR acc, 1 chain", "VGPR acc, 2 chains", "AGPR acc, 2 chains",
                          "VGPR acc, 1 chain + 5 VALU", "AGPR acc, 1 chain + 5 VALU", "VGPR acc, 2 chains + 5 VALU",
                          "AGPR acc, 2 chains + 5 VALU"};
  long long h[256];
  for (int m = 0; m < 8; m++) {
    for (int rep = 0; rep < 3; rep++) {
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
        case 7: hipLaunchKernelGGL(k<7>, dim3(256), dim3(256), 0, 0, in, out, cyc); break;
      }
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; i++) s += h[i];
    printf("%-32s %6.1f cycles per MFMA\n", names[m], s / 256 / N);
  }
  return 0;
}
