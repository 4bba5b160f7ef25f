// mlp_train.hip — fused forward + loss gradient + backward + weight gradient of
// one continuous-head Model_PPO (13 -> 32 -> 64 -> 32 -> 1, ReLU;
// Coop-MH-PPO-scalable.py:42-93) over M rows, on f32 MFMA (v_mfma_f32_32x32x2_f32,
// exact fp32 products/sums).  Replaces, per epoch and head, the torch forward
// GEMMs, autograd backward and weight-gradient GEMMs of train_model_c
// (:778-815) whose K = M reductions ran at ~15 % of HBM bandwidth.
//
// Geometry: one wave owns a 32-row tile at a time (grid-stride over tiles) and
// keeps its running weight gradient in registers; 4 waves per block share the
// weights staged in LDS (padded strides, conflict-free operand reads).
// Orientation: activations are held TRANSPOSED, H^T [features x 32 rows]: the
// MFMA C tile then has the row on the lane (l & 31) and the features in the 16
// registers (feature(r, l) = (r&3) + 8(r>>2) + 4(l>>5)), so register s of a
// layer's output is the B operand of k-step s of the next layer (k order
// feature(s, l), matched by the A-operand weight reads) — no data movement
// between layers, forward or backward.  Weight gradients sum over rows, i.e.
// need rows on the K axis: the delta and activation tiles go through a
// wave-local LDS transpose [feature][row] (stride 33) for those MFMAs; bias
// gradients are row sums of the same LDS tiles.
//
// KIND 0 (critic pass): V = net(x); writes V, accumulates (sum A, sum A^2) of
//   A = ret - V (advantage statistics, :786-787) and the MSE loss; dV = 2(V-ret)/M.
// KIND 1 (actor pass): mu = tanh(y)*std + mean; A = ((ret - V) - mean_A) /
//   (std_A + 1e-10) from the global statistics; PPO clip surrogate with float64
//   ratio (:795-806); dy = dL/dmu * std * (1 - tanh^2).
// Outputs per wave: the packed torch-layout gradient (4673 floats) and float64
// partial sums; k_grad_stage1/2 sum the per-wave partials in fixed order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "../../include/mhppo.h"
#include "common.h"
#include "rollout_dev.h"

using namespace mhppo;

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int WAVES = 8;  // one 512-thread block per CU: 2 waves per SIMD (<= 256 registers each)
constexpr int NIN = 13;
constexpr int NW = 32 * NIN + 32 + 64 * 32 + 64 + 32 * 64 + 32 + 32 + 1;  // 4673 packed params
constexpr int S1 = 15, S2 = 33, S3 = 65, ST = 33;                          // LDS row strides
// LDS layout (floats)
constexpr int O_W1 = 0, O_B1 = O_W1 + 32 * S1, O_W2 = O_B1 + 32, O_B2 = O_W2 + 64 * S2, O_W3 = O_B2 + 64,
              O_B3 = O_W3 + 32 * S3, O_W4 = O_B3 + 32, O_B4 = O_W4 + 32, O_WEND = O_B4 + 4;
constexpr int TILE = 32 * ST;  // one transposed 32x32 tile
// per-wave input slot (one 32-row tile): X [32][13], s0 = [ret 32 | V 32], s1 = [act 32 | logp_old 32]
constexpr int IN_X = 0, IN_S0 = 32 * NIN, IN_S1 = IN_S0 + 64, IN_SZ = IN_S1 + 64;
// per-wave scratch: 3 transpose tiles, then 2 input slots (double buffer filled by LDS-DMA)
constexpr int O_T = 0, O_IN = 3 * TILE;
constexpr int WAVE_LDS = O_IN + 2 * IN_SZ;
constexpr int O_DACC = O_WEND + WAVES * WAVE_LDS;        // float64 [WAVES][3][32] per-lane running sums
constexpr int LDS_FLOATS = O_DACC + WAVES * 3 * 32 * 2;  // 40420 floats = 161,680 B
static_assert(LDS_FLOATS * 4 <= 160 * 1024, "LDS budget");
static_assert(O_DACC % 2 == 0, "8-B aligned float64 sums");
static_assert(O_WEND % 4 == 0 && WAVE_LDS % 4 == 0 && O_IN % 4 == 0, "16-B aligned LDS-DMA slots");
// packed gradient offsets (torch layout)
constexpr int G_W1 = 0, G_B1 = 32 * NIN, G_W2 = G_B1 + 32, G_B2 = G_W2 + 64 * 32, G_W3 = G_B2 + 64,
              G_B3 = G_W3 + 32 * 64, G_W4 = G_B3 + 32, G_B4 = G_W4 + 32;

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int feat(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// scheduling fence between phases: keeps the scheduler from hoisting the next phase's LDS
// operand reads (and their registers) into the current one
__device__ __forceinline__ void phase() { __builtin_amdgcn_sched_barrier(0); }
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}

typedef __attribute__((address_space(3))) void lds_void;
// Raw buffer resource over [p, p + bytes): SGPR base, 32-bit VGPR lane offsets (no 64-bit
// per-lane pointers for the compiler to hoist and spill), hardware range check (loads past
// `bytes` return 0, stores past it are dropped).  dword3 = gfx9 raw-buffer format.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}
// LDS-DMA (buffer_load ... lds): lane l's dword(s) land at lds_base + l * size, lds_base
// wave-uniform (M0).  Issued from inline asm so the compiler's waitcnt pass does not see
// it: the pass cannot tell the DMA'd slot from other LDS and would put vmcnt(0) before
// every LDS read, draining the prefetch; the kernel counts vmcnt itself (wait_vmcnt).
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4i rsrc_v(const void *p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  v4i d;
  d.x = (int)(uint32_t)a;
  d.y = (int)(uint32_t)(a >> 32) & 0xffff;  // stride 0
  d.z = (int)bytes;
  d.w = 0x00020000;
  return d;
}
__device__ __forceinline__ uint32_t lds_addr(const float *p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float *)p;
}
__device__ __forceinline__ void dma16(v4i r, const float *lds_base, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(lds_addr(lds_base))
      : "memory");
}
__device__ __forceinline__ void dma4(v4i r, const float *lds_base, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(lds_addr(lds_base))
      : "memory");
}
__device__ __forceinline__ float bload(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}
// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0], expcnt[6:4] = 7, lgkmcnt[11:8] = 15); the
// compiler does not track LDS-DMA completion, so reads of a DMA'd slot wait explicitly.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N < 16, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | N);
}
__device__ __forceinline__ float relu0(float x) { return __builtin_fmaxf(x, 0.0f); }
// v[r] = relu(v[r] + b[feature(r, l)]): the 4 features of register group q are contiguous
__device__ __forceinline__ void bias_relu(f32x16 &v, const float *b, int kh) {
  const float4 *b4 = reinterpret_cast<const float4 *>(b);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    float4 c = b4[2 * q + kh];
    v[4 * q + 0] = relu0(v[4 * q + 0] + c.x);
    v[4 * q + 1] = relu0(v[4 * q + 1] + c.y);
    v[4 * q + 2] = relu0(v[4 * q + 2] + c.z);
    v[4 * q + 3] = relu0(v[4 * q + 3] + c.w);
  }
}

// store a C tile (lane = row j, registers = feature(r,l)) as T[feature][row]
__device__ __forceinline__ void put_tile(float *T, const f32x16 &v, int l) {
#pragma unroll
  for (int r = 0; r < 16; r++) T[feat(r, l) * ST + (l & 31)] = v[r];
}
// row sum of T[f][0..31] for f = l & 31 (lanes >= 32 return the same sum)
__device__ __forceinline__ float row_sum(const float *T, int l) {
  const float *p = T + (l & 31) * ST;
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 32; c++) s += p[c];
  return s;
}

// Inputs of one full 32-row tile -> an input slot, by LDS-DMA (no VGPRs, no wait here).
// X: 416 contiguous floats = 104 16-B chunks (64 + 40 lanes); s0/s1: one dword per lane,
// exec masks pick the lanes (a DMA's inactive lanes write nothing).
template <int KIND>
__device__ __forceinline__ void prefetch_tile(float *slot, const float *X, const float *ret, const float *V,
                                              const float *act, const float *lp, int64_t row0, int l) {
  const v4i rx = rsrc_v(X + row0 * NIN, 32 * NIN * 4);
  dma16(rx, slot + IN_X, 16 * l);
  if (l < 40) dma16(rx, slot + IN_X + 256, 1024 + 16 * l);
  const uint32_t vo = 4 * (l & 31);
  if (l < 32) dma4(rsrc_v(ret + row0, 128), slot + IN_S0, vo);
  if (KIND == 1) {
    if (l >= 32) dma4(rsrc_v(V + row0, 128), slot + IN_S0, vo);
    if (l < 32) dma4(rsrc_v(act + row0, 128), slot + IN_S1, vo);
    if (l >= 32) dma4(rsrc_v(lp + row0, 128), slot + IN_S1, vo);
  }
}
template <int KIND>
constexpr int prefetch_ops() { return KIND == 0 ? 3 : 6; }  // DMA instructions per prefetch

// The ragged last tile (nrows < 32): ordinary buffer loads, rows past M read as 0.
template <int KIND>
__device__ __forceinline__ void load_tile_sync(float *slot, const float *X, const float *ret, const float *V,
                                               const float *act, const float *lp, int64_t row0, int nrows, int l) {
  const auto rx = rsrc(X + row0 * NIN, (uint32_t)nrows * NIN * 4);
  for (int q = l; q < 32 * NIN; q += 64) slot[IN_X + q] = bload(rx, 4 * q);
  const uint32_t nb = 4 * nrows, vo = 4 * (l & 31);
  slot[IN_S0 + l] = bload(rsrc((l < 32 || KIND == 0) ? ret + row0 : V + row0, nb), vo);
  if (KIND == 1) slot[IN_S1 + l] = bload(rsrc(l < 32 ? act + row0 : lp + row0, nb), vo);
}

template <int KIND>
__global__ void __launch_bounds__(64 * WAVES)
    k_mlp_train(const float *__restrict__ W, const float *__restrict__ X, int64_t M, const float *__restrict__ ret,
                float *__restrict__ V, const float *__restrict__ act, const float *__restrict__ lp_old,
                const double *__restrict__ stats, double m_global, float out_mean, float out_std,
                float *__restrict__ gpart, double *__restrict__ dpart) {
  extern __shared__ float lds[];
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile bookkeeping in SGPRs
  // ---- stage weights (padded strides)
  for (int i = tid; i < 32 * NIN; i += 64 * WAVES) lds[O_W1 + (i / NIN) * S1 + i % NIN] = W[i];
  for (int i = tid; i < 32 * S1; i += 64 * WAVES)
    if (i % S1 >= NIN) lds[O_W1 + i] = 0.0f;
  for (int i = tid; i < 32; i += 64 * WAVES) lds[O_B1 + i] = W[G_B1 + i];
  for (int i = tid; i < 64 * 32; i += 64 * WAVES) lds[O_W2 + (i >> 5) * S2 + (i & 31)] = W[G_W2 + i];
  for (int i = tid; i < 64; i += 64 * WAVES) lds[O_B2 + i] = W[G_B2 + i];
  for (int i = tid; i < 32 * 64; i += 64 * WAVES) lds[O_W3 + (i >> 6) * S3 + (i & 63)] = W[G_W3 + i];
  for (int i = tid; i < 32; i += 64 * WAVES) {
    lds[O_B3 + i] = W[G_B3 + i];
    lds[O_W4 + i] = W[G_W4 + i];
  }
  if (tid == 0) lds[O_B4] = W[G_B4];
  __syncthreads();
  float *ws = lds + O_WEND + w * WAVE_LDS;
  float *T0 = ws + O_T, *T1 = T0 + TILE, *T2 = T1 + TILE;
  const float b4 = lds[O_B4];
  const int j = l & 31;
  const int kh = l >> 5;

  // persistent accumulators
  f32x16 gW1 = zero16(), gW2a = zero16(), gW2b = zero16(), gW3a = zero16(), gW3b = zero16();
  float gB1 = 0.f, gB2 = 0.f, gB3 = 0.f, gW4 = 0.f, gB4 = 0.f;
  // float64 running sums (loss, sum A, sum A^2) live in LDS, one slot per lane of the low
  // half-wave: keeping them in VGPRs spills, and a spill reload's vmcnt(0) drains the prefetch
  double *dacc = reinterpret_cast<double *>(lds + O_DACC) + w * 96 + j;
  if (kh == 0) dacc[0] = dacc[32] = dacc[64] = 0.0;
  float meanf = 0.f, stdf = 1.f;
  if (KIND == 1) {
    double mean = stats[0] / m_global;
    double var = (stats[1] - stats[0] * mean) / (m_global - 1.0);
    meanf = (float)mean;
    stdf = (float)sqrt(var > 0 ? var : 0.0);
  }
  const double inv_m = 1.0 / m_global;
  const int64_t ntiles = (M + 31) / 32, nfull = M / 32;
  const int64_t gw = (int64_t)blockIdx.x * WAVES + w, nw = (int64_t)gridDim.x * WAVES;

  int cb = 0;
  if (gw < nfull) prefetch_tile<KIND>(ws + O_IN, X, ret, V, act, lp_old, gw * 32, l);
  for (int64_t tile = gw; tile < ntiles; tile += nw, cb ^= 1) {
    const int64_t row0 = tile * 32;
    const int nrows = (int)min((int64_t)32, M - row0);
    float *slot = ws + O_IN + cb * IN_SZ;
    const int64_t nxt = tile + nw;
    if (nxt < nfull) {
      prefetch_tile<KIND>(ws + O_IN + (cb ^ 1) * IN_SZ, X, ret, V, act, lp_old, nxt * 32, l);
      wait_vmcnt<prefetch_ops<KIND>()>();  // this tile's DMA (issued one iteration earlier) has landed
    } else if (tile < nfull) {
      wait_vmcnt<0>();
    } else {
      load_tile_sync<KIND>(slot, X, ret, V, act, lp_old, row0, nrows, l);
    }
    wave_sync();
    const float *Xs = slot + IN_X;
    // ---- forward
    f32x16 h1 = zero16();
#pragma unroll
    for (int s = 0; s < 7; s++) {
      int k = 2 * s + kh;
      float a = lds[O_W1 + j * S1 + k];
      float b = (k < NIN) ? Xs[j * NIN + k] : 0.0f;
      h1 = mfma(a, b, h1);
    }
    bias_relu(h1, lds + O_B1, kh);
    phase();
    f32x16 h2a = zero16(), h2b = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = feat(s, l);
      h2a = mfma(lds[O_W2 + j * S2 + k], h1[s], h2a);
      h2b = mfma(lds[O_W2 + (32 + j) * S2 + k], h1[s], h2b);
    }
    bias_relu(h2a, lds + O_B2, kh);
    bias_relu(h2b, lds + O_B2 + 32, kh);
    phase();
    f32x16 h3 = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[O_W3 + j * S3 + feat(s, l)], h2a[s], h3);
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[O_W3 + j * S3 + 32 + feat(s, l)], h2b[s], h3);
    // h2 leaves the registers: ReLU masks as bits, h2b parked in T2 for dW3b, h2a stays
    // live only until the dW4/dB3 row sums have freed T0
    uint32_t m2 = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) m2 |= ((h2a[r] > 0.0f) ? 1u : 0u) << r | ((h2b[r] > 0.0f) ? 1u : 0u) << (16 + r);
    put_tile(T2, h2b, l);
    bias_relu(h3, lds + O_B3, kh);
    float part = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      float4 c = reinterpret_cast<const float4 *>(lds + O_W4)[2 * q + kh];
      part = fmaf(c.x, h3[4 * q], part);
      part = fmaf(c.y, h3[4 * q + 1], part);
      part = fmaf(c.z, h3[4 * q + 2], part);
      part = fmaf(c.w, h3[4 * q + 3], part);
    }
    float y = (part + __shfl_xor(part, 32)) + b4;
    // ---- loss gradient dL/dy for this lane's row
    const bool valid = j < nrows;
    float dy = 0.0f;
    if (valid) {
      float rt = slot[IN_S0 + j];
      if (KIND == 0) {
        float v = y;
        if (kh == 0) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(V + row0, 128), 4 * j, 0, 0);
        float a = rt - v;
        float d = v - rt;
        if (kh == 0) {
          dacc[0] += (double)d * (double)d;
          dacc[32] += (double)a;
          dacc[64] += (double)a * (double)a;
        }
        dy = (float)(2.0 * inv_m * (double)d);
      } else {
        float t = tanhf(y);
        float mu = t * out_std + out_mean;
        float a = rt - slot[IN_S0 + 32 + j];
        float A = (a - meanf) / (stdf + 1e-10f);
        float diff = (float)((double)slot[IN_S1 + j] - (double)mu);
        float x = diff * MVN_INV_L;
        float lp = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HALF_LOGDET;
        double r = exp((double)lp - (double)slot[IN_S1 + 32 + j]);
        double Ad = (double)A;
        double rc = r < 0.8 ? 0.8 : (r > 1.2 ? 1.2 : r);
        double s1 = r * Ad, s2 = rc * Ad, in = (r >= 0.8 && r <= 1.2) ? 1.0 : 0.0;
        double g = (s1 < s2) ? Ad : ((s2 < s1) ? in * Ad : 0.5 * Ad + 0.5 * in * Ad);
        if (kh == 0) dacc[0] += -(s1 < s2 ? s1 : s2);
        float dmu = (float)(inv_m * (-g) * r * (double)x * (double)MVN_INV_L);
        dy = (dmu * out_std) * (1.0f - t * t);
      }
    }
    gB4 += (kh == 0) ? dy : 0.0f;
    // ---- layer 4 backward: dW4 = rowsum(dy * h3), dH3 = w4 * dy masked
    f32x16 g = zero16();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      float4 c = reinterpret_cast<const float4 *>(lds + O_W4)[2 * q + kh];
      float cw[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = 4 * q + i;
        g[r] = dy * h3[r];
        h3[r] = (h3[r] > 0.0f) ? cw[i] * dy : 0.0f;  // h3 := dH3^T
      }
    }
    put_tile(T0, g, l);
    put_tile(T1, h3, l);
    wave_sync();
    phase();
    if (kh == 0) {
      gW4 += row_sum(T0, l);
      gB3 += row_sum(T1, l);
    }
    wave_sync();
    phase();
    put_tile(T0, h2a, l);
    wave_sync();
    phase();
    // dW3[:, 0:32] += dH3^T . H2a ; dW3[:, 32:64] += dH3^T . H2b
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      gW3a = mfma(T1[j * ST + k], T0[j * ST + k], gW3a);
    }
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      gW3b = mfma(T1[j * ST + k], T2[j * ST + k], gW3b);
    }
    // dH2^T = W3^T . dH3^T, masked by h2 > 0
    f32x16 d2a = zero16(), d2b = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int f = feat(s, l);
      d2a = mfma(lds[O_W3 + f * S3 + j], h3[s], d2a);
      d2b = mfma(lds[O_W3 + f * S3 + 32 + j], h3[s], d2b);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
      d2a[r] = ((m2 >> r) & 1u) ? d2a[r] : 0.0f;
      d2b[r] = ((m2 >> (16 + r)) & 1u) ? d2b[r] : 0.0f;
    }
    wave_sync();
    phase();
    put_tile(T0, d2a, l);
    put_tile(T1, d2b, l);
    put_tile(T2, h1, l);
    wave_sync();
    phase();
    gB2 += row_sum(kh ? T1 : T0, l);
    // dW2 += dH2^T . H1
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      float b = T2[j * ST + k];
      gW2a = mfma(T0[j * ST + k], b, gW2a);
      gW2b = mfma(T1[j * ST + k], b, gW2b);
    }
    // dH1^T = W2^T . dH2^T, masked by h1 > 0
    f32x16 d1 = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) d1 = mfma(lds[O_W2 + feat(s, l) * S2 + j], d2a[s], d1);
#pragma unroll
    for (int s = 0; s < 16; s++) d1 = mfma(lds[O_W2 + (32 + feat(s, l)) * S2 + j], d2b[s], d1);
#pragma unroll
    for (int r = 0; r < 16; r++) d1[r] = (h1[r] > 0.0f) ? d1[r] : 0.0f;
    wave_sync();
    phase();
    put_tile(T0, d1, l);
    wave_sync();
    phase();
    if (kh == 0) gB1 += row_sum(T0, l);
    // dW1 += dH1^T . X
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = 2 * s + kh;
      float b = (j < NIN) ? Xs[k * NIN + j] : 0.0f;
      gW1 = mfma(T0[j * ST + k], b, gW1);
    }
    wave_sync();
    phase();
  }
  // ---- write this wave's partial gradient (packed torch layout)
  float *gp = gpart + (size_t)gw * NW;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    int f = feat(r, l);
    if (j < NIN) gp[G_W1 + f * NIN + j] = gW1[r];
    gp[G_W2 + f * 32 + j] = gW2a[r];
    gp[G_W2 + (32 + f) * 32 + j] = gW2b[r];
    gp[G_W3 + f * 64 + j] = gW3a[r];
    gp[G_W3 + f * 64 + 32 + j] = gW3b[r];
  }
  if (kh == 0) {
    gp[G_B1 + j] = gB1;
    gp[G_B3 + j] = gB3;
    gp[G_W4 + j] = gW4;
  }
  gp[G_B2 + l] = gB2;  // lanes 0-31: features 0-31 (T0), lanes 32-63: 32-63 (T1)
  // b4 and float64 sums: wave reductions
  float b4s = gB4;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) b4s += __shfl_xor(b4s, o);
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  if (kh == 0) s0 = dacc[0], s1 = dacc[32], s2 = dacc[64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (l == 0) {
    gp[G_B4] = b4s;
    dpart[gw * 3 + 0] = s0;
    dpart[gw * 3 + 1] = s1;
    dpart[gw * 3 + 2] = s2;
  }
}

// Deterministic two-stage gradient reduction over the per-wave partials (fixed order,
// float64): stage 1 sums contiguous groups of waves, stage 2 sums the RG group totals.
constexpr int RG = 32;
constexpr int NWD = NW + 3;  // gradient + (loss, sum A, sum A^2)

__global__ void __launch_bounds__(256)
    k_grad_stage1(const float *gpart, const double *dpart, int nw, double *tmp) {
  int k = blockIdx.x * 256 + threadIdx.x;
  int g = blockIdx.y;
  int i0 = (int)((int64_t)g * nw / RG), i1 = (int)((int64_t)(g + 1) * nw / RG);
  double s = 0.0;
  if (k < NW) {
    for (int i = i0; i < i1; i++) s += (double)gpart[(size_t)i * NW + k];
  } else if (k < NWD) {
    for (int i = i0; i < i1; i++) s += dpart[(size_t)i * 3 + (k - NW)];
  } else {
    return;
  }
  tmp[(size_t)g * NWD + k] = s;
}

__global__ void __launch_bounds__(256) k_grad_stage2(const double *tmp, float *grad, double *out3) {
  int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= NWD) return;
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < RG; g++) s += tmp[(size_t)g * NWD + k];
  if (k < NW)
    grad[k] = (float)s;
  else if (out3)
    out3[k - NW] += s;
}

struct Work {  // per-device partial buffers (calls on one device must share one stream)
  float *g = nullptr;
  double *d = nullptr;
  double *t = nullptr;
  int nw = 0;
};
Work g_work[16];

int grid_waves() {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return cus * WAVES;  // one block of 8 waves per CU
}
}  // namespace

extern "C" int mhppo_mlp_train_cont(int kind, const float *packed, const float *X, int64_t M, const float *ret,
                                    float *value, const float *act, const float *logp_old, const double *stats,
                                    double m_global, float out_mean, float out_std, float *grad, double *sums,
                                    void *stream) {
  if (!packed || !X || !ret || !value || !grad || M < 0 || (kind != 0 && kind != 1))
    return set_error(MHPPO_EINVAL, "bad argument");
  if (kind == 1 && (!act || !logp_old || !stats)) return set_error(MHPPO_EINVAL, "actor pass needs act/logp/stats");
  if (((uintptr_t)X & 15) != 0) return set_error(MHPPO_EINVAL, "X must be 16-byte aligned (LDS-DMA rows)");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  Work &wk = g_work[dev & 15];
  int nw = grid_waves();
  if (M > 0) nw = (int)min((int64_t)nw, ((M + 31) / 32 + WAVES - 1) / WAVES * WAVES);
  if (nw < WAVES) nw = WAVES;
  if (wk.nw < nw) {
    if (wk.g) (void)hipFree(wk.g);
    if (wk.d) (void)hipFree(wk.d);
    if (wk.t) (void)hipFree(wk.t);
    if (hipMalloc(&wk.g, sizeof(float) * (size_t)nw * NW) != hipSuccess ||
        hipMalloc(&wk.d, sizeof(double) * (size_t)nw * 3) != hipSuccess ||
        hipMalloc(&wk.t, sizeof(double) * (size_t)RG * NWD) != hipSuccess) {
      wk = Work{};
      return set_error(MHPPO_ENOMEM, "mlp_train partials");
    }
    wk.nw = nw;
  }
  dim3 grid(nw / WAVES), blk(64 * WAVES);
  size_t shm = sizeof(float) * LDS_FLOATS;
  if (kind == 0)
    hipLaunchKernelGGL(k_mlp_train<0>, grid, blk, shm, s, packed, X, M, ret, value, act, logp_old, stats, m_global,
                       out_mean, out_std, wk.g, wk.d);
  else
    hipLaunchKernelGGL(k_mlp_train<1>, grid, blk, shm, s, packed, X, M, ret, value, act, logp_old, stats, m_global,
                       out_mean, out_std, wk.g, wk.d);
  hipLaunchKernelGGL(k_grad_stage1, dim3((NWD + 255) / 256, RG), dim3(256), 0, s, wk.g, wk.d, nw, wk.t);
  hipLaunchKernelGGL(k_grad_stage2, dim3((NWD + 255) / 256), dim3(256), 0, s, wk.t, grad, sums);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}
