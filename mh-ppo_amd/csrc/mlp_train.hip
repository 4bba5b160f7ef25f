// mlp_train.hip — fused forward + loss gradient + backward + weight gradient of one
// Model_PPO head (n_in -> 32 -> 64 -> 32 -> n_out, ReLU; Coop-MH-PPO-scalable.py:42-93)
// over M rows, on f32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products/sums).
// Replaces, per epoch and head, the torch forward GEMMs, autograd backward and the
// K = M weight-gradient GEMMs of train_model_c / train_model_d (:778-851).
//
// Geometry: one wave owns a 32-row tile at a time (grid-stride over tiles) and keeps
// its running weight gradient in registers; the waves of a block share the weights
// staged in LDS (padded strides, conflict-free operand reads).
// Orientation: activations are held TRANSPOSED, H^T [features x 32 rows]: the MFMA C
// tile has the row on the lane (l & 31) and the features in the 16 registers
// (feature(r, l) = (r&3) + 8(r>>2) + 4(l>>5)), so register s of a layer's output is the
// B operand of k-step s of the next layer (k order feature(s, l), matched by the
// A-operand weight reads) — no data movement between layers, forward or backward.
// Weight gradients sum over rows, i.e. need rows on the K axis: the delta and
// activation tiles go through a wave-local LDS transpose [feature][row] (stride 33) for
// those MFMAs; bias gradients are row sums of the same LDS tiles.
//
// Kinds (the loss the head is trained on):
//   K_CRITIC  V = net(x); writes V, accumulates (sum A, sum A^2) of A = G - V (the
//             advantage statistics, :786-787 / :825-826) and the MSE loss; dV = 2(V-G)/M.
//   K_CONT    continuous actor: mu = tanh(y)*std + mean; A normalised from the GLOBAL
//             statistics; MVN log-prob, float64 ratio, clip surrogate (:795-806);
//             dy = dL/dmu * std * (1 - tanh^2).
//   K_CHOICE  choice actor: p = softmax(y0, y1); the reference's M x M Categorical
//             broadcast (:828-842) in its exact O(M) form: each row contributes
//             sum_k counts[k] * f(r_k, A) with r_k = p_k / exp(logp_old); dL/dp through the
//             pn = p / sum(p) normalisation and the clamp, then the softmax Jacobian.
// Continuous heads (13 inputs, the big batches) run 8 waves per CU (2 per SIMD) with the
// next tile's inputs prefetched into a double-buffered LDS slot by LDS-DMA; the other
// instantiations (choice obs of 12..64 features, small batches) load synchronously; their
// dW1 is one 32x32 tile per 32 input columns.
// Outputs per wave: the packed torch-layout gradient and float64 partial sums;
// k_grad_stage1/2 sum the per-wave partials in fixed order (deterministic).
#include <hip/hip_runtime.h>
#include <math.h>

#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "../../include/mhppo.h"
#include "common.h"
#include "rollout_dev.h"

using namespace mhppo;

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { K_CRITIC = 0, K_CONT = 1, K_CHOICE = 2 };
constexpr int NIN_CONT = 13;
constexpr int S2 = 33, S3 = 65, ST = 33;  // LDS row strides (W2, W3, transpose tiles)
constexpr int TILE = 32 * ST;             // one transposed 32x32 tile

__host__ __device__ constexpr int n_params(int nin, int nout) {
  return 32 * nin + 32 + 64 * 32 + 64 + 32 * 64 + 32 + nout * 32 + nout;
}
constexpr int NIN_MAX = 64;  // choice heads: dc = 2 + 6(S-1) + 10 = 54 for the scalable 8-slot env
constexpr int NW_MAX = n_params(NIN_MAX, 2);

// LDS layout (floats) of one instantiation: KS = layer-1 k-steps (inputs padded to 2 KS),
// PF = double-buffered DMA prefetch (13-input heads), NOUT = output width.
template <int KS, bool PF, int NOUT>
struct Lay {
  static constexpr int WAVES = PF ? 8 : 4;  // PF: 2 waves/SIMD (<= 256 VGPRs); else 1
  static constexpr int S1 = 2 * KS + 1;     // odd W1 row stride
  static constexpr int O_W1 = 0, O_B1 = 32 * S1, O_W2 = O_B1 + 32, O_B2 = O_W2 + 64 * S2, O_W3 = O_B2 + 64,
                       O_B3 = O_W3 + 32 * S3, O_W4 = O_B3 + 32, O_B4 = O_W4 + 32 * NOUT,
                       O_WEND = (O_B4 + NOUT + 3) / 4 * 4;
  // per-wave input slot: X [32][n_in], s0 = [ret 32 | V 32], s1 = [act or logp_old 32 | logp_old 32]
  static constexpr int XMAX = PF ? 32 * NIN_CONT : 64 * KS;
  // PF: 32 floats of pad after s1 take the unpredicated DMAs' overhang (prefetch_tile)
  static constexpr int IN_X = 0, IN_S0 = XMAX, IN_S1 = IN_S0 + 64, IN_SZ = IN_S1 + 64 + (PF ? 32 : 0);
  static constexpr int NSLOT = PF ? 2 : 1;
  // per-wave scratch: 3 transpose tiles, then the input slot(s)
  static constexpr int O_T = 0, O_IN = 3 * TILE, WAVE_LDS = O_IN + NSLOT * IN_SZ;
  static constexpr int O_DACC = O_WEND + WAVES * WAVE_LDS;  // float64 [WAVES][3][32]
  static constexpr int FLOATS = O_DACC + WAVES * 3 * 32 * 2;
  static_assert(FLOATS * 4 <= 160 * 1024, "LDS budget");
  static_assert(O_WEND % 4 == 0 && WAVE_LDS % 4 == 0 && O_IN % 4 == 0 && IN_SZ % 4 == 0, "16-B aligned slots");
};

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int feat(int r, int l) { return (r & 3) + 8 * (r >> 2) + 4 * (l >> 5); }
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// scheduling fence between phases: keeps the scheduler from hoisting the next phase's LDS
// operand reads (and their registers) into the current one
#ifndef MHPPO_NO_PHASE
__device__ __forceinline__ void phase() { __builtin_amdgcn_sched_barrier(0); }
#else
__device__ __forceinline__ void phase() {}
#endif
// wave-uniform values pinned to SGPRs (the compiler otherwise holds some in VGPRs)
__device__ __forceinline__ float uniform_f(float x) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ int64_t uniform_i64(int64_t x) {
  const uint64_t u = (uint64_t)x;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double uniform_d(double x) {
  return __longlong_as_double(uniform_i64(__double_as_longlong(x)));
}
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
// s_waitcnt vmcnt(N) (gfx9 encoding: vmcnt[3:0], expcnt[6:4] = 7, lgkmcnt[11:8] = 15)
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
// the C-layout broadcast of a per-feature vector b (register r of lane half kh = b[feature]):
// a bias as an MFMA chain's initial accumulator, or w4 for the output layer
// x[l] + x[l ^ 32] (the two half-wave partial sums of a row) through v_permlane32_swap: no LDS
// round trip on the loss section's serial chain (ds_bpermute's latency).  The same bits as
// x + __shfl_xor(x, 32): lanes 32-63 add the same two values in the other order.
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ f32x16 feat_vec(const float *b, int kh) {
  const float4 *b4 = reinterpret_cast<const float4 *>(b);
  f32x16 v;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const float4 c = b4[2 * q + kh];
    v[4 * q + 0] = c.x;
    v[4 * q + 1] = c.y;
    v[4 * q + 2] = c.z;
    v[4 * q + 3] = c.w;
  }
  return v;
}
// ReLU of an MFMA result as one integer max on the bits (signed compare orders non-negative
// floats like their values and sends every negative one, -0 included, to +0); fmaxf would
// first canonicalize the register (a second VALU op per element)
__device__ __forceinline__ float relu_bits(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
__device__ __forceinline__ void relu16(f32x16 &v) {
#pragma unroll
  for (int r = 0; r < 16; r++) v[r] = relu_bits(v[r]);
}
// sum_r w[feature(r, l)] * h[r] over this lane's 16 features
__device__ __forceinline__ float dot16(const float *w, const f32x16 &h, int kh) {
  float part = 0.0f;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    float4 c = reinterpret_cast<const float4 *>(w)[2 * q + kh];
    part = fmaf(c.x, h[4 * q], part);
    part = fmaf(c.y, h[4 * q + 1], part);
    part = fmaf(c.z, h[4 * q + 2], part);
    part = fmaf(c.w, h[4 * q + 3], part);
  }
  return part;
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
// Every DMA's buffer range is bounded by the rows the batch really has past row0 (M): a tile index
// past the batch (a prefetch-ring or tile-loop indexing error) reads zeros instead of touching
// memory outside the buffers (the raw-buffer range check bounds the offset from the base; with a
// zero range nothing is fetched, whatever the base).  Full tiles: the same 32-row ranges.
__device__ __forceinline__ uint32_t tile_rows(int64_t M, int64_t row0) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)max((int64_t)0, min((int64_t)32, M - row0)));
}
template <int KIND, class LY>
__device__ __forceinline__ void prefetch_tile(float *slot, const float *X, const float *ret, const float *V,
                                              const float *act, const float *lp, int64_t row0, int l, int64_t M) {
  const uint32_t rows = tile_rows(M, row0);
  const v4i rx = rsrc_v(X + row0 * NIN_CONT, rows * NIN_CONT * 4);
  // Every DMA on all 64 lanes (no exec-mask branches): an LDS-DMA lane writes base + 4 lane, so
  // the lanes past a piece's end land in the NEXT piece's place (or the 32-float pad after s1),
  // reading zeros past their buffer's bounds; the pieces are issued in address order and their
  // LDS writes land in issue order, so each overhang is overwritten by the piece it covers.
  dma16(rx, slot + LY::IN_X, 16 * l);
  dma16(rx, slot + LY::IN_X + 256, 1024 + 16 * l);  // X 256..415; lanes 40-63: zeros into s0
  const uint32_t vo = 4 * l;
  dma4(rsrc_v(ret + row0, 4 * rows), slot + LY::IN_S0, vo);  // ret [0, 32); lanes 32-63: zeros [32, 64)
  if (KIND == K_CONT) {
    dma4(rsrc_v(V + row0, 4 * rows), slot + LY::IN_S0 + 32, vo);   // V [32, 64); overhang into s1
    dma4(rsrc_v(act + row0, 4 * rows), slot + LY::IN_S1, vo);      // act [0, 32); overhang [32, 64)
    dma4(rsrc_v(lp + row0, 4 * rows), slot + LY::IN_S1 + 32, vo);  // logp_old [32, 64); overhang: pad
  }
}
template <int KIND>
constexpr int prefetch_ops() { return KIND == K_CRITIC ? 3 : 6; }  // DMA instructions per prefetch

// Tile inputs through registers: load_tile_regs issues every load of a 32-row tile (X rows,
// the s0/s1 targets) with none waiting on another; store_tile_regs writes them to the wave's
// input slot.  A runtime-trip-count load -> store loop would wait one memory round trip per 64
// floats (15 per tile at n_in = 30).  Rows past M read as 0 (buffer bounds).
template <class LY>
struct TileRegs {
  float x[(LY::XMAX + 63) / 64];
  float s0, s1;
};
template <int KIND, class LY>
__device__ __forceinline__ void load_tile_regs(TileRegs<LY> &t, const float *X, int nin, const float *ret,
                                               const float *V, const float *act, const float *lp, int64_t row0,
                                               int nrows, int l) {
  const auto rx = rsrc(X + row0 * nin, (uint32_t)(nrows * nin) * 4);
#pragma unroll
  for (int i = 0; i < (LY::XMAX + 63) / 64; i++) {
    const int q = l + 64 * i;
    t.x[i] = q < 32 * nin ? bload(rx, 4 * q) : 0.0f;
  }
  const uint32_t nb = 4 * nrows, vo = 4 * (l & 31);
  t.s0 = bload(rsrc((l < 32 || KIND == K_CRITIC) ? ret + row0 : V + row0, nb), vo);
  t.s1 = 0.0f;
  if (KIND == K_CONT) t.s1 = bload(rsrc(l < 32 ? act + row0 : lp + row0, nb), vo);
  if (KIND == K_CHOICE)  // [logp_old 32 | action 32] (the action is read only in per-row mode)
    t.s1 = bload(rsrc((l < 32 || act == nullptr) ? lp + row0 : act + row0, nb), vo);
}
template <int KIND, class LY>
__device__ __forceinline__ void store_tile_regs(float *slot, const TileRegs<LY> &t, int nin, int l) {
#pragma unroll
  for (int i = 0; i < (LY::XMAX + 63) / 64; i++) {
    const int q = l + 64 * i;
    if (q < 32 * nin) slot[LY::IN_X + q] = t.x[i];
  }
  slot[LY::IN_S0 + l] = t.s0;
  if (KIND == K_CONT || KIND == K_CHOICE) slot[LY::IN_S1 + l] = t.s1;
}
// Synchronous tile load (ragged last tile of the DMA path)
template <int KIND, class LY>
__device__ __forceinline__ void load_tile_sync(float *slot, const float *X, int nin, const float *ret,
                                               const float *V, const float *act, const float *lp, int64_t row0,
                                               int nrows, int l) {
  TileRegs<LY> t;
  load_tile_regs<KIND, LY>(t, X, nin, ret, V, act, lp, row0, nrows, l);
  store_tile_regs<KIND, LY>(slot, t, nin, l);
}

template <int KIND, int KS, bool PF>
__global__ void __launch_bounds__(PF ? 512 : 256)  // 64 * Lay::WAVES
    k_mlp_train(const float *__restrict__ W, const float *__restrict__ X, int nin, int64_t M,
                const float *__restrict__ ret, float *__restrict__ V, const float *__restrict__ act,
                const float *__restrict__ lp_old, const double *__restrict__ stats,
                const double *__restrict__ counts, double m_global, float out_mean, float out_std,
                float *__restrict__ gpart, double *__restrict__ dpart) {
  constexpr int NOUT = KIND == K_CHOICE ? 2 : 1;
  using LY = Lay<KS, PF, NOUT>;
  // 13-input heads: 13 < 2 KS = 14, so layer 1 has a free input column for the bias
  constexpr bool FOLD_B1 = PF;
  constexpr int WAVES = LY::WAVES;
  extern __shared__ float lds[];
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: tile bookkeeping in SGPRs
  if (PF) nin = NIN_CONT;
  // packed torch-layout offsets
  const int G_W1 = 0, G_B1 = 32 * nin, G_W2 = G_B1 + 32, G_B2 = G_W2 + 64 * 32, G_W3 = G_B2 + 64,
            G_B3 = G_W3 + 32 * 64, G_W4 = G_B3 + 32, G_B4 = G_W4 + 32 * NOUT, NWP = G_B4 + NOUT;
  // ---- stage weights (padded strides, zero padding).  Every global load is issued before
  // the first LDS store (one memory round trip; a strided load -> store loop per array costs
  // one dependent trip per iteration, ~24 per launch).
  {
    constexpr int NT = 64 * WAVES, N1 = (32 * LY::S1 + NT - 1) / NT, N2 = 2048 / NT;
    static_assert(2048 % NT == 0 && NT >= 64, "staging: block size");
    float v1[N1], v2[N2], v3[N2];
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int i = tid + q * NT, r = i / LY::S1, c = i % LY::S1;
      // FOLD_B1: b1 rides in the padding column nin of W1 against a constant-1 input
      v1[q] = i >= 32 * LY::S1 ? 0.0f
                               : (c < nin ? W[G_W1 + r * nin + c] : ((FOLD_B1 && c == nin) ? W[G_B1 + r] : 0.0f));
    }
#pragma unroll
    for (int q = 0; q < N2; q++) {
      v2[q] = W[G_W2 + tid + q * NT];
      v3[q] = W[G_W3 + tid + q * NT];
    }
    const float vb1 = tid < 32 ? W[G_B1 + tid] : 0.0f, vb3 = tid < 32 ? W[G_B3 + tid] : 0.0f;
    const float vb2 = tid < 64 ? W[G_B2 + tid] : 0.0f, vw4 = tid < 32 * NOUT ? W[G_W4 + tid] : 0.0f;
    const float vb4 = tid < NOUT ? W[G_B4 + tid] : 0.0f;
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int i = tid + q * NT;
      if (i < 32 * LY::S1) lds[LY::O_W1 + i] = v1[q];
    }
#pragma unroll
    for (int q = 0; q < N2; q++) {
      const int i = tid + q * NT;
      lds[LY::O_W2 + (i >> 5) * S2 + (i & 31)] = v2[q];
      lds[LY::O_W3 + (i >> 6) * S3 + (i & 63)] = v3[q];
    }
    if (tid < 32) {
      lds[LY::O_B1 + tid] = vb1;
      lds[LY::O_B3 + tid] = vb3;
    }
    if (tid < 64) lds[LY::O_B2 + tid] = vb2;
    if (tid < 32 * NOUT) lds[LY::O_W4 + tid] = vw4;
    if (tid < NOUT) lds[LY::O_B4 + tid] = vb4;
  }
  __syncthreads();
  float *ws = lds + LY::O_WEND + w * LY::WAVE_LDS;
  float *T0 = ws + LY::O_T, *T1 = T0 + TILE, *T2 = T1 + TILE;
  const float b40 = lds[LY::O_B4], b41 = NOUT == 2 ? lds[LY::O_B4 + 1] : 0.0f;
  const int j = l & 31;
  const int kh = l >> 5;

  // persistent accumulators (gW1b: input columns 32..63 of dW1, heads with n_in > 32)
  constexpr bool W1B = !PF && 2 * KS > 32;
  f32x16 gW1 = zero16(), gW1b = zero16(), gW2a = zero16(), gW2b = zero16(), gW3a = zero16(), gW3b = zero16();
  // 13-input heads: dW1 = dH1^T X is [32 features x 14 columns] — two 16x16 tiles of the
  // 16x16x4 MFMA (half the cycles of one 32x32 tile); D row (l>>4)*4 + r, column l & 15
  f32x4 gW1q[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  float gB1 = 0.f, gB2 = 0.f, gB3 = 0.f, gW40 = 0.f, gW41 = 0.f, gB40 = 0.f, gB41 = 0.f;
  // float64 running sums (loss, sum A, sum A^2) live in LDS, one slot per lane of the low
  // half-wave: keeping them in VGPRs spills, and a spill reload's vmcnt(0) drains the prefetch
  double *dacc = reinterpret_cast<double *>(lds + LY::O_DACC) + w * 96 + j;
  if (kh == 0) dacc[0] = dacc[32] = dacc[64] = 0.0;
  float meanf = 0.f, stdf = 1.f;
  if (KIND != K_CRITIC) {
    double mean = stats[0] / m_global;
    double var = (stats[1] - stats[0] * mean) / (m_global - 1.0);
    meanf = (float)mean;
    stdf = (float)sqrt(var > 0 ? var : 0.0);
  }
  const double inv_m = 1.0 / m_global;
  const int64_t ntiles = (M + 31) / 32, nfull = PF ? M / 32 : 0;
  const int64_t gw = (int64_t)blockIdx.x * WAVES + w, nw = (int64_t)gridDim.x * WAVES;

  int cb = 0;
  MHPPO_MARK(0);
  if (PF && gw < nfull) prefetch_tile<KIND, LY>(ws + LY::O_IN, X, ret, V, act, lp_old, gw * 32, l, M);
  TileRegs<LY> tnext;  // non-PF: the next tile's inputs in registers
  if (!PF && gw < ntiles)
    load_tile_regs<KIND, LY>(tnext, X, nin, ret, V, act, lp_old, gw * 32, (int)min((int64_t)32, M - gw * 32), l);
  for (int64_t tile = gw; tile < ntiles; tile += nw, cb ^= (PF ? 1 : 0)) {
    const int64_t row0 = tile * 32;
    const int nrows = (int)min((int64_t)32, M - row0);
    float *slot = ws + LY::O_IN + cb * LY::IN_SZ;
    if constexpr (PF) {
      const int64_t nxt = tile + nw;
      if (nxt < nfull) {
        prefetch_tile<KIND, LY>(ws + LY::O_IN + (cb ^ 1) * LY::IN_SZ, X, ret, V, act, lp_old, nxt * 32, l, M);
        wait_vmcnt<prefetch_ops<KIND>()>();  // this tile's DMA (issued one iteration earlier) has landed
      } else if (tile < nfull) {
        wait_vmcnt<0>();
      } else {
        load_tile_sync<KIND, LY>(slot, X, nin, ret, V, act, lp_old, row0, nrows, l);
      }
    } else {
      // this tile's inputs were loaded into registers one iteration earlier (the first tile's
      // before the loop); the next tile's loads are in flight during this tile's compute
      store_tile_regs<KIND, LY>(slot, tnext, nin, l);
      const int64_t nt = tile + nw;
      if (nt < ntiles)
        load_tile_regs<KIND, LY>(tnext, X, nin, ret, V, act, lp_old, nt * 32, (int)min((int64_t)32, M - nt * 32), l);
    }
    wave_sync();
    MHPPO_MARK(1);  // tile inputs landed
    const float *Xs = slot + LY::IN_X;
    // ---- forward
    f32x16 h1 = zero16();
#pragma unroll
    for (int s = 0; s < KS; s++) {
      int k = 2 * s + kh;
      float a = lds[LY::O_W1 + j * LY::S1 + k];
      float b = (k < nin) ? Xs[j * nin + k] : ((FOLD_B1 && k == nin) ? 1.0f : 0.0f);
      h1 = mfma(a, b, h1);
    }
    if constexpr (FOLD_B1) {  // the last fmaf of the chain added b1 (fma(b, 1, acc) == acc + b)
#pragma unroll
      for (int r = 0; r < 16; r++) h1[r] = relu0(h1[r]);
    } else {
      bias_relu(h1, lds + LY::O_B1, kh);
    }
    phase();
    f32x16 h2a = zero16(), h2b = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) {
      int k = feat(s, l);
      h2a = mfma(lds[LY::O_W2 + j * S2 + k], h1[s], h2a);
      h2b = mfma(lds[LY::O_W2 + (32 + j) * S2 + k], h1[s], h2b);
    }
    bias_relu(h2a, lds + LY::O_B2, kh);
    bias_relu(h2b, lds + LY::O_B2 + 32, kh);
    phase();
    f32x16 h3 = zero16();
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[LY::O_W3 + j * S3 + feat(s, l)], h2a[s], h3);
#pragma unroll
    for (int s = 0; s < 16; s++) h3 = mfma(lds[LY::O_W3 + j * S3 + 32 + feat(s, l)], h2b[s], h3);
    // h2 leaves the registers: ReLU masks as bits, h2b parked in T2 for dW3b, h2a stays
    // live only until the dW4/dB3 row sums have freed T0
    uint32_t m2 = 0;
#pragma unroll
    for (int r = 0; r < 16; r++) m2 |= ((h2a[r] > 0.0f) ? 1u : 0u) << r | ((h2b[r] > 0.0f) ? 1u : 0u) << (16 + r);
    put_tile(T2, h2b, l);
    bias_relu(h3, lds + LY::O_B3, kh);
    float part0 = dot16(lds + LY::O_W4, h3, kh);
    const float y0 = (part0 + __shfl_xor(part0, 32)) + b40;
    float y1 = 0.0f;
    if constexpr (NOUT == 2) {
      float part1 = dot16(lds + LY::O_W4 + 32, h3, kh);
      y1 = (part1 + __shfl_xor(part1, 32)) + b41;
    }
    MHPPO_MARK(2);  // forward
    // ---- loss gradient dL/dy for this lane's row
    const bool valid = j < nrows;
    float dy0 = 0.0f, dy1 = 0.0f;
    if (valid) {
      const float rt = slot[LY::IN_S0 + j];
      if constexpr (KIND == K_CRITIC) {
        const float v = y0;
        // the store's range is the tile's rows in the batch: no lane can write past the batch
        if (kh == 0) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(V + row0, 4 * nrows), 4 * j, 0, 0);
        const float a = rt - v;
        const float d = v - rt;
        if (kh == 0) {
          dacc[0] += (double)d * (double)d;
          dacc[32] += (double)a;
          dacc[64] += (double)a * (double)a;
        }
        dy0 = (float)(2.0 * inv_m * (double)d);
      } else if constexpr (KIND == K_CONT) {
        const float t = tanhf(y0);
        const float mu = t * out_std + out_mean;
        const float a = rt - slot[LY::IN_S0 + 32 + j];
        const float A = (a - meanf) / (stdf + 1e-10f);
        const float diff = (float)((double)slot[LY::IN_S1 + j] - (double)mu);
        const float x = diff * MVN_INV_L;
        const float lp = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HALF_LOGDET;
        const double r = exp((double)lp - (double)slot[LY::IN_S1 + 32 + j]);
        double dfdr;
        const double f = surr_and_grad(r, (double)A, dfdr);
        if (kh == 0) dacc[0] += f;
        const float dmu = (float)(inv_m * dfdr * r * (double)x * (double)MVN_INV_L);
        dy0 = (dmu * out_std) * (1.0f - t * t);
      } else {
        // softmax over the pair (as torch: shift by the max), pn = p / (p0 + p1)
        const float mx = fmaxf(y0, y1);
        const float e0 = expf(y0 - mx), e1 = expf(y1 - mx);
        const float se = e0 + e1;
        const float p[2] = {e0 / se, e1 / se};
        const float a = rt - slot[LY::IN_S0 + 32 + j];
        const float A = (a - meanf) / (stdf + 1e-10f);
        const double old = (double)slot[LY::IN_S1 + j];
        const float sp = p[0] + p[1];
        const float pn[2] = {p[0] / sp, p[1] / sp};
        const float eps = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
        const double inv_m2 = inv_m * inv_m;
        // reference: every row meets every action with the global counts (the M x M
        // broadcast); per-row mode (counts == NULL, opt-in bug fix): the row's own action
        // with weight M_global, i.e. the standard mean over rows of the PPO surrogate
        const int a_row = counts ? 0 : (int)slot[LY::IN_S1 + 32 + j];
        double dlp[2], f = 0.0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const double w = counts ? counts[k] : (k == a_row ? m_global : 0.0);
          const float pc = pn[k] < eps ? eps : (pn[k] > hi ? hi : pn[k]);
          const double r = exp((double)logf(pc) - old);
          double dfdr;
          const double fk = surr_and_grad(r, (double)A, dfdr);
          if (w != 0.0) f += w * fk;
          const double pass = (pn[k] >= eps && pn[k] <= hi) ? 1.0 : 0.0;
          dlp[k] = inv_m2 * w * dfdr * r * pass / (double)pc;  // dL/dpn_k
        }
        if (kh == 0) dacc[0] += f;
        const double sd = (double)sp;
        const double g0 = (dlp[0] * (1.0 - pn[0]) - dlp[1] * pn[1]) / sd;  // dL/dp_k
        const double g1 = (dlp[1] * (1.0 - pn[1]) - dlp[0] * pn[0]) / sd;
        const double dot = (double)p[0] * g0 + (double)p[1] * g1;
        dy0 = (float)((double)p[0] * (g0 - dot));  // softmax Jacobian
        dy1 = (float)((double)p[1] * (g1 - dot));
      }
    }
    MHPPO_MARK(3);  // loss gradient
    gB40 += (kh == 0) ? dy0 : 0.0f;
    gB41 += (kh == 0) ? dy1 : 0.0f;
    // ---- layer 4 backward: dW4 = rowsum(dy * h3), dH3 = W4^T dy masked
    f32x16 g = zero16(), g1v = zero16();
#pragma unroll
    for (int q = 0; q < 4; q++) {
      float4 c = reinterpret_cast<const float4 *>(lds + LY::O_W4)[2 * q + kh];
      float cw[4] = {c.x, c.y, c.z, c.w};
      float cw1[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (NOUT == 2) {
        float4 c1 = reinterpret_cast<const float4 *>(lds + LY::O_W4 + 32)[2 * q + kh];
        cw1[0] = c1.x, cw1[1] = c1.y, cw1[2] = c1.z, cw1[3] = c1.w;
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const int r = 4 * q + i;
        g[r] = dy0 * h3[r];
        if constexpr (NOUT == 2) {
          g1v[r] = dy1 * h3[r];
          h3[r] = (h3[r] > 0.0f) ? fmaf(cw1[i], dy1, cw[i] * dy0) : 0.0f;  // h3 := dH3^T
        } else {
          h3[r] = (h3[r] > 0.0f) ? cw[i] * dy0 : 0.0f;
        }
      }
    }
    put_tile(T0, g, l);
    put_tile(T1, h3, l);
    wave_sync();
    phase();
    if (kh == 0) {
      gW40 += row_sum(T0, l);
      gB3 += row_sum(T1, l);
    }
    if constexpr (NOUT == 2) {
      wave_sync();
      put_tile(T0, g1v, l);
      wave_sync();
      if (kh == 0) gW41 += row_sum(T0, l);
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
      d2a = mfma(lds[LY::O_W3 + f * S3 + j], h3[s], d2a);
      d2b = mfma(lds[LY::O_W3 + f * S3 + 32 + j], h3[s], d2b);
    }
#pragma unroll
    for (int r = 0; r < 16; r++) {
      d2a[r] = ((m2 >> r) & 1u) ? d2a[r] : 0.0f;
      d2b[r] = ((m2 >> (16 + r)) & 1u) ? d2b[r] : 0.0f;
    }
    MHPPO_MARK(4);  // layer-4 backward, dW3 + dH2
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
    for (int s = 0; s < 16; s++) d1 = mfma(lds[LY::O_W2 + feat(s, l) * S2 + j], d2a[s], d1);
#pragma unroll
    for (int s = 0; s < 16; s++) d1 = mfma(lds[LY::O_W2 + (32 + feat(s, l)) * S2 + j], d2b[s], d1);
#pragma unroll
    for (int r = 0; r < 16; r++) d1[r] = (h1[r] > 0.0f) ? d1[r] : 0.0f;
    MHPPO_MARK(5);  // dW2 + dH1
    wave_sync();
    phase();
    put_tile(T0, d1, l);
    wave_sync();
    phase();
    if (!FOLD_B1 && kh == 0) gB1 += row_sum(T0, l);  // FOLD_B1: column nin of dW1 is dB1
    // dW1 += dH1^T . X
    if constexpr (PF) {  // rows 4s..4s+3 per step, ascending: the same fmaf chain order
#pragma unroll
      for (int s = 0; s < 8; s++) {
        const int rr = 4 * s + (l >> 4), jj = l & 15;
        const float b = (jj < nin) ? Xs[rr * nin + jj] : ((FOLD_B1 && jj == nin) ? 1.0f : 0.0f);
#pragma unroll
        for (int ft = 0; ft < 2; ft++) gW1q[ft] = mfma16(T0[(16 * ft + (l & 15)) * ST + rr], b, gW1q[ft]);
      }
    } else {
#pragma unroll
      for (int s = 0; s < 16; s++) {
        int k = 2 * s + kh;
        float b = (j < nin) ? Xs[k * nin + j] : ((FOLD_B1 && j == nin) ? 1.0f : 0.0f);
        gW1 = mfma(T0[j * ST + k], b, gW1);
      }
      if constexpr (W1B) {
#pragma unroll
        for (int s = 0; s < 16; s++) {
          int k = 2 * s + kh;
          float b = (32 + j < nin) ? Xs[k * nin + 32 + j] : 0.0f;
          gW1b = mfma(T0[j * ST + k], b, gW1b);
        }
      }
    }
    wave_sync();
    phase();
    MHPPO_MARK(6);  // dW1 (timing builds only)
  }
  MHPPO_MARK_FLUSH();
  // ---- write this wave's partial gradient (packed torch layout)
  float *gp = gpart + (size_t)gw * NWP;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    int f = feat(r, l);
    if (!PF && j < nin) gp[G_W1 + f * nin + j] = gW1[r];
    if (W1B && 32 + j < nin) gp[G_W1 + f * nin + 32 + j] = gW1b[r];
    gp[G_W2 + f * 32 + j] = gW2a[r];
    gp[G_W2 + (32 + f) * 32 + j] = gW2b[r];
    gp[G_W3 + f * 64 + j] = gW3a[r];
    gp[G_W3 + f * 64 + 32 + j] = gW3b[r];
  }
  if constexpr (PF) {
#pragma unroll
    for (int ft = 0; ft < 2; ft++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int f = 16 * ft + (l >> 4) * 4 + r, jj = l & 15;
        if (jj < nin) gp[G_W1 + f * nin + jj] = gW1q[ft][r];
        if (FOLD_B1 && jj == nin) gp[G_B1 + f] = gW1q[ft][r];
      }
  }
  if (kh == 0) {
    if (!FOLD_B1) gp[G_B1 + j] = gB1;
    gp[G_B3 + j] = gB3;
    gp[G_W4 + j] = gW40;
    if (NOUT == 2) gp[G_W4 + 32 + j] = gW41;
  }
  gp[G_B2 + l] = gB2;  // lanes 0-31: features 0-31 (T0), lanes 32-63: 32-63 (T1)
  // b4 and float64 sums: wave reductions
  float b4s0 = gB40, b4s1 = gB41;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    b4s0 += __shfl_xor(b4s0, o);
    b4s1 += __shfl_xor(b4s1, o);
  }
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  if (kh == 0) s0 = dacc[0], s1 = dacc[32], s2 = dacc[64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s0 += __shfl_xor(s0, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if (l == 0) {
    gp[G_B4] = b4s0;
    if (NOUT == 2) gp[G_B4 + 1] = b4s1;
    dpart[gw * 3 + 0] = s0;
    dpart[gw * 3 + 1] = s1;
    dpart[gw * 3 + 2] = s2;
  }
}

// =====================================================================================
// Split-precision path of the 13-input heads (critic / continuous actor, the big batches).
// Every GEMM of the pass runs on bf16 MFMA (v_mfma_f32_32x32x16_bf16: 16x the f32-MFMA
// rate) with each f32 operand split EXACTLY into three bf16 parts, x = hi + mid + lo
// (round-to-nearest at each level: |mid| <= 2^-8 |x|, |lo| <= 2^-16 |x|), and the six
// products of combined order <= 2 accumulated in f32: the dropped terms are <= 2^-24
// relative, i.e. the accuracy of an f32 product (the f32-MFMA kernel above stays the exact
// k-ordered-fmaf reference, MHPPO_TRAIN_EXACT_F32).
// Orientation as above (activations transposed, C registers of one layer = B operand of
// the next with the permuted k order feature(16s + 8(j>>2) + 4h + (j&3)) of register
// 8s + j).  Weights: row-major bf16 images [out][in] per part in LDS with padded rows (odd
// multiples of 8 bytes: conflict-free row reads, linear addresses): the forward A fragments
// are two 8-byte row reads, the backward (W^T) ones two ds_read_b64_tr_b16 transposed reads
// of the same image.  Weight gradients sum over the tile's 32 rows: both operands go
// through one per-wave bf16 image [row][feature] of the split parts, read back transposed.
// Bias gradients and dW4 are f32 row sums through the same LDS slot.
// The continuous actor's ratio: its magnitude r = expf(lp - logp_old) in float32, its clip branch
// decided on the float64 difference lp - logp_old (surr_and_grad_fd: the decision of the
// reference's float64 ratio, Coop-MH-PPO-scalable.py:803-806), not a float64 exp.  The float64
// exp's temporaries kept W3's forward fragments out of the actor's registers (X3_ACT 63 fits at
// 510 VGPRs without them): cfg3 iteration -1.4 % over three interleaved bench pairs
// (profiles/r05_floss/); the float64-exp build on r06 driver-length benches: +1.1 % per iteration
// and the same gradient to 3 digits at bench scale with 23 % of the rows clipped
// (profiles/r06_a/).  Numerics: lp - logp_old in float32 is exact only while the two are within a
// factor 2 of each other (Sterbenz), which updates do not guarantee row by row, so r carries up to
// two float32 roundings (~1.2e-7 relative) — the level of the difference mu itself has from the
// reference's CPU GEMM; the clip decision carries none.  dmu's product stays
// float64 with one rounding: a float32 chain of four roundings there moved the 2-rank vs 1-rank
// nets of tests/test_dp_gpu.py from <= 7.6e-7 to 6.4e-5 (tools/dp_diff.py).  The exact f32
// kernel keeps the float64 ratio.

namespace x3 {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

struct F3 {  // one MFMA operand fragment (8 elements) as its three bf16 parts
  u32x4 p[3];
};

// row strides (bytes) of the bf16 images: odd multiples of 8 B over the data width
constexpr int W2_ROWB = 72, W3_ROWB = 136, IM_ROWB = 72;
constexpr int W2_PART = 64 * W2_ROWB, W3_PART = 32 * W3_ROWB, IM_PART = 32 * IM_ROWB;
constexpr int IMG = 3 * IM_PART;    // one tile image (three parts) = the per-wave LDS slot
constexpr int TS = 36;              // f32 transpose image row stride (floats; 16-B aligned rows)
static_assert(32 * TS * 4 <= IMG, "the f32 image shares the slot");
constexpr int WAVES = 4;  // one wave per SIMD (512 registers)

// Geometry of one split-precision net: K1 = layer-1 K (the inputs and the bias column, padded to
// whole 16-deep K-steps), NOUT outputs, NIC the compile-time input count (0: a kernel argument,
// nin <= NMX, by default K1 - 1).  LDS: the net's weights (bf16 images of W1..W3, f32 b2 b3 w4
// b4), then per wave: the tile image (also the f32 transpose image), two input slots (double
// buffered), a second tile image.
template <int K1_, int NOUT_, int NIC_, int NIM_ = 2, int NMX_ = K1_ - 1>
struct Geo {
  static constexpr int K1 = K1_, KS1 = K1 / 16, NOUT = NOUT_, NIC = NIC_, NIM = NIM_, NMX = NMX_;
  static_assert(K1 % 16 == 0 && (NIC == 0 || NIC < K1) && NMX < K1, "layer-1 geometry");
  static constexpr int W1_ROWB = 2 * K1 + 8, W1_PART = 32 * W1_ROWB;
  static constexpr int O_W1 = 0, O_W2 = O_W1 + 3 * W1_PART, O_W3 = O_W2 + 3 * W2_PART, O_F = O_W3 + 3 * W3_PART;
  static constexpr int F_W4 = 96, F_B4 = F_W4 + 32 * NOUT, NF = F_B4 + NOUT;  // f32: b2[64] b3[32] w4 b4
  static constexpr int NET_B = (O_F + NF * 4 + 15) / 16 * 16;
  // input slot (floats): X [32][nin] | s0 [32 | 32] | s1 [32 | 32].  A runtime nin gets an X region
  // of whole 1-KiB pieces, so every LDS-DMA piece lands unmasked (zeros past the rows).
  static constexpr int XMAX = NIC == NIN_CONT ? (32 * NIC + 3) / 4 * 4 : (32 * (NIC ? NIC : NMX) + 255) / 256 * 256;
  static constexpr int IN_X = 0, IN_S0 = XMAX, IN_S1 = XMAX + 64, IN_SZ = XMAX + 128 + (NIC ? 32 : 0);
  static constexpr int XPIECES = (XMAX * 4 + 1023) / 1024;
  // NIM tile-image slots per wave: slot 1 at 0, slot 2 at O_IM2, slots 3 and 4 after it (the
  // hand-placed passes write the forward's h1 / h2a images during the forward, into slots of their own)
  static constexpr int IMGA = (IMG + 15) / 16 * 16;
  static constexpr int O_IN = IMGA, O_IM2 = O_IN + 2 * IN_SZ * 4, O_IM3 = O_IM2 + IMGA, O_IM4 = O_IM3 + IMGA,
                       WAVE_B = O_IM2 + (NIM - 1) * IMGA;
  static constexpr int LDS_BYTES = NET_B + WAVES * WAVE_B;
  static constexpr int LDS_BYTES_PAIR = 2 * NET_B + WAVES * WAVE_B;  // two nets' weights (pair kernel)
  static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
  static_assert(WAVE_B % 16 == 0 && O_IN % 16 == 0 && IN_SZ % 4 == 0, "16-B aligned slots");
};
// the 13-input continuous heads (the big batches): the slot layout of the f32 path's Lay<7, true, 1>
using G13 = Geo<16, 1, NIN_CONT>;
using G13S = Geo<16, 1, NIN_CONT, 4>;  // the hand-placed single-net passes (four image slots per wave)
using LY = Lay<7, true, 1>;
static_assert(G13::IN_S0 == LY::IN_S0 && G13::IN_S1 == LY::IN_S1 && G13::IN_SZ == LY::IN_SZ, "13-input slot");
static_assert(G13::LDS_BYTES_PAIR <= 160 * 1024, "LDS budget (pair)");
// the choice heads' nets on this kernel: up to NIN_X3C inputs (wider ones stay on the f32 kernel).
// K = 64 (the scalable 8-slot env's dc = 54, Coop-MH-PPO-scalable.py:818-851): the input slots sized
// for 54 inputs (7 KiB of X rows), the four waves' slots and the weights then fit the 160 KiB of LDS
constexpr int NIN_X3C = 54;
using GC16 = Geo<16, 2, 0>;
using GV16 = Geo<16, 1, 0>;
using GC32 = Geo<32, 2, 0>;
using GV32 = Geo<32, 1, 0>;
using GC64 = Geo<64, 2, 0, 2, NIN_X3C>;
using GV64 = Geo<64, 1, 0, 2, NIN_X3C>;
// dc = 54 itself with a compile-time input count: the runtime count's address arithmetic spilled
// the choice actor (15 VGPRs at 512); compile-time: 496 VGPRs, no spill
using GC54 = Geo<64, 2, 54, 2, 54>;
using GV54 = Geo<64, 1, 54, 2, 54>;

#ifdef MHPPO_X3_PHASE
__device__ __forceinline__ void x3_phase() { __builtin_amdgcn_sched_barrier(0); }
#else
__device__ __forceinline__ void x3_phase() {}
#endif
// LDS image round trips within one wave: a wave's LDS instructions execute in issue order,
// so only the compiler must keep the write -> read order (no lgkmcnt drain)
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float x, float y) {  // one v_cvt_pk_bf16_f32
  const f32x2 v = {x, y};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// x - (the bf16 in the low / high half of h, as f32): the residual of a split level (exact: x and
// the bf16 rounding of x differ by a representable amount).  (One v_dot2c_f32_bf16 against
// (-1, 0) / (0, -1) instead of the back-conversion + subtraction pair: 1 437 instead of 1 560
// instructions per critic tile but +85 s_nop and +53 v_mov, train launch +6 %,
// profiles/r06_x3/ab_dot2_split.txt, tools/patches/x3_r06_dot2_split.patch.)
__device__ __forceinline__ float res_lo(uint32_t h, float x) { return x - __uint_as_float(h << 16); }
__device__ __forceinline__ float res_hi(uint32_t h, float y) { return y - __uint_as_float(h & 0xffff0000u); }
// (x, y) -> three packed bf16 pairs, x = hi + mid + lo exactly (element 0 in the low half)
__device__ __forceinline__ void split_pair(float x, float y, uint32_t &h, uint32_t &m, uint32_t &lo) {
  h = pk_bf16(x, y);
  const float x1 = res_lo(h, x), y1 = res_hi(h, y);
  m = pk_bf16(x1, y1);
  lo = pk_bf16(res_lo(m, x1), res_hi(m, y1));
}
// fragment element j = v[j]
__device__ __forceinline__ F3 split8(const float *v) {
  F3 f;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t a, b, c;
    split_pair(v[2 * q], v[2 * q + 1], a, b, c);
    f.p[0][q] = a;
    f.p[1][q] = b;
    f.p[2][q] = c;
  }
  return f;
}
// K-step s of a C tile (registers 8s .. 8s+7) as a B (or A) fragment
__device__ __forceinline__ F3 split_step(const f32x16 &c, int s) {
  float v[8];
#pragma unroll
  for (int q = 0; q < 8; q++) v[q] = c[8 * s + q];
  return split8(v);
}

__device__ __forceinline__ f32x16 mfma_b(u32x4 a, u32x4 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                  0, 0);
}
// C += A B on split operands: the six products of combined order <= 2, smallest first
__device__ __forceinline__ f32x16 mfma6(const F3 &a, const F3 &b, f32x16 c) {
  c = mfma_b(a.p[2], b.p[0], c);
  c = mfma_b(a.p[0], b.p[2], c);
  c = mfma_b(a.p[1], b.p[1], c);
  c = mfma_b(a.p[1], b.p[0], c);
  c = mfma_b(a.p[0], b.p[1], c);
  return mfma_b(a.p[0], b.p[0], c);
}

__device__ __forceinline__ f32x4 mfma_b16(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                  0, 0);
}
__device__ __forceinline__ f32x4 mfma6_16(const F3 &a, const F3 &b, f32x4 c) {
  c = mfma_b16(a.p[2], b.p[0], c);
  c = mfma_b16(a.p[0], b.p[2], c);
  c = mfma_b16(a.p[1], b.p[1], c);
  c = mfma_b16(a.p[1], b.p[0], c);
  c = mfma_b16(a.p[0], b.p[1], c);
  return mfma_b16(a.p[0], b.p[0], c);
}
// Weight-gradient accumulation C += A B (six products, as mfma6) with the accumulator pinned
// to AGPRs: it is touched by nothing but these MFMAs inside the loop, so it never moves
// between the register files and the arch VGPRs stay free for the tile's values.  Written as
// one asm block: "s_nop 1" covers the VALU-write -> MFMA-read hazard on A / B (the compiler
// cannot see the MFMAs inside), and back-to-back accumulation into the same AGPRs needs none.
#define X3_MACC6_BODY(OP)                                                                                \
  "s_nop 1\n\t" OP " %0, %3, %4, %0\n\t" OP " %0, %1, %6, %0\n\t" OP " %0, %2, %5, %0\n\t" OP " %0, %2, %4, %0\n\t" OP \
  " %0, %1, %5, %0\n\t" OP " %0, %1, %4, %0"                                                                      \
      : "+a"(c)                                                                                                      \
      : "v"(a.p[0]), "v"(a.p[1]), "v"(a.p[2]), "v"(b.p[0]), "v"(b.p[1]), "v"(b.p[2])
#define X3_MACC6(OP) asm(X3_MACC6_BODY(OP))
__device__ __forceinline__ void macc6(const F3 &a, const F3 &b, f32x16 &c) { X3_MACC6("v_mfma_f32_32x32x16_bf16"); }
__device__ __forceinline__ void macc6_16(const F3 &a, const F3 &b, f32x4 &c) { X3_MACC6("v_mfma_f32_16x16x32_bf16"); }
#undef X3_MACC6
// C += A B (six products, as macc6) with the next fragment's six transposed image reads issued
// in the MFMA gaps (an LDS read between two 32x32x16 MFMAs costs the wave almost nothing, a run
// of them costs their issue and puts their latency in front of the MFMAs that need them).  The
// compiler does not see these reads: WAIT puts an lgkmcnt(0) in front of a block whose B
// fragment came from the previous block's reads (LDS returns in order, so the compiler's own
// counted waits stay sufficient with them in flight).  nx <- image K-step rows at rbase + off.
#define X3_MACC6_RD(NAME, ACC, OP)                                                                          \
  template <bool WAIT, int OFF>                                                                              \
  __device__ __forceinline__ void NAME(const F3 &a, const F3 &b, ACC &c, F3 &nx, const char *rbase) {       \
    constexpr int U = 4 * IM_ROWB;                                                                           \
    const uint32_t ad = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char *)rbase;         \
    uint2 r0, r1, r2, r3, r4, r5;                                                                            \
    if constexpr (WAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                  \
    asm volatile("s_nop 1\n\t" OP " %0, %9, %10, %0\n\tds_read_b64_tr_b16 %1, %13 offset:%14\n\t" OP          \
                 " %0, %7, %12, %0\n\tds_read_b64_tr_b16 %2, %13 offset:%15\n\t" OP                           \
                 " %0, %8, %11, %0\n\tds_read_b64_tr_b16 %3, %13 offset:%16\n\t" OP                           \
                 " %0, %8, %10, %0\n\tds_read_b64_tr_b16 %4, %13 offset:%17\n\t" OP                           \
                 " %0, %7, %11, %0\n\tds_read_b64_tr_b16 %5, %13 offset:%18\n\t" OP                           \
                 " %0, %7, %10, %0\n\tds_read_b64_tr_b16 %6, %13 offset:%19"                                 \
                 : "+a"(c), "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5)                 \
                 : "v"(a.p[0]), "v"(a.p[1]), "v"(a.p[2]), "v"(b.p[0]), "v"(b.p[1]), "v"(b.p[2]), "v"(ad),    \
                   "i"(OFF), "i"(OFF + U), "i"(OFF + IM_PART), "i"(OFF + IM_PART + U), "i"(OFF + 2 * IM_PART), \
                   "i"(OFF + 2 * IM_PART + U)                                                                \
                 : "memory");                                                                                \
    nx.p[0] = u32x4{r0.x, r0.y, r1.x, r1.y};                                                                  \
    nx.p[1] = u32x4{r2.x, r2.y, r3.x, r3.y};                                                                  \
    nx.p[2] = u32x4{r4.x, r4.y, r5.x, r5.y};                                                                  \
  }
X3_MACC6_RD(macc6_rd, f32x16, "v_mfma_f32_32x32x16_bf16")
X3_MACC6_RD(macc6_16_rd, f32x4, "v_mfma_f32_16x16x32_bf16")
#undef X3_MACC6_RD
// the last block of a chain: wait for its asm-read fragment, then the six MFMAs — ONE volatile
// statement: as two, the compiler may hoist the (non-volatile) MFMA block above the wait, and the
// MFMAs then read registers whose LDS data is still in flight (tools/check_asm_rd.py found
// exactly that in the actor's last dW3 block before this was one statement)
#define X3_MACC6_W(OP) asm volatile("s_waitcnt lgkmcnt(0)\n\t" X3_MACC6_BODY(OP) : "memory")
__device__ __forceinline__ void macc6_w(const F3 &a, const F3 &b, f32x16 &c) { X3_MACC6_W("v_mfma_f32_32x32x16_bf16"); }
__device__ __forceinline__ void macc6_16_w(const F3 &a, const F3 &b, f32x4 &c) { X3_MACC6_W("v_mfma_f32_16x16x32_bf16"); }
#undef X3_MACC6_W
#undef X3_MACC6_BODY
// C += A B for a B whose mid / lo parts are zero (the one-hot bias-sum columns: bf16 1.0 is exact),
// three products, smallest first, accumulator in AGPRs.  Volatile: its A may be a fragment an
// earlier asm block read, and it must stay behind the wait that completed it.
__device__ __forceinline__ void macc3(const F3 &a, const u32x4 &b, f32x16 &c) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %3, %4, %0\n\tv_mfma_f32_32x32x16_bf16 %0, %2, %4, %0\n\t"
               "v_mfma_f32_32x32x16_bf16 %0, %1, %4, %0"
               : "+a"(c)
               : "v"(a.p[0]), "v"(a.p[1]), "v"(a.p[2]), "v"(b));
}
// before the accumulators are read: the last MFMA's result latency (>= 18 passes)
__device__ __forceinline__ void macc_drain(f32x16 &a, f32x16 &b, f32x16 &c, f32x16 &d, f32x4 &e, f32x4 &f) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(a), "+a"(b), "+a"(c), "+a"(d), "+a"(e), "+a"(f));
}
__device__ __forceinline__ void macc_drain2(f32x16 &a, f32x16 &b, f32x16 &c, f32x16 &d, f32x4 &e, f32x4 &f,
                                            f32x4 &g, f32x4 &h) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(a), "+a"(b), "+a"(c), "+a"(d), "+a"(e), "+a"(f), "+a"(g),
               "+a"(h));
}
__device__ __forceinline__ uint2 lds_u2(const char *p) { return *reinterpret_cast<const uint2 *>(p); }
__device__ __forceinline__ uint2 tr16(const char *p) {
  v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16 *)(p));
  return __builtin_bit_cast(uint2, v);
}
// two 8-byte reads (at p and p + du) of each part -> fragment elements 0-3 / 4-7
template <int PART>
__device__ __forceinline__ F3 rd_pair(const char *p, int du) {
  F3 f;
#pragma unroll
  for (int pt = 0; pt < 3; pt++) {
    const uint2 a = lds_u2(p + pt * PART), b = lds_u2(p + pt * PART + du);
    f.p[pt] = u32x4{a.x, a.y, b.x, b.y};
  }
  return f;
}
template <int PART>
__device__ __forceinline__ F3 tr_pair(const char *p, int du) {
  F3 f;
#pragma unroll
  for (int pt = 0; pt < 3; pt++) {
    const uint2 a = tr16(p + pt * PART), b = tr16(p + pt * PART + du);
    f.p[pt] = u32x4{a.x, a.y, b.x, b.y};
  }
  return f;
}
// Lane address bases (loop invariants; every fragment is base + a compile-time offset):
//  row read   (forward A of W, lane row r, half h): r * ROWB + 8 h; K-step s, u -> + 8 (4s + 2u)
//  transposed (W^T A / image B, lane 16G + 4q + p): (4 (G>>1) + q) * ROWB... see below
// Forward A fragment of W (rows `out` = base row + 32 t), K-step s, permuted k order:
// element j <- in feature 16s + 8(j>>2) + 4h + (j&3), i.e. 8-byte chunk 4s + 2u + h.
template <int ROWB, int PART>
__device__ __forceinline__ F3 w_fwd(const char *rowbase, int t, int s) {
  return rd_pair<PART>(rowbase + t * 32 * ROWB + 32 * s, 16);
}
// Backward A fragment of W^T (lane: in feature 32t + (l & 31)), K-step s over the out
// features in the permuted order: element j <- W[16s + 8(j>>2) + 4h + (j&3)][in]; lane
// 4q + p of group G addresses row 16s + 8u + 4(G>>1) + q, chunk 8t + 4(G&1) + p
// (trbase = W + (4 (G>>1) + q) * ROWB + 8 (4 (G&1) + p)).
template <int ROWB, int PART>
__device__ __forceinline__ F3 w_bwd(const char *trbase, int t, int s) {
  return tr_pair<PART>(trbase + 16 * s * ROWB + 64 * t, 8 * ROWB);
}
// Tile image [32 rows][32 features] of a C tile given as its two split K-step fragments:
// lane (row r, half h) writes register group g (features 8g + 4h .. +3) as chunk 2g + h
// (wbase = img + r * IM_ROWB + 8 h).
template <int PART = IM_PART>
__device__ __forceinline__ void img_write(char *wbase, const F3 &f0, const F3 &f1) {
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const F3 &f = g < 2 ? f0 : f1;
    const int q = 2 * (g & 1);
#pragma unroll
    for (int pt = 0; pt < 3; pt++)
      *reinterpret_cast<uint2 *>(wbase + pt * PART + 16 * g) = make_uint2(f.p[pt][q], f.p[pt][q + 1]);
  }
}
// one part (hi / mid / lo) of img_write: two 16-byte row stores per lane (the hand-placed passes
// spread an image's parts over MFMA shadows: at most two LDS stores or three reads per shadow keep
// the LDS pipe from stalling the issue, MI355X_MICROARCH.md §LDS)
__device__ __forceinline__ void img_write_pt(char *wbase, const F3 &f0, const F3 &f1, int pt) {
#pragma unroll
  for (int g = 0; g < 4; g++) {
    const F3 &f = g < 2 ? f0 : f1;
    const int q = 2 * (g & 1);
    *reinterpret_cast<uint2 *>(wbase + pt * IM_PART + 16 * g) = make_uint2(f.p[pt][q], f.p[pt][q + 1]);
  }
}
// one half of img_write_pt: ONE 16-byte-per-lane LDS store (a ds_write2_b64), register groups 2 hf
// and 2 hf + 1 of part pt (f = f0 for hf 0, f1 for hf 1).  The hand-placed passes issue an image as
// six of these, at most one per two MFMA shadows: with four waves storing, a store after every MFMA
// costs each wave 27 cycles per store, two after every MFMA 95, one after every second MFMA nothing
// (tools/probes/lds_store_mfma.hip, profiles/r05_lds_store/)
__device__ __forceinline__ void img_write_h(char *wbase, const F3 &f, int pt, int hf) {
  *reinterpret_cast<uint2 *>(wbase + pt * IM_PART + 32 * hf) = make_uint2(f.p[pt][0], f.p[pt][1]);
  *reinterpret_cast<uint2 *>(wbase + pt * IM_PART + 32 * hf + 16) = make_uint2(f.p[pt][2], f.p[pt][3]);
}
// one part of a transposed fragment read (tr_pair): two ds_read_b64_tr_b16
__device__ __forceinline__ void tr_pt(const char *p, int du, int pt, F3 &f) {
  const uint2 a = tr16(p + pt * IM_PART), b = tr16(p + pt * IM_PART + du);
  f.p[pt] = u32x4{a.x, a.y, b.x, b.y};
}
// K-step s (rows 16s .. 16s+15) of the image read transposed: lane (feature l & 31, half h)
// gets rows 16s + 8h + j, j = 0..7; lane 4q + p of group G addresses row 16s + 8(G>>1) +
// 4u + q, chunk 4(G&1) + p (rbase = img + (8 (G>>1) + q) * IM_ROWB + 8 (4 (G&1) + p)).
__device__ __forceinline__ F3 img_read(const char *rbase, int s) {
  return tr_pair<IM_PART>(rbase + 16 * s * IM_ROWB, 4 * IM_ROWB);
}
// f32 transpose image T[feature][row] (stride TS) of a C tile, and the half-row sum of
// feature (l & 31) over rows 16h .. 16h+15 (the halves are combined once, at the end)
__device__ __forceinline__ void put_t(float *T, const f32x16 &v, int l) {
  float *b = T + 4 * (l >> 5) * TS + (l & 31);  // lane base; register r at a constant offset
#pragma unroll
  for (int r = 0; r < 16; r++) b[((r & 3) + 8 * (r >> 2)) * TS] = v[r];
}
#define X3_ROWSUM(k, v) \
  do {                   \
    put_t(T, v, l);      \
    lds_order();         \
    radd(k, half_row_sum(T, l)); \
    lds_order();         \
  } while (0)
__device__ __forceinline__ float half_row_sum(const float *T, int l) {
  const float4 *p = reinterpret_cast<const float4 *>(T + (l & 31) * TS + 16 * (l >> 5));
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const float4 v = p[c];
    s += v.x;
    s += v.y;
    s += v.z;
    s += v.w;
  }
  return s;
}
// stage one f32 weight element (split) into a row-major bf16 image
__device__ __forceinline__ void stage_w(char *Wimg, int part, int rowb, int row, int col, float w) {
  const __bf16 hi = (__bf16)w;
  const float r1 = w - (float)hi;
  const __bf16 mid = (__bf16)r1;
  const __bf16 lo = (__bf16)(r1 - (float)mid);
  const int off = row * rowb + col * 2;
  *reinterpret_cast<__bf16 *>(Wimg + off) = hi;
  *reinterpret_cast<__bf16 *>(Wimg + part + off) = mid;
  *reinterpret_cast<__bf16 *>(Wimg + 2 * part + off) = lo;
}
// d = (h > 0) ? d : 0 (ReLU derivative)
__device__ __forceinline__ void relu_mask(f32x16 &d, const f32x16 &h) {
#pragma unroll
  for (int r = 0; r < 16; r++) d[r] = h[r] > 0.0f ? d[r] : 0.0f;
}
}  // namespace x3

namespace x3 {
// ---- Hand-placed backward (SCH passes): each block of MFMAs carries the NEXT block's VALU / LDS
// work in its MFMA shadows.  One wave per SIMD issues in order: a run of back-to-back MFMAs leaves
// the vector issue idle for 24 of every 32 cycles, a run of VALU leaves the matrix pipe idle, and
// the compiler cannot place VALU between the MFMAs of an opaque inline-asm block.  So every MFMA
// is its own statement and `weave` cuts the block into regions (sched_barrier: nothing crosses),
// region k = MFMA k + a share of the payload units, spread evenly (unit u in region u NMU / NU).
template <int B, int E, class F>
__device__ __forceinline__ void sfor(F &&f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}
// A payload plan: segments {first region, end region, units}, the units numbered in segment order
// and spread evenly over their segment's regions (unit t of a segment in r0 + t (r1 - r0) / n).
template <int... S>
struct Plan {
  static constexpr int NS = sizeof...(S) / 3;
  static constexpr int s[sizeof...(S)] = {S...};
  static constexpr int units() {
    int n = 0;
    for (int i = 0; i < NS; i++) n += s[3 * i + 2];
    return n;
  }
  static constexpr int NU = units();
  static constexpr int reg(int u) {  // the region of unit u
    for (int i = 0; i < NS; i++) {
      const int n = s[3 * i + 2];
      if (u < n) return s[3 * i] + u * (s[3 * i + 1] - s[3 * i]) / n;
      u -= n;
    }
    return -1;
  }
  static constexpr int first(int seg) {  // the first unit of segment seg
    int n = 0;
    for (int i = 0; i < seg; i++) n += s[3 * i + 2];
    return n;
  }
  static_assert(sizeof...(S) % 3 == 0, "plan: {r0, r1, units} triples");
};
// region k = MFMA k (mf(k)), then the payload units the plan puts in region k; nothing crosses a
// region border (sched_barrier)
template <int NM, class PL, class M, class U>
__device__ __forceinline__ void weave(M &&mf, U &&un) {
  static_assert(PL::NU == 0 || PL::reg(PL::NU - 1) < NM, "plan: units past the block's last region");
  sfor<0, NM>([&](auto kc) {
    constexpr int K = decltype(kc)::value;
    mf(kc);
    sfor<0, PL::NU>([&](auto uc) {
      if constexpr (PL::reg(decltype(uc)::value) == K) un(uc);
    });
    __builtin_amdgcn_sched_barrier(0);
  });
}
// the six products of a split x split MFMA (mfma6 order, smallest first) and the three of a
// split x one-hot one (macc3)
constexpr int P6A[6] = {2, 0, 1, 1, 0, 0}, P6B[6] = {0, 2, 1, 0, 1, 0};
// one weight-gradient MFMA, accumulator in AGPRs (volatile: kept in its region).  Its A / B come
// from LDS reads (or loop-invariant registers), never from a VALU write just before it: no wait
// states needed (tools/check_asm_rd.py checks the built code)
__device__ __forceinline__ void mac1(const u32x4 &a, const u32x4 &b, f32x16 &c) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// the bias-sum MFMA: B = a loop-invariant one-hot fragment, kept in AGPRs (an MFMA reads A / B from
// either file; as "v" the compiler would copy it from the AGPR it parks it in right before the MFMA,
// a VALU write the MFMA then reads without its two wait states)
__device__ __forceinline__ void mac1_oh(const u32x4 &a, const u32x4 &oh, f32x16 &c) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "a"(oh));
}
__device__ __forceinline__ void mac1_16(const u32x4 &a, const u32x4 &b, f32x4 &c) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
// The regions hold because the train translation unit is built with the source-order SelectionDAG
// scheduler (csrc/Makefile: -pre-RA-sched=source): instruction selection keeps each payload unit
// where the source puts it, and the machine scheduler never moves an instruction across a region
// barrier.  (Pinning the units with empty volatile asm statements instead cost one copy and one
// wait state per pinned value.)
// opaque loaded values: unconditional loads (hipcc otherwise turns `cond ? load : const` into a
// branch around the load); all of a unit's loads are pinned in ONE statement, after the last one
// is issued, so they wait once, together
__device__ __forceinline__ void pin4(float *v) { asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3])); }
// split level 1 of element pair q of an 8-element fragment v: hi part, residuals r[2q], r[2q+1]
__device__ __forceinline__ void split_l1(const float *v, int q, F3 &f, float *r) {
  const uint32_t h = pk_bf16(v[2 * q], v[2 * q + 1]);
  f.p[0][q] = h;
  r[2 * q] = res_lo(h, v[2 * q]);
  r[2 * q + 1] = res_hi(h, v[2 * q + 1]);
}
// split levels 2-3 of pair q from its residuals (as split_pair: the same bits)
__device__ __forceinline__ void split_l2(int q, F3 &f, const float *r) {
  const uint32_t m = pk_bf16(r[2 * q], r[2 * q + 1]);
  f.p[1][q] = m;
  f.p[2][q] = pk_bf16(res_lo(m, r[2 * q]), res_hi(m, r[2 * q + 1]));
}
// ReLU-derivative mask of elements r, r + 1 of d by h > 0
__device__ __forceinline__ void mask2(f32x16 &d, const f32x16 &h, int r) {
  d[r] = h[r] > 0.0f ? d[r] : 0.0f;
  d[r + 1] = h[r + 1] > 0.0f ? d[r + 1] : 0.0f;
}
__device__ __forceinline__ void relu4(f32x16 &h, int r0) {
#pragma unroll
  for (int r = r0; r < r0 + 4; r++) h[r] = relu_bits(h[r]);
}
}  // namespace x3

// One wave per SIMD (512 registers: the weight-gradient accumulators and the loop-invariant
// weight fragments sit in AGPRs).  Measured alternatives: two waves per SIMD at
// 256 registers (no hoisted fragments, h1 recomputed: 12 % slower), two tiles per wave in lock
// step (spills), a software-pipelined loop (backward of tile i beside the forward of tile i+1:
// 10 % slower).
namespace x3 {
// packed torch-layout offsets of one Model_PPO (W1 b1 W2 b2 W3 b3 W4 b4)
struct Packed {
  int W1, B1, W2, B2, W3, B3, W4, B4, NP;
  __host__ __device__ constexpr Packed(int nin, int nout)
      : W1(0), B1(32 * nin), W2(B1 + 32), B2(W2 + 64 * 32), W3(B2 + 64), B3(W3 + 32 * 64), W4(B3 + 32),
        B4(W4 + 32 * nout), NP(B4 + nout) {}
};
template <class G>
__device__ __forceinline__ int geo_nin(int nin_rt) { return G::NIC ? G::NIC : nin_rt; }

// Stage one net's weights at Lw: bf16 images (three parts), b1 as input column nin of W1.  Every
// global load is issued before the first LDS store (one memory round trip per launch; a strided
// load -> split -> store loop per array costs one dependent trip per iteration).
template <class G>
__device__ __forceinline__ void stage_net(const float *__restrict__ W, char *Lw, int tid, int nin_rt) {
  const int nin = geo_nin<G>(nin_rt);
  const Packed P(nin, G::NOUT);
  constexpr int K1 = G::K1, NF = G::NF;
  float *F = reinterpret_cast<float *>(Lw + G::O_F);  // b2 [0, 64) b3 [64, 96) w4 [96, ...) b4
  constexpr int NT = 64 * WAVES, N1 = (32 * K1 + NT - 1) / NT, N2 = 2048 / NT, NFQ = (NF + NT - 1) / NT;
  static_assert(2048 % NT == 0, "staging: block size");
  float v1[N1], v2[N2], v3[N2], vf[NFQ];
#pragma unroll
  for (int q = 0; q < N1; q++) {
    const int i = tid + q * NT, r = i / K1, c = i % K1;
    v1[q] = i >= 32 * K1 ? 0.0f : (c < nin ? W[P.W1 + r * nin + c] : (c == nin ? W[P.B1 + r] : 0.0f));
  }
#pragma unroll
  for (int q = 0; q < N2; q++) {
    v2[q] = W[P.W2 + tid + q * NT];
    v3[q] = W[P.W3 + tid + q * NT];
  }
#pragma unroll
  for (int q = 0; q < NFQ; q++) {
    const int i = tid + q * NT;
    vf[q] = i < 64 ? W[P.B2 + i]
                   : (i < 96 ? W[P.B3 + i - 64]
                             : (i < G::F_B4 ? W[P.W4 + i - 96] : (i < NF ? W[P.B4 + i - G::F_B4] : 0.f)));
  }
#pragma unroll
  for (int q = 0; q < N1; q++) {
    const int i = tid + q * NT;
    if (i < 32 * K1) stage_w(Lw + G::O_W1, G::W1_PART, G::W1_ROWB, i / K1, i % K1, v1[q]);
  }
#pragma unroll
  for (int q = 0; q < N2; q++) {
    const int i = tid + q * NT;
    stage_w(Lw + G::O_W2, W2_PART, W2_ROWB, i >> 5, i & 31, v2[q]);
    stage_w(Lw + G::O_W3, W3_PART, W3_ROWB, i >> 6, i & 63, v3[q]);
  }
#pragma unroll
  for (int q = 0; q < NFQ; q++) {
    const int i = tid + q * NT;
    if (i < NF) F[i] = vf[q];
  }
}

// The per-wave lane geometry of the wave's LDS slot (images, f32 transpose image, input slots)
template <class GEO>
struct WaveSlot {
  char *wb;          // this wave's image / f32 transpose slot
  float *T;          // f32 transpose image (shares the slot)
  float *inb;        // input slots (double buffered)
  char *imw;         // image write base
  const char *imr;   // image transposed-read base (32x32x16 operands)
  const char *imr16; // image transposed-read base (16x16x32 operands)
  int l, j, kh, G;
  __device__ __forceinline__ WaveSlot(char *L8, int w, int l_) : l(l_), j(l_ & 31), kh(l_ >> 5), G(l_ >> 4) {
    const int q4 = (l >> 2) & 3, p4 = l & 3;
    wb = L8 + w * GEO::WAVE_B;
    T = reinterpret_cast<float *>(wb);
    inb = reinterpret_cast<float *>(wb + GEO::O_IN);
    imw = wb + j * IM_ROWB + 8 * kh;
    // image reads: rows 8 (G >> 1) + 4u + q, chunk 4 (G & 1) + p
    imr = wb + (8 * (G >> 1) + q4) * IM_ROWB + 8 * (4 * (G & 1) + p4);
    imr16 = wb + (8 * G + q4) * IM_ROWB + 8 * p4;  // 16x16x32 A: rows 8G + 4u + q, chunk 4t + p
  }
};

// One net's pass over 32-row tiles (forward, loss gradient, backward, weight gradients), with its
// per-wave state: lane bases into its staged weights, the loop-invariant weight fragments, the
// weight-gradient accumulators and the bias / loss sums.  HF: the forward weight fragments are
// held in registers too (one critic pass alone; the actor pass's loss, and a second net in the
// same wave, need those registers) — and then dW2 cannot carry its image reads in its MFMA gaps.
// HB: the backward (W^T) fragments are held in registers (not with two nets in one wave).
// G: the net's geometry (inputs, outputs); K_CHOICE: the choice actor (two outputs, softmax pair).
#ifndef MHPPO_X3_W4R
#define MHPPO_X3_W4R 1  // A/B builds override
#endif
constexpr bool X3_W4R = MHPPO_X3_W4R;
// BS: the bias gradients dB3 / dB2 as MFMA row sums of the d3 / d2 image fragments the weight
// gradients already read (a one-hot B column each, three products: one 16-register accumulator)
// instead of a per-tile LDS transpose and VALU sum each (probe: -5.6 % critic / -8.4 % actor
// tile time without those sums, profiles/r04_x3_bs/).
// DH2F: the on-chain dH2 MFMAs issued before the off-chain dW3 block (the h2 image splits in their
// shadow); XCE: dW1's first input-column split issued before the dH1 MFMAs.  Measured per kernel
// (profiles/r04_x3_bs/ab_order.txt): continuous actor both (-1.9 %), fused pair DH2F (-1.6 %), the
// critic neither (its 512 registers: +3 % with either).
// SCH: the hand-placed backward (bwd_s) — the 13-input heads' single-net passes.
template <int KIND, int HF, int HB, class G, bool BS = false, bool DH2F = false, bool XCE = false,
          bool W4R_ = KIND == K_CONT, bool SCH = false>
struct Pass {
  static constexpr int KS1 = G::KS1, NOUT = G::NOUT;
  static_assert(NOUT == (KIND == K_CHOICE ? 2 : 1), "outputs");
  const char *w1row, *w2row, *w3row, *w2tr, *w3tr;
  const float *F;
  float b40, b41;
  int nin;
  const double *counts;  // K_CHOICE: the global action counts (nullptr: per-row mode)
  double m_global;
  F3 wf2[2][2], wf3[4], wb3[2][2], wb2[4];
  // SCH: the previous tile's dW1 block (E), deferred into this tile's layer-1 shadows: its A operands
  // (the d1 image's transposed reads) and B operand (the input columns); zero before the first tile
  F3 ea0, ea1, exb;
  f32x16 gW2a, gW2b, gW3a, gW3b;
  f32x4 gW1t[KS1][2];
  f32x16 gBS;    // BS: column 0 = dB3, 1 = dB2[0:32], 2 = dB2[32:64] (rows = out features)
  u32x4 oh[3];   // BS: B fragments with bf16 1.0 in column q only
  // W4R (the actor passes: registers to spare): dW4 = sum over rows of dy h3 accumulated per lane
  // and register across the wave's tiles (one FMA per element) and summed over the lanes once, in
  // finish, instead of a per-tile LDS transpose (probe: -2.7 % actor tile time without that sum)
  // (the continuous actor: the choice actor's second output would spill the K = 32 geometry)
  static constexpr bool W4R = W4R_ && X3_W4R;
  f32x16 gW4r, gW4r1;
  // bias-gradient half-row sums (lane j, half kh): gB2a gB2b gB3 gW4[0] gB4[0] gW4[1] gB4[1]
  float gsum[7];
  // float64 loss / advantage sums in registers (lanes kh == 0), folded once after the loop: an
  // LDS read-modify-write per tile put its latency on the loss section's serial chain (-1 %)
  double dsum0, dsum1, dsum2;

  __device__ __forceinline__ void init(const char *Lw, const WaveSlot<G> &ws, int nin_rt = 0,
                                       const double *counts_ = nullptr, double m_global_ = 0.0) {
    const int j = ws.j, kh = ws.kh, G_ = ws.G, q4 = (ws.l >> 2) & 3, p4 = ws.l & 3;
    nin = geo_nin<G>(nin_rt);
    counts = counts_;
    m_global = m_global_;
    // lane address bases: every fragment access is one of these plus a constant
    w1row = Lw + G::O_W1 + j * G::W1_ROWB + 16 * kh;
    w2row = Lw + G::O_W2 + j * W2_ROWB + 8 * kh;
    w3row = Lw + G::O_W3 + j * W3_ROWB + 8 * kh;
    w2tr = Lw + G::O_W2 + (4 * (G_ >> 1) + q4) * W2_ROWB + 8 * (4 * (G_ & 1) + p4);
    w3tr = Lw + G::O_W3 + (4 * (G_ >> 1) + q4) * W3_ROWB + 8 * (4 * (G_ & 1) + p4);
    F = reinterpret_cast<const float *>(Lw + G::O_F);
    b40 = uniform_f(F[G::F_B4]);
    b41 = NOUT == 2 ? uniform_f(F[G::F_B4 + 1]) : 0.0f;
    // loop-invariant weight fragments read from LDS once
    if constexpr (HF & 1) {
      for (int t = 0; t < 2; t++)
        for (int s = 0; s < 2; s++) wf2[t][s] = w_fwd<W2_ROWB, W2_PART>(w2row, t, s);
    }
    if constexpr (HF & 2) {
      for (int s = 0; s < 4; s++) wf3[s] = w_fwd<W3_ROWB, W3_PART>(w3row, 0, s);
    }
    if constexpr (HB & 1) {
      for (int t = 0; t < 2; t++)
        for (int s = 0; s < 2; s++) wb3[t][s] = w_bwd<W3_ROWB, W3_PART>(w3tr, t, s);
    }
    if constexpr (HB & 2) {
      for (int s = 0; s < 4; s++) wb2[s] = w_bwd<W2_ROWB, W2_PART>(w2tr, 0, s);
    }
    gW2a = zero16(), gW2b = zero16(), gW3a = zero16(), gW3b = zero16();
    for (int c = 0; c < KS1; c++) gW1t[c][0] = gW1t[c][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < 7; k++) gsum[k] = 0.f;
    dsum0 = dsum1 = dsum2 = 0.0;
    if constexpr (W4R) {
      gW4r = zero16();
      if constexpr (NOUT == 2) gW4r1 = zero16();
    }
    if constexpr (BS) {
      gBS = zero16();
      if constexpr (SCH) {
        for (int q = 0; q < 3; q++) ea0.p[q] = ea1.p[q] = exb.p[q] = u32x4{0u, 0u, 0u, 0u};
      }
      for (int q = 0; q < 3; q++) {
        const uint32_t v = j == q ? 0x3f803f80u : 0u;
        oh[q] = u32x4{v, v, v, v};
        // opaque (not a rematerialisable constant): the compiler would rebuild it with a
        // v_accvgpr_write right before its MFMA, a write the MFMA reads without wait states
        if constexpr (SCH) asm volatile("" : "+a"(oh[q]));
      }
    }
  }
  __device__ __forceinline__ F3 fw2(int t, int s) const {
    if constexpr (HF & 1) return wf2[t][s];
    else return w_fwd<W2_ROWB, W2_PART>(w2row, t, s);
  }
  __device__ __forceinline__ F3 fw3(int s) const {
    if constexpr (HF & 2) return wf3[s];
    else return w_fwd<W3_ROWB, W3_PART>(w3row, 0, s);
  }
  __device__ __forceinline__ F3 bw3(int t, int s) const {
    if constexpr (HB & 1) return wb3[t][s];
    else return w_bwd<W3_ROWB, W3_PART>(w3tr, t, s);
  }
  __device__ __forceinline__ F3 bw2(int s) const {
    if constexpr (HB & 2) return wb2[s];
    else return w_bwd<W2_ROWB, W2_PART>(w2tr, 0, s);
  }

  // One 32-row tile whose inputs sit in `slot` (X [32][13] | ret V | act logp_old).  The critic
  // writes V (rows row0 .. row0 + nrows) to Vout; the actor normalises A = ret - V with
  // (meanf, stdf).
  __device__ __forceinline__ void tile(const WaveSlot<G> &ws, const float *slot, int64_t row0, int nrows,
                                       float *__restrict__ Vout, float meanf, float stdf, double inv_m,
                                       float out_mean, float out_std) {
    const int nin = G::NIC ? G::NIC : this->nin;
    const int l = ws.l, j = ws.j, kh = ws.kh, G_ = ws.G;
    float *T = ws.T;
    char *imw = ws.imw;
    const char *imr = ws.imr, *imr16 = ws.imr16;
    constexpr int O_IM2 = G::O_IM2;
    auto radd = [&](int k, float v) { gsum[k] += v; };
    const float *Xs = slot + G::IN_X;
    // ---- layer 1: h1^T = W1 . [X | 1]^T (b1 rides in input column nin), K-step s = columns 16s..
    auto layer1 = [&]() {
      f32x16 h = zero16();
#pragma unroll
      for (int s = 0; s < KS1; s++) {
        float v8[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          // row j, input column k = 16s + 8h + q (the bias input at k = nin).  Columns past nin
          // read the next row's first inputs (the slot's last row reads into its s0 block).
          const int k = 16 * s + 8 * kh + q;
          const float v = Xs[j * nin + k];
          v8[q] = k < nin ? v : (k == nin ? 1.0f : 0.0f);
        }
        h = mfma6(rd_pair<G::W1_PART>(w1row + 32 * s, 8), split8(v8), h);
      }
      relu16(h);
      return h;
    };
    f32x16 h1;
    if constexpr (SCH) h1 = layer1_s(ws, Xs);
    else h1 = layer1();
    x3_phase();
    MHPPO_MARK(2);
    // ---- layer 2 (the biases ride in as the chains' initial accumulators)
    f32x16 h2a = feat_vec(F, kh), h2b = feat_vec(F + 32, kh);
    f32x16 h3 = feat_vec(F + 64, kh);
    F3 h1s[2], h2as[2], h2bs[2], xb;  // SCH: the forward's splits (kept for the backward's images)
    F3 sha0, sha1;                    // SCH: dW3's B operands (the h2a image's reads, in layer 3's shadows)
    if constexpr (SCH) {
      fwd_s(ws, Xs, h1, h1s, h2a, h2b, h2as, h2bs, h3, xb, sha0, sha1);
    } else {
#pragma unroll
      for (int s = 0; s < 2; s++) {
        const F3 b = split_step(h1, s);
        h2a = mfma6(fw2(0, s), b, h2a);
        h2b = mfma6(fw2(1, s), b, h2b);
      }
      relu16(h2a);
      relu16(h2b);
      x3_phase();
      MHPPO_MARK(3);
      // ---- layer 3
#pragma unroll
      for (int s = 0; s < 2; s++) h3 = mfma6(fw3(s), split_step(h2a, s), h3);
#pragma unroll
      for (int s = 0; s < 2; s++) h3 = mfma6(fw3(2 + s), split_step(h2b, s), h3);
    }
    relu16(h3);
    x3_phase();
    MHPPO_MARK(4);
    // ---- output and loss gradient dL/dy for this lane's row (as the f32 path)
    const f32x16 w4v = feat_vec(F + G::F_W4, kh);
    float part0 = 0.0f;
#pragma unroll
    for (int r = 0; r < 16; r++) part0 = fmaf(w4v[r], h3[r], part0);
    const float y0 = xhalf_sum(part0) + b40;
    f32x16 w4v1;
    float y1 = 0.0f;
    if constexpr (NOUT == 2) {
      w4v1 = feat_vec(F + G::F_W4 + 32, kh);
      float part1 = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; r++) part1 = fmaf(w4v1[r], h3[r], part1);
      y1 = xhalf_sum(part1) + b41;
    }
    const bool valid = j < nrows;
    float dy0 = 0.0f, dy1 = 0.0f;
    if (valid) {
      const float rt = slot[G::IN_S0 + j];
      if constexpr (KIND == K_CRITIC) {
        const float v = y0;
        // the store's range is the tile's rows in the batch (a wrong row index reaches no memory)
        if (kh == 0)
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rsrc(Vout + row0, 4 * nrows), 4 * j, 0, 0);
        const float a = rt - v;
        const float d = v - rt;
        if (kh == 0) {
          dsum0 += (double)d * (double)d;
          dsum1 += (double)a;
          dsum2 += (double)a * (double)a;
        }
        dy0 = (float)(2.0 * inv_m * (double)d);
      } else if constexpr (KIND == K_CONT) {
        const float t = tanhf(y0);
        const float mu = t * out_std + out_mean;
        const float a = rt - slot[G::IN_S0 + 32 + j];
        const float A = (a - meanf) / (stdf + 1e-10f);
        const float diff = (float)((double)slot[G::IN_S1 + j] - (double)mu);
        const float x = diff * MVN_INV_L;
        const float lp = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HALF_LOGDET;
        // the ratio's magnitude in float32, its clip branch decided in float64 (see the note at
        // the head of namespace x3)
        const float lpo = slot[G::IN_S1 + 32 + j];
        const float r = expf(lp - lpo);
        float dfdr;
        const float f = surr_and_grad_fd(r, (double)lp - (double)lpo, A, dfdr);
        if (kh == 0) dsum0 += (double)f;
        const float dmu = (float)(inv_m * (double)dfdr * (double)r * (double)x * (double)MVN_INV_L);
        dy0 = (dmu * out_std) * (1.0f - t * t);
      } else {
        // choice actor (train_model_d :818-851): softmax over the pair (as torch: shift by the
        // max), pn = p / (p0 + p1), the M x M Categorical broadcast in its O(M) form with the
        // global action counts (or the opt-in per-row loss: the row's own action, weight M)
        const float mx = fmaxf(y0, y1);
        const float e0 = expf(y0 - mx), e1 = expf(y1 - mx);
        const float se = e0 + e1;
        const float p[2] = {e0 / se, e1 / se};
        const float a = rt - slot[G::IN_S0 + 32 + j];
        const float A = (a - meanf) / (stdf + 1e-10f);
        const double old = (double)slot[G::IN_S1 + j];
        const float sp = p[0] + p[1];
        const float pn[2] = {p[0] / sp, p[1] / sp};
        const float eps = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
        const double inv_m2 = inv_m * inv_m;
        const int a_row = counts ? 0 : (int)slot[G::IN_S1 + 32 + j];
        double dlp[2], f = 0.0;
#pragma unroll
        for (int k = 0; k < 2; k++) {
          const double wk = counts ? counts[k] : (k == a_row ? m_global : 0.0);
          const float pc = pn[k] < eps ? eps : (pn[k] > hi ? hi : pn[k]);
          const double r = exp((double)logf(pc) - old);
          double dfdr;
          const double fk = surr_and_grad(r, (double)A, dfdr);
          if (wk != 0.0) f += wk * fk;
          const double pass = (pn[k] >= eps && pn[k] <= hi) ? 1.0 : 0.0;
          dlp[k] = inv_m2 * wk * dfdr * r * pass / (double)pc;  // dL/dpn_k
        }
        if (kh == 0) dsum0 += f;
        const double sd = (double)sp;
        const double g0 = (dlp[0] * (1.0 - pn[0]) - dlp[1] * pn[1]) / sd;  // dL/dp_k
        const double g1 = (dlp[1] * (1.0 - pn[1]) - dlp[0] * pn[0]) / sd;
        const double dot = (double)p[0] * g0 + (double)p[1] * g1;
        dy0 = (float)((double)p[0] * (g0 - dot));  // softmax Jacobian
        dy1 = (float)((double)p[1] * (g1 - dot));
      }
    }
    radd(4, (kh == 0) ? dy0 : 0.0f);
    if constexpr (NOUT == 2) radd(6, (kh == 0) ? dy1 : 0.0f);
    if constexpr (SCH) {
      bwd_s(ws, h1, h2a, h2b, h3, w4v, dy0, xb, sha0, sha1);
      return;
    }
    // ---- layer 4 backward: d3 = dH3^T masked; dW4 = row sums of dy h3; dB3 = row sums of d3
    f32x16 g, d3;
#pragma unroll
    for (int r = 0; r < 16; r++) {
      g[r] = dy0 * h3[r];
      if constexpr (NOUT == 2) d3[r] = (h3[r] > 0.0f) ? fmaf(w4v1[r], dy1, w4v[r] * dy0) : 0.0f;
      else d3[r] = (h3[r] > 0.0f) ? w4v[r] * dy0 : 0.0f;
    }
    if constexpr (W4R) {
#pragma unroll
      for (int r = 0; r < 16; r++) gW4r[r] = fmaf(dy0, h3[r], gW4r[r]);
      if constexpr (NOUT == 2) {
#pragma unroll
        for (int r = 0; r < 16; r++) gW4r1[r] += dy1 * h3[r];
      }
    } else {
      X3_ROWSUM(3, g);
      if constexpr (NOUT == 2) {
        f32x16 g1;
#pragma unroll
        for (int r = 0; r < 16; r++) g1[r] = dy1 * h3[r];
        X3_ROWSUM(5, g1);
      }
    }
    if constexpr (!BS) X3_ROWSUM(2, d3);
    x3_phase();
    MHPPO_MARK(5);
    // ---- dW3 = sum over rows of d3 (x) h2: A = d3 image, B = h2a / h2b images
    const F3 d3f0 = split_step(d3, 0), d3f1 = split_step(d3, 1);
    // dH2^T = W3^T . dH3^T (below, or here with DH2F: issued before the dW3 block)
    f32x16 d2a = zero16(), d2b = zero16();
    auto dh2 = [&]() {
      d2a = mfma6(bw3(0, 0), d3f0, d2a);
      d2a = mfma6(bw3(0, 1), d3f1, d2a);
      d2b = mfma6(bw3(1, 0), d3f0, d2b);
      d2b = mfma6(bw3(1, 1), d3f1, d2b);
    };
    if constexpr (DH2F) dh2();
    img_write(imw, d3f0, d3f1);
    lds_order();
    const F3 ad0 = img_read(imr, 0), ad1 = img_read(imr, 1);
    lds_order();
    // h2a to the second image, h2b behind the d3 reads in the first: every later fragment is
    // read in the gaps of the MFMA block before the one that consumes it
    img_write(imw + O_IM2, split_step(h2a, 0), split_step(h2a, 1));
    lds_order();
    const F3 ha0 = img_read(imr + O_IM2, 0);
    lds_order();
    img_write(imw, split_step(h2b, 0), split_step(h2b, 1));
    lds_order();
    {
      F3 ha1, hb0, hb1;
      macc6_rd<false, O_IM2 + 16 * IM_ROWB>(ad0, ha0, gW3a, ha1, imr);
      macc6_rd<true, 0>(ad1, ha1, gW3a, hb0, imr);
      macc6_rd<true, 16 * IM_ROWB>(ad0, hb0, gW3b, hb1, imr);
      macc6_w(ad1, hb1, gW3b);
    }
    if constexpr (BS) {
      macc3(ad0, oh[0], gBS);
      macc3(ad1, oh[0], gBS);
    }
    lds_order();
    x3_phase();
    MHPPO_MARK(6);
    // ---- dH2^T = W3^T . dH3^T, masked by h2 > 0; dB2 = row sums
    if constexpr (!DH2F) dh2();
    relu_mask(d2a, h2a);
    relu_mask(d2b, h2b);
    if constexpr (!BS) {
      X3_ROWSUM(0, d2a);
      X3_ROWSUM(1, d2b);
    }
    x3_phase();
    MHPPO_MARK(7);
    // the B operand of dW1's input columns 16c .. 16c + 15: rows 8G .. 8G + 7 of column 16c + n
    auto xcols = [&](int c) {
      float xv[8];
      const int n = 16 * c + (l & 15);
#pragma unroll
      for (int q = 0; q < 8; q++) {
        const float v = Xs[(8 * G_ + q) * nin + (n < nin ? n : 0)];
        xv[q] = n < nin ? v : (n == nin ? 1.0f : 0.0f);
      }
      return split8(xv);
    };
    F3 xb0;  // XCE: dW1's first input-column split, issued ahead of the dH1 MFMAs (into their shadow)
    if constexpr (XCE) xb0 = xcols(0);
    // ---- dH1^T = W2^T . dH2^T, masked by h1 > 0; dW2 = sum over rows of d2 (x) h1
    f32x16 d1 = zero16();
    if constexpr (HF != 3) {
      const F3 f0 = split_step(d2a, 0), f1 = split_step(d2a, 1);
      d1 = mfma6(bw2(0), f0, d1);
      d1 = mfma6(bw2(1), f1, d1);
      // B = h1 image (second slot), A = d2a image (first slot), then d2b into the second slot
      // behind the h1 reads; the A fragments after the first are read in the MFMA gaps
      img_write(imw + O_IM2, split_step(h1, 0), split_step(h1, 1));
      lds_order();
      const F3 bh0 = img_read(imr + O_IM2, 0), bh1 = img_read(imr + O_IM2, 1);
      lds_order();
      img_write(imw, f0, f1);
      lds_order();
      const F3 f2 = split_step(d2b, 0), f3 = split_step(d2b, 1);
      img_write(imw + O_IM2, f2, f3);
      lds_order();
      d1 = mfma6(bw2(2), f2, d1);
      d1 = mfma6(bw2(3), f3, d1);
      const F3 da0 = img_read(imr, 0);
      lds_order();
      {
        F3 da1, db0, db1;
        macc6_rd<false, 16 * IM_ROWB>(da0, bh0, gW2a, da1, imr);
        macc6_rd<true, O_IM2>(da1, bh1, gW2a, db0, imr);
        macc6_rd<true, O_IM2 + 16 * IM_ROWB>(db0, bh0, gW2b, db1, imr);
        macc6_w(db1, bh1, gW2b);
        if constexpr (BS) {  // every fragment complete: macc6_w waited for db1, the blocks before for the rest
          macc3(da0, oh[1], gBS);
          macc3(da1, oh[1], gBS);
          macc3(db0, oh[2], gBS);
          macc3(db1, oh[2], gBS);
        }
      }
      lds_order();
    } else {  // (the forward weight fragments are held: no registers for the reads ahead)
      const F3 f0 = split_step(d2a, 0), f1 = split_step(d2a, 1);
      d1 = mfma6(bw2(0), f0, d1);
      d1 = mfma6(bw2(1), f1, d1);
      // B = h1 image, A = d2a image
      img_write(imw, split_step(h1, 0), split_step(h1, 1));
      lds_order();
      const F3 bh0 = img_read(imr, 0), bh1 = img_read(imr, 1);
      lds_order();
      img_write(imw, f0, f1);
      lds_order();
      {
        const F3 da0 = img_read(imr, 0), da1 = img_read(imr, 1);
        macc6(da0, bh0, gW2a);
        macc6(da1, bh1, gW2a);
        if constexpr (BS) {
          macc3(da0, oh[1], gBS);
          macc3(da1, oh[1], gBS);
        }
      }
      lds_order();
      const F3 f2 = split_step(d2b, 0), f3 = split_step(d2b, 1);
      d1 = mfma6(bw2(2), f2, d1);
      d1 = mfma6(bw2(3), f3, d1);
      img_write(imw, f2, f3);
      lds_order();
      {
        const F3 db0 = img_read(imr, 0), db1 = img_read(imr, 1);
        macc6(db0, bh0, gW2b);
        macc6(db1, bh1, gW2b);
        if constexpr (BS) {
          macc3(db0, oh[2], gBS);
          macc3(db1, oh[2], gBS);
        }
      }
      lds_order();
    }
    relu_mask(d1, h1);
    x3_phase();
    MHPPO_MARK(8);
    // ---- dW1 = sum over rows of d1 (x) [X | 1]: A = d1 image, B = the input rows (column 13:
    // the constant 1, i.e. dB1).  16x16x32 tiles (out features 16t..16t+15 x input columns
    // 0..15, all 32 rows in one K-step): lane l of group G = l >> 4 holds rows 8G..8G+7 of
    // column l & 15 / feature l & 15
    img_write(imw, split_step(d1, 0), split_step(d1, 1));
    lds_order();
    {
      F3 b;
      if constexpr (XCE) b = xb0;
      else b = xcols(0);
      const F3 a0 = tr_pair<IM_PART>(imr16, 4 * IM_ROWB);
      F3 a1;
      macc6_16_rd<false, 32>(a0, b, gW1t[0][0], a1, imr16);
      macc6_16_w(a1, b, gW1t[0][1]);
#pragma unroll
      for (int c = 1; c < KS1; c++) {
        const F3 bc = xcols(c);
        macc6_16(a0, bc, gW1t[c][0]);
        macc6_16(a1, bc, gW1t[c][1]);
      }
    }
    lds_order();
    x3_phase();
    MHPPO_MARK(9);
  }

  // The previous tile's dW1 block E: 12 AGPR MFMAs (16x16x32) on the deferred operands
  template <int K>
  __device__ __forceinline__ void mac_e() {
    constexpr int P = K % 6;
    if constexpr (K < 6) mac1_16(ea0.p[P6A[P]], exb.p[P6B[P]], gW1t[0][0]);
    else mac1_16(ea1.p[P6A[P]], exb.p[P6B[P]], gW1t[0][1]);
  }
  // Layer 1 of one tile, hand-placed (SCH), with the PREVIOUS tile's dW1 block in its shadows: the
  // input loads first, then E's MFMAs carry the input split, then layer 1's six MFMAs alternate with
  // E's last ones.  (E used to end the tile: twelve 16-cycle MFMAs with nothing beside them, behind
  // the LDS latency of their operand reads; deferred, its operands are already in registers.)  The
  // per-accumulator product order is unchanged: the same bits.  Returns ReLU(h1).
  __device__ __forceinline__ f32x16 layer1_s(const WaveSlot<G> &ws, const float *Xs) {
    const int j = ws.j, kh = ws.kh;
    float v8[8], rs[8];
#pragma unroll
    for (int q = 0; q < 8; q++) v8[q] = Xs[j * NIN_CONT + 8 * kh + q];  // past column 12: unused
    pin4(v8);
    pin4(v8 + 4);
#pragma unroll
    for (int q = 0; q < 8; q++) {  // row j, input column 8h + q (the bias input at column 13)
      const int k = 8 * kh + q;
      v8[q] = k < NIN_CONT ? v8[q] : (k == NIN_CONT ? 1.0f : 0.0f);
    }
    const F3 w1 = rd_pair<G::W1_PART>(w1row, 8);
    F3 xs;
    f32x16 h = zero16();
    // regions: E0 E1 | E2..E9 + the input split | L0 E10 L1 E11 L2 L3 L4 L5
    constexpr int ORD[18] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 100, 10, 101, 11, 102, 103, 104, 105};
    weave<18, Plan<2, 10, 8>>(
        [&](auto kc) {
          constexpr int K = decltype(kc)::value, M = ORD[K];
          if constexpr (M < 100) mac_e<M>();
          else h = mfma_b(w1.p[P6A[M - 100]], xs.p[P6B[M - 100]], h);
        },
        [&](auto uc) {
          constexpr int U = decltype(uc)::value;
          if constexpr (U % 2 == 0) split_l1(v8, U / 2, xs, rs);
          else split_l2(U / 2, xs, rs);
        });
    relu16(h);
    return h;
  }
  // after the tile loop: the last tile's deferred dW1 block (once per launch: every MFMA behind
  // enough wait states for a compiler copy of its accumulator or operands just before it)
  __device__ __forceinline__ void drain() {
    if constexpr (SCH) {
      sfor<0, 12>([&](auto kc) {
        constexpr int K = decltype(kc)::value, P = K % 6;
        f32x4 &c = K < 6 ? gW1t[0][0] : gW1t[0][1];
        const F3 &a = K < 6 ? ea0 : ea1;
        asm volatile("s_nop 4\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a.p[P6A[P]]), "v"(exb.p[P6B[P]]));
      });
    }
  }

  // Layers 2 and 3 of one tile, hand-placed (SCH): each layer's MFMAs carry the splits its own later
  // K-steps and the next layer need (the same products in the same order per accumulator as the
  // plain forward, so the same bits):
  //   L2  [h2a s0 | h2a s1 | h2b s0 | h2b s1]  | h1's K-step 1 split, dW1's input-column split,
  //                                              h2a's ReLU and split (after its last MFMA)
  //   L3  [h2a s0 | h2a s1 | h2b s0 | h2b s1]  | the rest of h2a's split, h2b's ReLU and split
  // h1 arrives ReLU'd; h2a / h2b / h3 leave as the layers' pre-ReLU accumulators for h3 (the caller
  // applies its ReLU) and ReLU'd for h2a / h2b.
  __device__ __forceinline__ void fwd_s(const WaveSlot<G> &ws, const float *Xs, const f32x16 &h1, F3 (&h1s)[2],
                                        f32x16 &h2a, f32x16 &h2b, F3 (&h2as)[2], F3 (&h2bs)[2], f32x16 &h3,
                                        F3 &xb, F3 &ha0, F3 &ha1) {
    const int l = ws.l, G_ = ws.G;
    char *imw = ws.imw;
    const char *imr = ws.imr;
    constexpr int RS = 16 * IM_ROWB, DU = 4 * IM_ROWB;
    float rs[8], rt[8], xv[8];
    float h1v[16];
#pragma unroll
    for (int r = 0; r < 16; r++) h1v[r] = h1[r];
#pragma unroll
    for (int q = 0; q < 4; q++) split_l1(h1v, q, h1s[0], rs);
#pragma unroll
    for (int q = 0; q < 4; q++) split_l2(q, h1s[0], rs);
    {
      const F3 w00 = fw2(0, 0), w01 = fw2(0, 1), w10 = fw2(1, 0), w11 = fw2(1, 1);
      // h1 s1 split (8 units, before k = 6), dW1's B operand (1 + 8), h2a ReLU (4, after its last
      // MFMA k = 11 has landed) + h2a s0 split (8) + h2a s1 split level 1 (4); the h1 image (slot 3,
      // six stores, one per two shadows; its K-step 1 half after that split)
      using PL = Plan<0, 5, 8, 5, 12, 10, 13, 24, 16, 1, 13, 6>;
      static_assert(PL::reg(7) < 6 && PL::reg(7) < PL::reg(37), "h1's K-step 1 before its MFMAs and its image");
      weave<24, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) h2a = mfma_b(w00.p[P6A[P]], h1s[0].p[P6B[P]], h2a);
            if constexpr (T == 1) h2a = mfma_b(w01.p[P6A[P]], h1s[1].p[P6B[P]], h2a);
            if constexpr (T == 2) h2b = mfma_b(w10.p[P6A[P]], h1s[0].p[P6B[P]], h2b);
            if constexpr (T == 3) h2b = mfma_b(w11.p[P6A[P]], h1s[1].p[P6B[P]], h2b);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            if constexpr (U < 8) {
              if constexpr (U % 2 == 0) split_l1(h1v + 8, U / 2, h1s[1], rs);
              else split_l2(U / 2, h1s[1], rs);
            } else if constexpr (U < 10) {  // dW1's B operand: rows 8G .. 8G + 7 of input column l & 15
              const int n = l & 15, nc = n < NIN_CONT ? n : NIN_CONT - 1;
              float v[4];
#pragma unroll
              for (int q = 0; q < 4; q++) v[q] = Xs[(8 * G_ + 4 * (U - 8) + q) * NIN_CONT + nc];
              pin4(v);
#pragma unroll
              for (int q = 0; q < 4; q++) xv[4 * (U - 8) + q] = n < NIN_CONT ? v[q] : (n == NIN_CONT ? 1.0f : 0.0f);
            } else if constexpr (U < 18) {
              constexpr int V = U - 10;
              if constexpr (V % 2 == 0) split_l1(xv, V / 2, xb, rt);
              else split_l2(V / 2, xb, rt);
            } else if constexpr (U < 22) {  // h2a's ReLU
              relu4(h2a, 4 * (U - 18));
            } else if constexpr (U < 30) {  // h2a K-step 0 split
              constexpr int V = U - 22;
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = h2a[e];
              if constexpr (V % 2 == 0) split_l1(v, V / 2, h2as[0], rs);
              else split_l2(V / 2, h2as[0], rs);
            } else if constexpr (U < 34) {  // h2a K-step 1 split, level 1 (level 2 in L3)
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = h2a[8 + e];
              split_l1(v, U - 30, h2as[1], rt);
            } else {  // the h1 image (slot 3): part (U - 34) % 3 of K-step half (U - 34) / 3
              constexpr int V = U - 34;
              img_write_h(imw + G::O_IM3, h1s[V / 3], V % 3, V / 3);
              lds_order();
            }
          });
    }
    MHPPO_MARK(3);
    {
      const F3 w0 = fw3(0), w1 = fw3(1), w2 = fw3(2), w3 = fw3(3);
      // h2a s1 level 2 (4, before k = 6) + h2b ReLU 0-7 (2) + h2b s0 level 1 (4); h2b s0 level 2 (4,
      // before k = 12) + h2b ReLU 8-15 (2) + h2b s1 level 1 (4); h2b s1 level 2 (4, before k = 18);
      // the h2a image (slot 4) and the h2b image (slot 2), one store per two shadows, each half after
      // its split; the h2a image's transposed reads (dW3's B operands) behind its stores
      using PL = Plan<0, 6, 10, 6, 12, 10, 12, 18, 4, 1, 13, 6, 13, 25, 6, 12, 24, 6>;
      static_assert(PL::reg(3) < 6 && PL::reg(13) < 12 && PL::reg(23) < 18, "splits before their MFMAs");
      static_assert(PL::reg(3) < PL::reg(27) && PL::reg(13) < PL::reg(30) && PL::reg(23) < PL::reg(33) &&
                        PL::reg(29) < PL::reg(36),
                    "image halves after their splits, reads after the stores");
      weave<24, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) h3 = mfma_b(w0.p[P6A[P]], h2as[0].p[P6B[P]], h3);
            if constexpr (T == 1) h3 = mfma_b(w1.p[P6A[P]], h2as[1].p[P6B[P]], h3);
            if constexpr (T == 2) h3 = mfma_b(w2.p[P6A[P]], h2bs[0].p[P6B[P]], h3);
            if constexpr (T == 3) h3 = mfma_b(w3.p[P6A[P]], h2bs[1].p[P6B[P]], h3);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            if constexpr (U < 4) {
              split_l2(U, h2as[1], rt);
            } else if constexpr (U < 6) {  // h2b's ReLU, elements 0-7
              relu4(h2b, 4 * (U - 4));
            } else if constexpr (U < 10) {
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = h2b[e];
              split_l1(v, U - 6, h2bs[0], rs);
            } else if constexpr (U < 14) {
              split_l2(U - 10, h2bs[0], rs);
            } else if constexpr (U < 16) {  // h2b's ReLU, elements 8-15
              relu4(h2b, 8 + 4 * (U - 14));
            } else if constexpr (U < 20) {
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = h2b[8 + e];
              split_l1(v, U - 16, h2bs[1], rt);
            } else if constexpr (U < 24) {
              split_l2(U - 20, h2bs[1], rt);
            } else if constexpr (U < 30) {  // the h2a image (slot 4)
              constexpr int V = U - 24;
              img_write_h(imw + G::O_IM4, h2as[V / 3], V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 36) {  // the h2b image (slot 2: the previous tile's d2b reads are issued)
              constexpr int V = U - 30;
              img_write_h(imw + G::O_IM2, h2bs[V / 3], V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 39) {
              tr_pt(imr + G::O_IM4, DU, U - 36, ha0);
            } else {
              tr_pt(imr + G::O_IM4 + RS, DU, U - 39, ha1);
              lds_order();
            }
          });
    }
  }

  // The backward of one tile, hand-placed (SCH): five MFMA blocks, each carrying the work the
  // next block needs in its MFMA shadows (the plans below place it).  An image goes out as six
  // single stores at most one per two shadows (img_write_h: LDS stores, not the MFMAs, otherwise set
  // the pace), its reads one part (two ds_read_b64_tr_b16) per unit:
  //   A  dH2 = W3^T d3      24 on-chain MFMAs | d3's K-step-1 split, the d3 image and its reads, dW4 sums
  //   B  dW3 (+ dB3)        30 AGPR MFMAs     | the h2b image reads, d2a / d2b masks, d2a's split
  //   C  dH1 = W2^T d2      24 on-chain MFMAs | d2b's split, the d2a / d2b images, the h1 / d2a reads
  //   D  dW2 (+ dB2)        36 AGPR MFMAs     | the d2 image reads, d1's mask and split, d1's image
  //                                             and dW1's operand reads
  //   E  dW1 (+ dB1)        12 AGPR MFMAs (16x16x32), deferred into the next tile's layer 1
  // The forward wrote the h1 (slot 3), h2a (slot 4) and h2b (slot 2) images and read h2a's (ha0,
  // ha1).  Slot 1: d3, then d2a, then d1; slot 2: h2b, then d2b.  The same products in the same order
  // per accumulator as the phase-by-phase backward (the same bits); an image slot is rewritten only
  // after its last reads were issued (a wave's LDS operations execute in order).  xb: dW1's B operand
  // (input columns), split in the forward.
  __device__ __forceinline__ void bwd_s(const WaveSlot<G> &ws, const f32x16 &h1, const f32x16 &h2a, const f32x16 &h2b,
                                        const f32x16 &h3, const f32x16 &w4v, float dy0, const F3 &xb, const F3 &ha0,
                                        const F3 &ha1) {
    static_assert(KS1 == 1 && NOUT == 1 && BS && W4R && G::NIC == NIN_CONT && G::NIM == 4,
                  "SCH: the 13-input single-net passes, four image slots");
    char *imw = ws.imw;
    const char *imr = ws.imr, *imr16 = ws.imr16;
    constexpr int O_IM2 = G::O_IM2, O_IM3 = G::O_IM3, RS = 16 * IM_ROWB, DU = 4 * IM_ROWB;  // K-step 1 rows; tr_pair stride
    // d3 = dH3 masked by h3 > 0 (on the chain); its K-step 0 split here, K-step 1 in block A
    float d3[16];
#pragma unroll
    for (int r = 0; r < 16; r++) d3[r] = (h3[r] > 0.0f) ? w4v[r] * dy0 : 0.0f;
    F3 d3f0, d3f1;
    float rs[8];  // the level-1 residuals of the split in progress
#pragma unroll
    for (int q = 0; q < 4; q++) split_l1(d3, q, d3f0, rs);
#pragma unroll
    for (int q = 0; q < 4; q++) split_l2(q, d3f0, rs);
    MHPPO_MARK(5);
    f32x16 d2a = zero16(), d2b = zero16(), d1 = zero16();
    F3 ad0, ad1, hb0, hb1;
    // ---- block A: dH2^T = W3^T dH3^T, K-step 0 of both output tiles first (d3f1 is split meanwhile)
    {
      const F3 w00 = bw3(0, 0), w10 = bw3(1, 0), w01 = bw3(0, 1), w11 = bw3(1, 1);
      // d3f1 split (8), the d3 image (K-step 0 half in 1 3 5, K-step 1 half in 9 11 13), its reads
      // (14 .. 19), dW4 (20 .. 23)
      using PL = Plan<0, 8, 8, 1, 7, 3, 9, 15, 3, 14, 20, 6, 20, 24, 4>;
      static_assert(PL::reg(7) < PL::reg(11) && PL::reg(13) < PL::reg(14), "split, then stores, then reads");
      weave<24, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) d2a = mfma_b(w00.p[P6A[P]], d3f0.p[P6B[P]], d2a);
            if constexpr (T == 1) d2b = mfma_b(w10.p[P6A[P]], d3f0.p[P6B[P]], d2b);
            if constexpr (T == 2) d2a = mfma_b(w01.p[P6A[P]], d3f1.p[P6B[P]], d2a);
            if constexpr (T == 3) d2b = mfma_b(w11.p[P6A[P]], d3f1.p[P6B[P]], d2b);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            if constexpr (U < 8) {  // d3's K-step 1 split
              if constexpr (U % 2 == 0) split_l1(d3 + 8, U / 2, d3f1, rs);
              else split_l2(U / 2, d3f1, rs);
            } else if constexpr (U < 14) {  // the d3 image (slot 1: the previous tile's d1 reads are issued)
              constexpr int V = U - 8;
              img_write_h(imw, V < 3 ? d3f0 : d3f1, V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 17) {
              tr_pt(imr, DU, U - 14, ad0);
            } else if constexpr (U < 20) {
              tr_pt(imr + RS, DU, U - 17, ad1);
              lds_order();
            } else {  // dW4: sum over rows of dy h3, per lane and register
#pragma unroll
              for (int r = 4 * (U - 20); r < 4 * (U - 19); r++) gW4r[r] = fmaf(dy0, h3[r], gW4r[r]);
            }
          });
    }
    MHPPO_MARK(6);
    // ---- block B: dW3 = sum over rows of d3 (x) h2 (A = the d3 image, B = the h2a / h2b images), dB3
    F3 f0, f1;  // d2a's split (block C's first operands)
    {
      using PL = Plan<0, 6, 6, 6, 30, 32>;
      static_assert(PL::reg(2) < 12 && PL::reg(5) < 18, "image reads before their MFMAs");
      weave<30, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) mac1(ad0.p[P6A[P]], ha0.p[P6B[P]], gW3a);
            if constexpr (T == 1) mac1(ad1.p[P6A[P]], ha1.p[P6B[P]], gW3a);
            if constexpr (T == 2) mac1(ad0.p[P6A[P]], hb0.p[P6B[P]], gW3b);
            if constexpr (T == 3) mac1(ad1.p[P6A[P]], hb1.p[P6B[P]], gW3b);
            if constexpr (T == 4) mac1_oh((P < 3 ? ad0 : ad1).p[2 - P % 3], oh[0], gBS);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            if constexpr (U < 3) {  // the h2b image (slot 2, written in layer 3)
              tr_pt(imr + O_IM2, DU, U, hb0);
            } else if constexpr (U < 6) {
              tr_pt(imr + O_IM2 + RS, DU, U - 3, hb1);
              lds_order();
            } else if constexpr (U < 14) {  // d2a masked by h2a > 0, two elements per unit
              mask2(d2a, h2a, 2 * (U - 6));
            } else if constexpr (U < 30) {  // d2a's split: K-step 0 -> f0, 1 -> f1
              constexpr int V = U - 14, st = V / 8, q = (V % 8) / 2;
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = d2a[8 * st + e];
              if constexpr (V % 2 == 0) split_l1(v, q, st ? f1 : f0, rs);
              else split_l2(q, st ? f1 : f0, rs);
            } else {  // d2b masked by h2b > 0 (block A's last MFMAs have landed by now)
              mask2(d2b, h2b, 2 * (U - 30));
            }
          });
    }
    MHPPO_MARK(7);
    // ---- block C: dH1^T = W2^T dH2^T (one accumulator chain over the four K-steps)
    F3 f2, f3, bh0, bh1, da0;
    {
      const F3 w0 = bw2(0), w1 = bw2(1), w2 = bw2(2), w3 = bw2(3);
      // d2b's split (K-step 0 in 0 .. 10, 1 in 11 .. 16), the d2a image (0 2 .. 10, slot 1: the d3
      // reads are issued) and the d2b image (12 14 .. 22, slot 2: the h2b reads are issued), the h1
      // image reads (1 .. 11), d2a's first reads (13 15 17)
      using PL = Plan<0, 11, 8, 11, 17, 8, 0, 12, 6, 12, 24, 6, 1, 7, 3, 7, 13, 3, 13, 19, 3>;
      static_assert(PL::reg(7) < 12 && PL::reg(15) < 18, "d2b's split before its MFMAs");
      static_assert(PL::reg(7) < PL::reg(22) && PL::reg(15) < PL::reg(25) && PL::reg(21) < PL::reg(34),
                    "image halves after their splits, reads after the stores");
      weave<24, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) d1 = mfma_b(w0.p[P6A[P]], f0.p[P6B[P]], d1);
            if constexpr (T == 1) d1 = mfma_b(w1.p[P6A[P]], f1.p[P6B[P]], d1);
            if constexpr (T == 2) d1 = mfma_b(w2.p[P6A[P]], f2.p[P6B[P]], d1);
            if constexpr (T == 3) d1 = mfma_b(w3.p[P6A[P]], f3.p[P6B[P]], d1);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            auto split_d2b = [&](int st, int V) {  // d2b's split: K-step 0 -> f2, 1 -> f3
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = d2b[8 * st + e];
              if (V % 2 == 0) split_l1(v, V / 2, st ? f3 : f2, rs);
              else split_l2(V / 2, st ? f3 : f2, rs);
            };
            if constexpr (U < 8) {
              split_d2b(0, U);
            } else if constexpr (U < 16) {
              split_d2b(1, U - 8);
            } else if constexpr (U < 22) {  // the d2a image (slot 1)
              constexpr int V = U - 16;
              img_write_h(imw, V < 3 ? f0 : f1, V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 28) {  // the d2b image (slot 2)
              constexpr int V = U - 22;
              img_write_h(imw + O_IM2, V < 3 ? f2 : f3, V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 31) {  // the h1 image (slot 3, written in layer 2)
              tr_pt(imr + O_IM3, DU, U - 28, bh0);
            } else if constexpr (U < 34) {
              tr_pt(imr + O_IM3 + RS, DU, U - 31, bh1);
            } else {
              tr_pt(imr, DU, U - 34, da0);
              lds_order();
            }
          });
    }
    MHPPO_MARK(8);
    // ---- block D: dW2 = sum over rows of d2 (x) h1 (A = the d2a / d2b images, B = the h1 image), dB2
    F3 a0, a1;
    {
      F3 da1, db0, db1, e0, e1;
      // the d2 reads (0 .. 8), d1's mask (2 .. 9, after block C's last MFMA has landed) and split
      // (10 .. 25), the d1 image (19 21 23 | 27 29 31, slot 1: the d2a reads are issued), dW1's
      // operand reads (32 .. 35)
      using PL = Plan<0, 9, 9, 2, 10, 8, 10, 26, 16, 19, 25, 3, 27, 33, 3, 32, 36, 6>;
      static_assert(PL::reg(2) < 6 && PL::reg(5) < 12 && PL::reg(8) < 18, "image reads before their MFMAs");
      static_assert(PL::reg(24) < PL::reg(33) && PL::reg(32) < PL::reg(36) && PL::reg(38) < PL::reg(39),
                    "image halves after their splits, reads after the stores");
      weave<36, PL>(
          [&](auto kc) {
            constexpr int K = decltype(kc)::value, P = K % 6, T = K / 6;
            if constexpr (T == 0) mac1(da0.p[P6A[P]], bh0.p[P6B[P]], gW2a);
            if constexpr (T == 1) mac1(da1.p[P6A[P]], bh1.p[P6B[P]], gW2a);
            if constexpr (T == 2) mac1(db0.p[P6A[P]], bh0.p[P6B[P]], gW2b);
            if constexpr (T == 3) mac1(db1.p[P6A[P]], bh1.p[P6B[P]], gW2b);
            if constexpr (T == 4) mac1_oh((P < 3 ? da0 : da1).p[2 - P % 3], oh[1], gBS);
            if constexpr (T == 5) mac1_oh((P < 3 ? db0 : db1).p[2 - P % 3], oh[2], gBS);
          },
          [&](auto uc) {
            constexpr int U = decltype(uc)::value;
            if constexpr (U < 3) {
              tr_pt(imr + RS, DU, U, da1);
              lds_order();
            } else if constexpr (U < 6) {
              tr_pt(imr + O_IM2, DU, U - 3, db0);
            } else if constexpr (U < 9) {
              tr_pt(imr + O_IM2 + RS, DU, U - 6, db1);
            } else if constexpr (U < 17) {  // d1 masked by h1 > 0
              mask2(d1, h1, 2 * (U - 9));
            } else if constexpr (U < 33) {  // d1's split -> e0, e1
              constexpr int V = U - 17, st = V / 8, q = (V % 8) / 2;
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; e++) v[e] = d1[8 * st + e];
              if constexpr (V % 2 == 0) split_l1(v, q, st ? e1 : e0, rs);
              else split_l2(q, st ? e1 : e0, rs);
            } else if constexpr (U < 39) {  // the d1 image (slot 1)
              constexpr int V = U - 33;
              img_write_h(imw, V < 3 ? e0 : e1, V % 3, V / 3);
              lds_order();
            } else if constexpr (U < 42) {  // dW1's A operands: 16x16x32 transposed reads
              tr_pt(imr16, DU, U - 39, a0);
            } else {
              tr_pt(imr16 + 32, DU, U - 42, a1);
            }
          });
    }
    MHPPO_MARK(9);
    // ---- block E: dW1 = sum over rows of d1 (x) [X | 1] (column 13: dB1), two 16x16x32 tiles,
    // deferred into the next tile's layer-1 shadows (layer1_s; the last tile's: drain)
    ea0 = a0;
    ea1 = a1;
    exb = xb;
    lds_order();
  }

  // this wave's partial gradient (packed torch layout) and float64 sums
  __device__ __forceinline__ void finish(const WaveSlot<G> &ws, float *__restrict__ gp, double *__restrict__ dp) {
    const int nin = G::NIC ? G::NIC : this->nin;
    const Packed P(nin, NOUT);
    const int l = ws.l, j = ws.j, kh = ws.kh, G_ = ws.G;
    if constexpr (KS1 == 1) macc_drain(gW2a, gW2b, gW3a, gW3b, gW1t[0][0], gW1t[0][1]);
    else macc_drain2(gW2a, gW2b, gW3a, gW3b, gW1t[0][0], gW1t[0][1], gW1t[KS1 - 1][0], gW1t[KS1 - 1][1]);
    if constexpr (BS) asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" : "+a"(gBS));
    float gB2a = gsum[0], gB2b = gsum[1], gB3 = gsum[2], gW4 = gsum[3], gB4 = gsum[4];
    float gW41 = gsum[5], gB41 = gsum[6];
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const int f = feat(r, l);
      gp[P.W2 + f * 32 + j] = gW2a[r];
      gp[P.W2 + (32 + f) * 32 + j] = gW2b[r];
      gp[P.W3 + f * 64 + j] = gW3a[r];
      gp[P.W3 + f * 64 + 32 + j] = gW3b[r];
    }
#pragma unroll
    for (int c = 0; c < KS1; c++) {
#pragma unroll
      for (int t = 0; t < 2; t++) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int f = 16 * t + 4 * G_ + r, n = 16 * c + (l & 15);
          if (n < nin) gp[P.W1 + f * nin + n] = gW1t[c][t][r];
          if (n == nin) gp[P.B1 + f] = gW1t[c][t][r];
        }
      }
    }
    // halves of the row sums: lanes j and j + 32 hold rows 0-15 / 16-31 of feature j
    gB2a += __shfl_xor(gB2a, 32);
    gB2b += __shfl_xor(gB2b, 32);
    gB3 += __shfl_xor(gB3, 32);
    gW4 += __shfl_xor(gW4, 32);
    if (NOUT == 2) gW41 += __shfl_xor(gW41, 32);
    if (kh == 0) {
      if constexpr (!BS) {
        gp[P.B2 + j] = gB2a;
        gp[P.B2 + 32 + j] = gB2b;
        gp[P.B3 + j] = gB3;
      }
      if constexpr (!W4R) {
        gp[P.W4 + j] = gW4;
        if (NOUT == 2) gp[P.W4 + 32 + j] = gW41;
      }
    }
    if constexpr (W4R) {  // register r of lane (row j, half kh) holds feature feat(r, l): sum over j
#pragma unroll
      for (int r = 0; r < 16; r++) {
        float v = gW4r[r], v1 = NOUT == 2 ? gW4r1[r] : 0.0f;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          v += __shfl_xor(v, o);
          if constexpr (NOUT == 2) v1 += __shfl_xor(v1, o);
        }
        if (j == 0) {
          gp[P.W4 + feat(r, l)] = v;
          if constexpr (NOUT == 2) gp[P.W4 + 32 + feat(r, l)] = v1;
        }
      }
    }
    if constexpr (BS) {  // column q of the row-sum accumulator: lanes q, q + 32 (rows: feat(r, l))
      if (j < 3) {
        const int base = j == 0 ? P.B3 : (j == 1 ? P.B2 : P.B2 + 32);
#pragma unroll
        for (int r = 0; r < 16; r++) gp[base + feat(r, l)] = gBS[r];
      }
    }
    float b4s0 = gB4, b4s1 = gB41;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      b4s0 += __shfl_xor(b4s0, o);
      if (NOUT == 2) b4s1 += __shfl_xor(b4s1, o);
    }
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    if (kh == 0) s0 = dsum0, s1 = dsum1, s2 = dsum2;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      s0 += __shfl_xor(s0, o);
      s1 += __shfl_xor(s1, o);
      s2 += __shfl_xor(s2, o);
    }
    if (l == 0) {
      gp[P.B4] = b4s0;
      if (NOUT == 2) gp[P.B4 + 1] = b4s1;
      dp[0] = s0;
      dp[1] = s1;
      dp[2] = s2;
    }
  }
};

// the normalisation of the actor's advantage from the critic pass's global sums
__device__ __forceinline__ void adv_norm(const double *stats, double m_global, float &meanf, float &stdf) {
  double mean = stats[0] / m_global;
  double var = (stats[1] - stats[0] * mean) / (m_global - 1.0);
  meanf = uniform_f((float)mean);
  stdf = uniform_f((float)sqrt(var > 0 ? var : 0.0));
}

// Tile inputs of a runtime-width geometry (the choice heads): the X rows as whole 1-KiB LDS-DMA
// pieces (unmasked: buffer loads past the tile's rows return zeros, which land inside the X
// region), s0 = [ret | V], s1 = [logp_old | action] (K_CHOICE; the action only in per-row mode,
// else the lanes re-read logp_old: the same instruction count either way).
template <int KIND, class G>
__device__ __forceinline__ void prefetch_g(float *slot, const float *X, int nin, const float *ret, const float *V,
                                           const float *act, const float *lp, int64_t row0, int l, int64_t M) {
  const uint32_t rows = tile_rows(M, row0);
  const v4i rx = rsrc_v(X + row0 * nin, rows * nin * 4);
#pragma unroll
  for (int c = 0; c < G::XPIECES; c++) dma16(rx, slot + G::IN_X + 256 * c, 1024 * c + 16 * l);
  const uint32_t vo = 4 * (l & 31);
  if (l < 32) dma4(rsrc_v(ret + row0, 4 * rows), slot + G::IN_S0, vo);
  if (KIND != K_CRITIC) {
    if (l >= 32) dma4(rsrc_v(V + row0, 4 * rows), slot + G::IN_S0, vo);
    if (l < 32) dma4(rsrc_v(lp + row0, 4 * rows), slot + G::IN_S1, vo);
    if (l >= 32) dma4(rsrc_v((act ? act : lp) + row0, 4 * rows), slot + G::IN_S1, vo);
  }
}
template <int KIND, class G>
constexpr int prefetch_g_ops() { return G::XPIECES + (KIND == K_CRITIC ? 1 : 4); }

template <int KIND, class G>
__device__ __forceinline__ void load_sync_g(float *slot, const float *X, int nin, const float *ret, const float *V,
                                            const float *act, const float *lp, int64_t row0, int nrows, int l) {
  constexpr int NX = G::XMAX / 64;
  static_assert(G::XMAX % 64 == 0, "X region");
  const auto rx = rsrc(X + row0 * nin, (uint32_t)(nrows * nin) * 4);
  float x[NX];
#pragma unroll
  for (int i = 0; i < NX; i++) x[i] = bload(rx, 4 * (l + 64 * i));  // past the rows: 0
  const uint32_t nb = 4 * nrows, vo = 4 * (l & 31);
  const float s0 = bload(rsrc((l < 32 || KIND == K_CRITIC) ? ret + row0 : V + row0, nb), vo);
  float s1 = 0.0f;
  if (KIND != K_CRITIC) s1 = bload(rsrc((l < 32 || act == nullptr) ? lp + row0 : act + row0, nb), vo);
#pragma unroll
  for (int i = 0; i < NX; i++) slot[G::IN_X + l + 64 * i] = x[i];
  slot[G::IN_S0 + l] = s0;
  slot[G::IN_S1 + l] = s1;
}

// Inputs of this wave's tiles: LDS-DMA one tile ahead into the double-buffered slot; the ragged
// last tile loads synchronously.  body(slot, row0, nrows) runs each tile.  (Two tiles ahead in a
// three-slot ring measured no faster: 1.764 / 1.867-1.871 ms vs 1.749-1.776 / 1.869-1.871 ms per
// critic / actor launch, profiles/r04_x3_probe/ab_pf2.txt.)
template <int KIND, class G>
__device__ __forceinline__ void prefetch_any(const WaveSlot<G> &ws, float *slot, int64_t row0, const float *X, int nin,
                                             const float *ret, const float *V, const float *act, const float *lp_old,
                                             int64_t M) {
  if constexpr (G::NIC == NIN_CONT) prefetch_tile<KIND, LY>(slot, X, ret, V, act, lp_old, row0, ws.l, M);
  else prefetch_g<KIND, G>(slot, X, nin, ret, V, act, lp_old, row0, ws.l, M);
}
// The first tile's LDS-DMA, issued by the kernel before it stages the weights (its own slot is
// disjoint from the weight images), so the HBM latency of the first inputs overlaps the staging;
// tile_loop(..., first_issued = true) then skips it.
template <int KIND, class G>
__device__ __forceinline__ void prefetch_first(const WaveSlot<G> &ws, int64_t gw, int64_t M, const float *X, int nin,
                                               const float *ret, const float *V, const float *act,
                                               const float *lp_old) {
  if (gw < uniform_i64(M / 32)) prefetch_any<KIND, G>(ws, ws.inb, gw * 32, X, nin, ret, V, act, lp_old, M);
}

template <int KIND, class G, class Body>
__device__ __forceinline__ void tile_loop(const WaveSlot<G> &ws, int64_t gw, int64_t nw, int64_t M, const float *X,
                                          int nin, const float *ret, const float *V, const float *act,
                                          const float *lp_old, Body &&body, bool first_issued = false) {
  const int64_t ntiles = uniform_i64((M + 31) / 32), nfull = uniform_i64(M / 32);
  constexpr bool FIXED = G::NIC == NIN_CONT;  // the 13-input heads: the f32 path's slot loaders
  auto prefetch = [&](float *slot, int64_t row0) {
    prefetch_any<KIND, G>(ws, slot, row0, X, nin, ret, V, act, lp_old, M);
  };
  int cb = 0;
  MHPPO_MARK(0);
  if (gw < nfull && !first_issued) prefetch(ws.inb, gw * 32);
  for (int64_t tile = gw; tile < ntiles; tile += nw, cb ^= 1) {
    const int64_t row0 = tile * 32;
    const int nrows = (int)min((int64_t)32, M - row0);
    float *slot = ws.inb + cb * G::IN_SZ;
    const int64_t nxt = tile + nw;
    if (nxt < nfull) {
      prefetch(ws.inb + (cb ^ 1) * G::IN_SZ, nxt * 32);
      if constexpr (FIXED) wait_vmcnt<prefetch_ops<KIND>()>();
      else wait_vmcnt<prefetch_g_ops<KIND, G>()>();
    } else if (tile < nfull) {
      wait_vmcnt<0>();
    } else {
      if constexpr (FIXED) load_tile_sync<KIND, LY>(slot, X, NIN_CONT, ret, V, act, lp_old, row0, nrows, ws.l);
      else load_sync_g<KIND, G>(slot, X, nin, ret, V, act, lp_old, row0, nrows, ws.l);
    }
    wave_sync();  // the tile's inputs have landed
    MHPPO_MARK(1);  // timing builds: the tile-input wait
    body(slot, row0, nrows);
  }
  MHPPO_MARK_FLUSH();
}
// The four waves' gradient partials folded per block through LDS (fixed order, float64): one
// float64 partial per block, a quarter of the per-wave partials' bytes for the two-stage
// reduction to write and read.  The weight images and tile slots are dead once every wave has
// left its tile loop (the first barrier); the second publishes the four partials.
template <class G, class PassT>
__device__ __forceinline__ void fold_partials(PassT &p, const WaveSlot<G> &ws, char *L8, int w, int tid, int np,
                                              double *__restrict__ gblk, double *__restrict__ dblk) {
  static_assert(WAVES * Packed(G::K1 - 1, G::NOUT).NP * 4 + 8 + WAVES * 3 * 8 <= G::LDS_BYTES,
                "the four partials fit the kernel's LDS");
  __syncthreads();
  float *part = reinterpret_cast<float *>(L8);
  double *dl = reinterpret_cast<double *>(L8 + (WAVES * np * 4 + 7) / 8 * 8);
  p.finish(ws, part + w * np, dl + w * 3);
  __syncthreads();
  for (int k = tid; k < np; k += 64 * WAVES)
    gblk[k] = (((double)part[k] + (double)part[np + k]) + (double)part[2 * np + k]) + (double)part[3 * np + k];
  if (tid < 3) dblk[tid] = ((dl[tid] + dl[3 + tid]) + dl[6 + tid]) + dl[9 + tid];
}
}  // namespace x3

#ifndef MHPPO_X3_BS
#define MHPPO_X3_BS 7  // bits: 1 critic passes, 2 actor passes, 4 the fused pair (A/B builds override)
#endif
constexpr bool X3_BS_CRITIC = MHPPO_X3_BS & 1, X3_BS_ACTOR = MHPPO_X3_BS & 2, X3_BS_PAIR = MHPPO_X3_BS & 4;
// the 13-input critic pass: bits 0-1 = forward fragments held in registers (1 W2, 2 W3), bit 2 =
// dW4 in registers, bit 3 = DH2F + XCE ordering
// 15: dW4 in registers, DH2F + XCE, W2's and W3's forward fragments held (the hand-placed passes
// have the registers since the forward writes the h images: 509 VGPRs; 12 -> 13 -2.1 %, 13 -> 15
// -3.5 %, profiles/r05_x3/ab.txt, ab_hf3.txt)
constexpr int X3_CRIT = 15;
constexpr int X3_CRIT_HF = X3_CRIT & 3;
constexpr int X3_CRIT_HB = 3 & ~((X3_CRIT >> 4) & 3);  // bits 4-5: backward fragments NOT held (1 W3^T, 2 W2^T)
constexpr bool X3_CRIT_W4R = X3_CRIT & 4, X3_CRIT_ORD = X3_CRIT & 8;
// the continuous actor pass: bits 0-1 = forward fragments held (1 W2, 2 W3), bits 2-3 = backward
// fragments held (1 W3^T, 2 W2^T), bit 4 = dW4 in registers, bit 5 = DH2F + XCE
// 61: both backward fragments held, dW4 in registers, DH2F + XCE, W2's forward fragments held (485
// VGPRs since the forward writes the h images; -1.5 % vs 60, profiles/r05_x3/ab.txt); 63: W3's
// forward fragments too, which fit (512 VGPRs, no spill) only with the float32 loss math
// (with a float64 exp 63 spilled 60 B)
constexpr int X3_ACT = 63;
constexpr int X3_ACT_HF = X3_ACT & 3, X3_ACT_HB = (X3_ACT >> 2) & 3;
constexpr bool X3_ACT_W4R = X3_ACT & 16, X3_ACT_ORD = X3_ACT & 32;
#ifndef MHPPO_X3_CC
#define MHPPO_X3_CC 0  // the choice critic (runtime input count), bits as X3_CRIT (A/B overrides)
#endif
#ifndef MHPPO_X3_CA
#define MHPPO_X3_CA 0  // the choice actor: bits 0-1 forward fragments held, bit 3 DH2F + XCE
#endif
constexpr int X3_CC_HF = MHPPO_X3_CC & 3, X3_CA_HF = MHPPO_X3_CA & 3;
#ifndef MHPPO_X3_SCH
#define MHPPO_X3_SCH 1  // the 13-input single-net passes with the hand-placed backward (A/B builds override)
#endif
constexpr bool X3_SCH = MHPPO_X3_SCH;
namespace x3 {
using G13P = std::conditional_t<X3_SCH, G13S, G13>;  // the 13-input single-net passes' geometry
}
constexpr bool X3_CC_W4R = MHPPO_X3_CC & 4, X3_CC_ORD = MHPPO_X3_CC & 8, X3_CA_ORD = MHPPO_X3_CA & 8;
template <int KIND, class G>
__global__ void __launch_bounds__(64 * x3::WAVES)
    k_mlp_train_x3(const float *__restrict__ W, const float *__restrict__ X, int nin, int64_t M,
                   const float *__restrict__ ret, float *__restrict__ V, const float *__restrict__ act,
                   const float *__restrict__ lp_old, const double *__restrict__ stats,
                   const double *__restrict__ counts, double m_global, float out_mean, float out_std,
                   double *__restrict__ gpart, double *__restrict__ dpart) {
  using namespace x3;
  extern __shared__ float lds[];
  char *L8 = reinterpret_cast<char *>(lds);
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const WaveSlot<G> ws(L8 + G::NET_B, w, l);
  const int64_t gw = (int64_t)blockIdx.x * WAVES + w, nw = (int64_t)gridDim.x * WAVES;
  prefetch_first<KIND, G>(ws, gw, M, X, nin, ret, V, act, lp_old);
  stage_net<G>(W, L8, tid, nin);
  __syncthreads();
  // the 13-input critic pass alone holds its forward weight fragments in registers (with a
  // runtime input count the choice critic has no registers for them: 23-38 spills)
  constexpr bool C13 = KIND == K_CRITIC && G::NIC == NIN_CONT;  // the 13-input critic
  constexpr bool A13 = KIND == K_CONT;
  constexpr bool CC = KIND == K_CRITIC && !C13, CA = KIND == K_CHOICE;  // the choice head's nets
  constexpr bool ORD = (A13 && X3_ACT_ORD) || (C13 && X3_CRIT_ORD) || (CC && X3_CC_ORD) || (CA && X3_CA_ORD);
  Pass<KIND, C13 ? X3_CRIT_HF : (A13 ? X3_ACT_HF : (CC ? X3_CC_HF : X3_CA_HF)),
       A13 ? X3_ACT_HB : (C13 ? X3_CRIT_HB : 3), G,
       (KIND == K_CRITIC ? X3_BS_CRITIC : X3_BS_ACTOR), ORD, ORD,
       (A13 && X3_ACT_W4R) || (C13 && X3_CRIT_W4R) || (CC && X3_CC_W4R), (A13 || C13) && X3_SCH>
      p;
  p.init(L8, ws, nin, counts, m_global);
  float meanf = 0.f, stdf = 1.f;
  if (KIND != K_CRITIC) adv_norm(stats, m_global, meanf, stdf);
  const double inv_m = uniform_d(1.0 / m_global);
  tile_loop<KIND, G>(
      ws, gw, nw, M, X, nin, ret, V, act, lp_old,
      [&](const float *slot, int64_t row0, int nrows) {
        p.tile(ws, slot, row0, nrows, V, meanf, stdf, inv_m, out_mean, out_std);
      },
      true);
  p.drain();
  const int np = Packed(geo_nin<G>(nin), G::NOUT).NP;
  fold_partials<G>(p, ws, L8, w, tid, np, gpart + (size_t)blockIdx.x * np, dpart + blockIdx.x * 3);
}

// Actor pass of epoch e fused with the critic pass of epoch e + 1 (Algo_PPO.train_model_c
// :778-815 run as a pipeline: the actor of epoch e needs only V_e and the advantage sums of the
// critic pass e; the critic of epoch e + 1 needs only the critic's Adam step e).  Both nets
// train on the same tile: one input load, one launch and one weight-staging prologue instead of
// two.  The actor reads V_e from the tile's prefetched inputs before the critic overwrites those
// rows of V with V_{e+1} (each tile belongs to one wave; its inputs land one tile ahead).
// Partials: actor at gpart[gw], critic at gpart[nw + gw] (and dpart likewise).
__global__ void __launch_bounds__(64 * x3::WAVES)
    k_mlp_train_x3_pair(const float *__restrict__ Wa, const float *__restrict__ Wc, const float *__restrict__ X,
                        int64_t M, const float *__restrict__ ret, float *__restrict__ V,
                        const float *__restrict__ act, const float *__restrict__ lp_old,
                        const double *__restrict__ stats, double m_global, float out_mean, float out_std,
                        double *__restrict__ gpart, double *__restrict__ dpart) {
  using namespace x3;
  extern __shared__ float lds[];
  char *L8 = reinterpret_cast<char *>(lds);
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  using G = G13;
  const WaveSlot<G> ws(L8 + 2 * G::NET_B, w, l);
  const int64_t gw = (int64_t)blockIdx.x * WAVES + w, nw = (int64_t)gridDim.x * WAVES;
  prefetch_first<K_CONT, G>(ws, gw, M, X, NIN_CONT, ret, V, act, lp_old);
  stage_net<G>(Wa, L8, tid, NIN_CONT);
  stage_net<G>(Wc, L8 + G::NET_B, tid, NIN_CONT);
  __syncthreads();
  Pass<K_CONT, false, 0, G, X3_BS_PAIR, true> pa;  // two nets in one wave: no fragments held
  Pass<K_CRITIC, false, 0, G, X3_BS_PAIR, true, false, true> pc;  // dW4 in registers as the single critic pass: the same bits
  pa.init(L8, ws);
  pc.init(L8 + G::NET_B, ws);
  float meanf, stdf;
  adv_norm(stats, m_global, meanf, stdf);
  const double inv_m = uniform_d(1.0 / m_global);
  tile_loop<K_CONT, G>(
      ws, gw, nw, M, X, NIN_CONT, ret, V, act, lp_old,
      [&](const float *slot, int64_t row0, int nrows) {
        pa.tile(ws, slot, row0, nrows, V, meanf, stdf, inv_m, out_mean, out_std);
        pc.tile(ws, slot, row0, nrows, V, 0.f, 1.f, inv_m, out_mean, out_std);
      },
      true);
  constexpr int NWP = Packed(NIN_CONT, 1).NP;
  const int64_t nb = gridDim.x, b = blockIdx.x;
  fold_partials<G>(pa, ws, L8, w, tid, NWP, gpart + (size_t)b * NWP, dpart + b * 3);
  fold_partials<G>(pc, ws, L8, w, tid, NWP, gpart + (size_t)(nb + b) * NWP, dpart + (nb + b) * 3);
}


// Deterministic two-stage gradient reduction over the per-wave partials (fixed order,
// float64): stage 1 sums contiguous groups of waves, stage 2 sums the RG group totals.
// Slot k < np is gradient k, slots np..np+2 the float64 sums.
constexpr int RG = 64;

// blockIdx.z = net: a fused pair launch reduces both nets' partials (net z's partials follow net
// z - 1's in gpart / dpart; its group totals at tmp + z RG (np + 3)) in the same two launches.
// Partials: float per wave (the f32 kernel), float64 per block (the split kernel's LDS fold).
template <class T>
__global__ void __launch_bounds__(256)
    k_grad_stage1(const T *gpart, const double *dpart, int nw, int np, double *tmp) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  const int g = blockIdx.y, nd = np + 3, z = blockIdx.z;
  gpart += (size_t)z * nw * np;
  dpart += (size_t)z * nw * 3;
  tmp += (size_t)z * RG * nd;
  const int i0 = (int)((int64_t)g * nw / RG), i1 = (int)((int64_t)(g + 1) * nw / RG);
  double s = 0.0;
  if (k < np) {
    // unrolled: the group's loads issue together (the sum order, and so the bits, unchanged)
#pragma unroll 16
    for (int i = i0; i < i1; i++) s += (double)gpart[(size_t)i * np + k];
  } else if (k < nd) {
    for (int i = i0; i < i1; i++) s += dpart[(size_t)i * 3 + (k - np)];
  } else {
    return;
  }
  tmp[(size_t)g * nd + k] = s;
}

// The split kernels' block partials (at most one per CU: nb <= 1024) in ONE launch: a 1 024-thread
// block per 64 gradient slots; thread (g, c) sums partials [g nb / 16, (g + 1) nb / 16) of slot c
// in order (16 coalesced rows per load step), then thread (0, c) adds the 16 group sums in order.
// blockIdx.y = net (the pair launch).  Fixed order: deterministic.
constexpr int RD_COLS = 64, RD_GROUPS = 16;
__global__ void __launch_bounds__(RD_COLS * RD_GROUPS)
    k_grad_reduce_blocks(const double *gpart, const double *dpart, int nb, int np, float *grad, double *out3,
                         float *grad1, double *out3_1) {
  __shared__ double red[RD_GROUPS][RD_COLS];
  const int c = blockIdx.x * RD_COLS + (threadIdx.x & (RD_COLS - 1)), g = threadIdx.x / RD_COLS;
  const int nd = np + 3;
  if (blockIdx.y) {
    gpart += (size_t)nb * np;
    dpart += (size_t)nb * 3;
    grad = grad1;
    out3 = out3_1;
  }
  const int i0 = g * nb / RD_GROUPS, i1 = (g + 1) * nb / RD_GROUPS;
  double s = 0.0;
  if (c < np) {
#pragma unroll 16
    for (int i = i0; i < i1; i++) s += gpart[(size_t)i * np + c];
  } else if (c < nd) {
    for (int i = i0; i < i1; i++) s += dpart[(size_t)i * 3 + (c - np)];
  }
  red[g][threadIdx.x & (RD_COLS - 1)] = s;
  __syncthreads();
  if (g != 0 || c >= nd) return;
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < RD_GROUPS; q++) t += red[q][threadIdx.x];
  if (c < np)
    grad[c] = (float)t;
  else if (out3)
    out3[c - np] += t;
}

__global__ void __launch_bounds__(256)
    k_grad_stage2(const double *tmp, int np, float *grad, double *out3, float *grad1, double *out3_1) {
  const int k = blockIdx.x * 256 + threadIdx.x, nd = np + 3;
  if (k >= nd) return;
  if (blockIdx.z) {
    tmp += (size_t)RG * nd;
    grad = grad1;
    out3 = out3_1;
  }
  double s = 0.0;
#pragma unroll 8
  for (int g = 0; g < RG; g++) s += tmp[(size_t)g * nd + k];
  if (k < np)
    grad[k] = (float)s;
  else if (out3)
    out3[k - np] += s;
}

struct Work {  // per-device partial buffers (calls on one device must share one stream)
  float *g = nullptr;
  double *d = nullptr;
  double *t = nullptr;
  int nw = 0;
  int cus = 0;
};
// per device and stream (up to WORK_STREAMS streams per device may run train passes concurrently:
// each stream's passes reduce through their own partial buffers)
constexpr int WORK_STREAMS = 4;
Work g_work[mhppo::MAX_DEVICES][WORK_STREAMS];
hipStream_t g_work_stream[mhppo::MAX_DEVICES][WORK_STREAMS];
int g_work_used[mhppo::MAX_DEVICES] = {0};
// partial buffers for `slots` waves' partials (a fused pair launch uses two slots per wave)
bool ensure_work(Work &wk, int slots) {
  if (wk.nw >= slots) return true;
  if (wk.g) (void)hipFree(wk.g);
  if (wk.d) (void)hipFree(wk.d);
  if (wk.t) (void)hipFree(wk.t);
  if (hipMalloc(&wk.g, sizeof(float) * (size_t)slots * NW_MAX) != hipSuccess ||
      hipMalloc(&wk.d, sizeof(double) * (size_t)slots * 3) != hipSuccess ||
      hipMalloc(&wk.t, sizeof(double) * (size_t)2 * RG * (NW_MAX + 3)) != hipSuccess) {
    wk = Work{};
    return false;
  }
  wk.nw = slots;
  return true;
}
Work *device_work(int dev, hipStream_t s) {
  int k = 0;
  while (k < g_work_used[dev] && g_work_stream[dev][k] != s) k++;
  if (k == g_work_used[dev]) {
    if (k == WORK_STREAMS) return nullptr;
    g_work_stream[dev][k] = s;
    g_work_used[dev] = k + 1;
  }
  Work &wk = g_work[dev][k];
  if (wk.cus == 0) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    wk.cus = cus;
  }
  return &wk;
}

template <int KIND, int KS, bool PF>
void launch(dim3 grid, hipStream_t s, const float *packed, const float *X, int nin, int64_t M, const float *ret,
            float *value, const float *act, const float *logp_old, const double *stats, const double *counts,
            double m_global, float out_mean, float out_std, float *gp, double *dp) {
  using LY = Lay<KS, PF, (KIND == K_CHOICE ? 2 : 1)>;
  hipLaunchKernelGGL((k_mlp_train<KIND, KS, PF>), grid, dim3(64 * LY::WAVES), sizeof(float) * LY::FLOATS, s,
                     packed, X, nin, M, ret, value, act, logp_old, stats, counts, m_global, out_mean, out_std, gp, dp);
}
}  // namespace

#ifdef MHPPO_TIMING
// A/B timing builds only (not in include/mhppo.h): copy out and clear this TU's g_timing
extern "C" int mhppo_debug_timing_train(unsigned long long *out16) {
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_timing), sizeof(unsigned long long) * 16));
  unsigned long long z[16] = {0};
  CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_timing), z, sizeof(z)));
  return MHPPO_OK;
}
#endif

extern "C" int mhppo_mlp_train(int kind, int n_in, const float *packed, const float *X, int64_t M, const float *ret,
                               float *value, const float *act, const float *logp_old, const double *stats,
                               const double *counts, double m_global, float out_mean, float out_std, float *grad,
                               double *sums, void *stream) {
  const bool exact = (kind & MHPPO_TRAIN_EXACT_F32) != 0;
  kind &= ~MHPPO_TRAIN_EXACT_F32;
  if (!grad || M < 0 || kind < K_CRITIC || kind > K_CHOICE || n_in < 1 || n_in > NIN_MAX)
    return set_error(MHPPO_EINVAL, "bad argument (kind 0..2 [| MHPPO_TRAIN_EXACT_F32], 1 <= n_in <= %d)", NIN_MAX);
  hipStream_t s = (hipStream_t)stream;
  if (M == 0) {  // an empty shard (data parallel): zero gradient, sums unchanged; X/ret/value may be NULL
    CHECK_HIP(hipMemsetAsync(grad, 0, sizeof(float) * n_params(n_in, kind == K_CHOICE ? 2 : 1), s));
    return MHPPO_OK;
  }
  if (!packed || !X || !ret || !value) return set_error(MHPPO_EINVAL, "null packed/X/ret/value");
  if (kind == K_CONT && (n_in != NIN_CONT || !act || !logp_old || !stats))
    return set_error(MHPPO_EINVAL, "continuous actor pass needs n_in 13 and act/logp_old/stats");
  if (kind == K_CHOICE && (!logp_old || !stats || (!counts && !act)))
    return set_error(MHPPO_EINVAL, "choice actor pass needs logp_old/stats and counts (or act for per-row mode)");
  if (M > ((int64_t)1 << 40)) return set_error(MHPPO_EINVAL, "M too large");
  const bool pf = n_in == NIN_CONT && kind != K_CHOICE;
  if (pf && ((uintptr_t)X & 15) != 0) return set_error(MHPPO_EINVAL, "X must be 16-byte aligned (LDS-DMA rows)");
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= mhppo::MAX_DEVICES) return set_error(MHPPO_EINVAL, "device %d >= %d", dev, mhppo::MAX_DEVICES);
  Work *wkp = device_work(dev, s);
  if (!wkp) return set_error(MHPPO_EINVAL, "train passes on more than %d streams of one device", WORK_STREAMS);
  Work &wk = *wkp;
  const bool split = pf && !exact;  // bf16x3 split-precision kernel (default for the 13-input heads)
  // the choice heads' nets (up to NIN_X3C inputs) on the split-precision kernel too (wider: f32 MFMA)
  const bool split_c = !pf && !exact && n_in <= x3::NIN_X3C;
  if (split_c && ((uintptr_t)X & 15) != 0) return set_error(MHPPO_EINVAL, "X must be 16-byte aligned (LDS-DMA rows)");
  const int waves = (split || split_c) ? x3::WAVES : (pf ? 8 : 4);
  int64_t blocks = wk.cus;  // one block per CU, grid-stride over 32-row tiles
  const int64_t tiles = (M + 31) / 32;
  blocks = std::max<int64_t>(1, std::min<int64_t>(blocks, (tiles + waves - 1) / waves));
  const int nw = (int)blocks * waves;
  if (!ensure_work(wk, nw)) return set_error(MHPPO_ENOMEM, "mlp_train partials");
  const dim3 grid((unsigned)blocks);
#define MLP_ARGS grid, s, packed, X, n_in, M, ret, value, act, logp_old, stats, counts, m_global, out_mean, out_std, wk.g, wk.d
  if (split || split_c) {
#define X3_LAUNCH(KIND_, G_)                                                                                 \
  hipLaunchKernelGGL((k_mlp_train_x3<KIND_, x3::G_>), grid, dim3(64 * x3::WAVES), x3::G_::LDS_BYTES, s, packed, X, \
                     n_in, M, ret, value, act, logp_old, stats, counts, m_global, out_mean, out_std,                 \
                     reinterpret_cast<double *>(wk.g), wk.d)
    if (split) {
      if (kind == K_CRITIC) X3_LAUNCH(K_CRITIC, G13P);
      else X3_LAUNCH(K_CONT, G13P);
    } else if (n_in <= 15) {
      if (kind == K_CRITIC) X3_LAUNCH(K_CRITIC, GV16);
      else X3_LAUNCH(K_CHOICE, GC16);
    } else if (n_in <= 31) {
      if (kind == K_CRITIC) X3_LAUNCH(K_CRITIC, GV32);
      else X3_LAUNCH(K_CHOICE, GC32);
    } else {
      if (n_in == 54) {
        if (kind == K_CRITIC) X3_LAUNCH(K_CRITIC, GV54);
        else X3_LAUNCH(K_CHOICE, GC54);
      } else if (kind == K_CRITIC) X3_LAUNCH(K_CRITIC, GV64);
      else X3_LAUNCH(K_CHOICE, GC64);
    }
#undef X3_LAUNCH
  } else if (pf) {
    if (kind == K_CRITIC)
      launch<K_CRITIC, 7, true>(MLP_ARGS);
    else
      launch<K_CONT, 7, true>(MLP_ARGS);
  } else {
    // layer-1 k-steps: inputs padded to 2 KS columns
    const int ks = n_in <= 16 ? 8 : (n_in <= 24 ? 12 : (n_in <= 32 ? 16 : (n_in <= 48 ? 24 : (n_in <= 56 ? 28 : 32))));
#define KS_CASES(KIND_)                                       \
    switch (ks) {                                             \
      case 8: launch<KIND_, 8, false>(MLP_ARGS); break;       \
      case 12: launch<KIND_, 12, false>(MLP_ARGS); break;     \
      case 16: launch<KIND_, 16, false>(MLP_ARGS); break;     \
      case 24: launch<KIND_, 24, false>(MLP_ARGS); break;     \
      case 28: launch<KIND_, 28, false>(MLP_ARGS); break;     \
      default: launch<KIND_, 32, false>(MLP_ARGS); break;     \
    }
    if (kind == K_CRITIC) {
      KS_CASES(K_CRITIC)
    } else {
      KS_CASES(K_CHOICE)
    }
#undef KS_CASES
  }
#undef MLP_ARGS
  const int np = n_params(n_in, kind == K_CHOICE ? 2 : 1);
  if (split || split_c) {  // one float64 partial per block: one reduction launch
    hipLaunchKernelGGL(k_grad_reduce_blocks, dim3((np + 3 + RD_COLS - 1) / RD_COLS), dim3(RD_COLS * RD_GROUPS), 0, s,
                       reinterpret_cast<const double *>(wk.g), wk.d, (int)blocks, np, grad, sums, nullptr, nullptr);
  } else {  // one float partial per wave: two stages
    hipLaunchKernelGGL(k_grad_stage1<float>, dim3((np + 3 + 255) / 256, RG), dim3(256), 0, s, wk.g, wk.d, nw, np,
                       wk.t);
    hipLaunchKernelGGL(k_grad_stage2, dim3((np + 3 + 255) / 256), dim3(256), 0, s, wk.t, np, grad, sums, nullptr,
                       nullptr);
  }
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

extern "C" int mhppo_mlp_train_pair(const float *packed_actor, const float *packed_critic, const float *X, int64_t M,
                                    const float *ret, float *value, const float *act, const float *logp_old,
                                    const double *stats, double m_global, float out_mean, float out_std,
                                    float *grad_actor, double *sums_actor, float *grad_critic, double *sums_critic,
                                    void *stream) {
  if (!grad_actor || !grad_critic || M < 0) return set_error(MHPPO_EINVAL, "bad argument");
  hipStream_t s = (hipStream_t)stream;
  const int np = n_params(NIN_CONT, 1);
  if (M == 0) {  // an empty shard: zero gradients, sums unchanged
    CHECK_HIP(hipMemsetAsync(grad_actor, 0, sizeof(float) * np, s));
    CHECK_HIP(hipMemsetAsync(grad_critic, 0, sizeof(float) * np, s));
    return MHPPO_OK;
  }
  if (!packed_actor || !packed_critic || !X || !ret || !value || !act || !logp_old || !stats)
    return set_error(MHPPO_EINVAL, "null pointer");
  if (M > ((int64_t)1 << 40)) return set_error(MHPPO_EINVAL, "M too large");
  if (((uintptr_t)X & 15) != 0) return set_error(MHPPO_EINVAL, "X must be 16-byte aligned (LDS-DMA rows)");
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  if (dev < 0 || dev >= mhppo::MAX_DEVICES) return set_error(MHPPO_EINVAL, "device %d >= %d", dev, mhppo::MAX_DEVICES);
  Work *wkp = device_work(dev, s);
  if (!wkp) return set_error(MHPPO_EINVAL, "train passes on more than %d streams of one device", WORK_STREAMS);
  Work &wk = *wkp;
  const int64_t tiles = (M + 31) / 32;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(wk.cus, (tiles + x3::WAVES - 1) / x3::WAVES));
  const int nw = (int)blocks * x3::WAVES;
  if (!ensure_work(wk, 2 * nw)) return set_error(MHPPO_ENOMEM, "mlp_train partials");
  hipLaunchKernelGGL(k_mlp_train_x3_pair, dim3((unsigned)blocks), dim3(64 * x3::WAVES), x3::G13::LDS_BYTES_PAIR, s,
                     packed_actor, packed_critic, X, M, ret, value, act, logp_old, stats, m_global, out_mean, out_std,
                     reinterpret_cast<double *>(wk.g), wk.d);
  // the two nets' block partials (actor [0, blocks), critic [blocks, 2 blocks)) in one launch
  hipLaunchKernelGGL(k_grad_reduce_blocks, dim3((np + 3 + RD_COLS - 1) / RD_COLS, 2), dim3(RD_COLS * RD_GROUPS), 0, s,
                     reinterpret_cast<const double *>(wk.g), wk.d, (int)blocks, np, grad_actor, sums_actor,
                     grad_critic, sums_critic);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}
