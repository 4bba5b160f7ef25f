// rollout.hip — GPU rollout collector, returns scan and PPO loss kernels (+ C-ABI).
//
// Per PPO iteration (Env_rollout.iterations_rand + Algo_PPO.train,
// Coop-MH-PPO-scalable.py:357-517, :658-684, :778-917), for N envs at once:
//   begin:  env reset -> choice features -> choice actor -> Categorical draw
//   step t: [k_policy_mfma] per (env, slot, ped) row: obs_car_ped features and the
//           cross/wait actor picked by action_d (head-sorted 32-row f32-MFMA tiles);
//           [k_sample_env] one lane per env: min over pedestrians, MVN draw,
//           log-prob, rollout-buffer writes, then the env step itself (the same
//           env_step_one the standalone step kernel runs) and the episodic min.
//   end:    reverse discounted scan per (env, slot) segment.
// Update-time kernels (advantage stats/normalise, PPO surrogates, MSE) are
// elementwise + deterministic two-pass reductions (fixed summation order).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <vector>

#include <algorithm>
#include <math.h>
#include <string.h>

#include "../../include/mhppo.h"
#include "common.h"
#include "env_body.h"
#include "rollout_dev.h"
#include "libm_glibc.h"

using namespace mhppo;

namespace mhppo {
const Cfg &env_cfg(const mhppo_env *env);
const Bufs &env_bufs(const mhppo_env *env);
int env_device(const mhppo_env *env);
}  // namespace mhppo

namespace {
constexpr int TPB = 256;

__device__ inline void stage_weights(float *lds, const float *W, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) lds[i] = W[i];
  __syncthreads();
}

// -------------------------------------------------------------- begin
// one lane per (env, slot, ped): choice features, choice actor, Categorical draw.
// LDS: the observation rows of the block's envs (one flat coalesced copy:
// a lane's features read its env's row from LDS, not one strided global load per feature), then the
// block's feature rows (row-per-lane, stride dc + 1: conflict-free), written to feat_d as ONE flat
// coalesced run of TPB x dc floats after the forward (which reads its inputs from that LDS row).
// Before: each lane stored its dc-float row straight to global memory at a dc-float stride and the
// forward read it back from there — 8.6x (cfg3) / 17x (cfg4) the algorithmic HBM traffic.
__host__ __device__ inline int choice_env_span(const Cfg &c) {  // envs a TPB-row block can touch
  return (TPB + c.nS * c.P - 1) / (c.nS * c.P) + 1;
}
// (The actor's weights are wave-uniform: read through the scalar cache as SGPR operands of the
// fmaf chains — W is a separate __restrict__ argument, so the compiler may use scalar loads — not
// staged in LDS, where every weight cost the LDS pipe a read per lane-group.)
__host__ __device__ inline size_t choice_lds_floats(const Cfg &c, int n_in) {
  return (size_t)choice_env_span(c) * c.obs_dim + (size_t)TPB * (choice_dim(c) + 1);
}
template <int V>
__global__ void __launch_bounds__(TPB)
    k_choice(Cfg c, const float *__restrict__ W, const float *u, const int32_t *forced, mhppo_rollout_bufs B) {
  extern __shared__ float lds[];
  const ObsLayout L = obs_layout(c);
  const int dc = choice_dim(c), SP = c.nS * c.P, od = L.obs_dim;
  const size_t R = (size_t)c.N * SP, r0 = (size_t)blockIdx.x * TPB;
  const int nr = (int)min((size_t)TPB, R - r0);
  float *s_obs = lds, *s_f = s_obs + (size_t)choice_env_span(c) * od;
  const size_t e0 = r0 / SP, e1 = (r0 + nr - 1) / SP;  // the block's envs [e0, e1]
  const int nobs = (int)(e1 - e0 + 1) * od;
  for (int i = threadIdx.x; i < nobs; i += TPB) s_obs[i] = B.obs[e0 * od + i];
  __syncthreads();
  const int t = threadIdx.x;
  const size_t r = r0 + t;
  const int fs = dc + 1;  // LDS feature-row stride (odd: conflict-free row-per-lane access)
  float *f = s_f + (size_t)t * fs;
  if (t < nr) {
    const int p = (int)(r % c.P), i = (int)((r / c.P) % c.nS);
    const size_t e = r / SP;
    const float *o = s_obs + (e - e0) * od;
    obs_car_ped_d(o, L, i, p, f);
    if (p == 0) {
      B.closest[e * c.nS + i] = closest_ped_d(o, L, i);
      B.exist[e * c.nS + i] = L.scalable ? (uint8_t)(o[i * L.cw + 6] != 0.0f) : (uint8_t)1;
    }
    float pr[2];
    // the scalable 8-slot head (dc 54) and the coop / 4cars 4-slot one (27) fully unrolled
    if (dc == 54) mlp_forward_rows<54, 2>(W, f, pr);
    else if (dc == 27) mlp_forward_rows<27, 2>(W, f, pr);
    else mlp_forward<0, 2>(W, dc, f, pr);
    // Softmax over the pair (Model_PPO type 2, :81-85)
    float mx = pr[0] > pr[1] ? pr[0] : pr[1];
    float ex0 = mhppo_expf(pr[0] - mx), ex1 = mhppo_expf(pr[1] - mx);
    float s = ex0 + ex1;
    float p0 = ex0 / s, p1 = ex1 / s;
    reinterpret_cast<float2 *>(B.probs_d)[r] = make_float2(p0, p1);
    if ((p0 != p0 || p1 != p1) && B.status) atomicOr(B.status, 1u);  // Categorical raises on NaN probs
    // Categorical(probs): normalise, clamp to [eps, 1-eps], log (torch/distributions/utils.py)
    float sum = p0 + p1;
    float n0 = p0 / sum, n1 = p1 / sum;
    int a = forced ? forced[r] : (u[r] >= n0 ? 1 : 0);
    const float eps = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
    float pn = a ? n1 : n0;
    pn = pn < eps ? eps : (pn > hi ? hi : pn);
    B.a_d[r] = a;
    B.logp_d[r] = logf(pn);
  }
  __syncthreads();
  // the block's feature rows [r0, r0 + nr) x dc: one contiguous run of floats
  float *dst = B.feat_d + r0 * dc;
  for (int k = t; k < nr * dc; k += TPB) dst[k] = s_f[(k / dc) * fs + k % dc];
}

// -------------------------------------------------------------- step
// one lane per (env, slot, ped): obs_car_ped features + cross/wait actor
// Record index of segment s = env * nS + slot in the time-major records: B.rec_of[s] in the
// compact layout (-1: the segment stores no record), else s (include/mhppo.h mhppo_rollout_bufs)
// The compact layout is the scalable env's only (the variant whose car slots can be absent;
// mhppo_rollout_begin rejects rec_of for the others), so the other variants compile without it.
template <int V>
__device__ __forceinline__ const int32_t *rec_map(const mhppo_rollout_bufs &B) {
  return V == V_SCALABLE ? B.rec_of : nullptr;
}
template <int V>
__device__ __forceinline__ int64_t rec_index(const mhppo_rollout_bufs &B, int64_t s) {
  const int32_t *m = rec_map<V>(B);
  return m ? (int64_t)m[s] : s;
}
// feat_c row of policy row r = (env, slot, ped): with one pedestrian and the compact layout, feat_c
// is the step's record obs_c[t] and row r its segment's record (-1: none)
template <int V>
__device__ __forceinline__ int64_t feat_row(const mhppo_rollout_bufs &B, int P, int64_t r) {
  return P == 1 ? rec_index<V>(B, r) : r;
}

#ifdef MHPPO_TEST_KERNELS
// The VALU policy kernels (test build only, tests/lib/libmhppo_test.so: the bit-identity reference of
// k_policy_mfma, tests/test_rollout_gpu.py).  The shipped library runs k_policy_mfma alone.
template <int V>
__global__ void __launch_bounds__(TPB) k_policy(Cfg c, mhppo_mlp mc, mhppo_mlp mw, mhppo_rollout_bufs B) {
  extern __shared__ float lds[];
  const int sz = mlp_size(NF_C, 1);
  for (int i = threadIdx.x; i < sz; i += blockDim.x) {
    lds[i] = mc.packed[i];
    lds[sz + i] = mw.packed[i];
  }
  __syncthreads();
  const ObsLayout L = obs_layout(c);
  size_t r = (size_t)blockIdx.x * TPB + threadIdx.x;
  size_t R = (size_t)c.N * c.nS * c.P;
  if (r >= R) return;
  int p = (int)(r % c.P), i = (int)((r / c.P) % c.nS);
  size_t e = r / ((size_t)c.P * c.nS);
  const float *o = B.obs + e * L.obs_dim;
  float f[NF_C];
  float ex = obs_car_ped(o, L, i, p, f);
  const int64_t fr = feat_row<V>(B, c.P, (int64_t)r);
  if (fr >= 0) {
    float *fo = B.feat_c + fr * NF_C;
#pragma unroll
    for (int k = 0; k < NF_C; k++) fo[k] = f[k];
  }
  if (L.scalable && ex == 0.0f) return;  // `if exist:` gate of the scalable driver (:439)
  // action_d = 2*a - 1; cross head when action_d <= 0 (:440-445)
  bool wait = (2 * B.a_d[r] - 1) > 0;
  const float *W = wait ? lds + sz : lds;
  const mhppo_mlp &m = wait ? mw : mc;
  float out;
  mlp_forward<NF_C, 1>(W, NF_C, f, &out);
  // Model_PPO type 1: tanh(x) * std + mean (:87-89), two roundings
  float t = mhppo_tanhf(out) * m.std;
  B.out_c[r] = t + m.mean;
}

// Head-sorted policy step.  mhppo_rollout_begin lists the rows (env, slot, ped) of the
// cross head, then those of the wait head (B.rows, counts at [R], [R+1]; the choice is
// fixed for the episode); each wave takes 64 rows of ONE head, so the actor weights are
// wave-uniform and stream through the scalar cache as SGPR operands of the FMAs.  (With
// per-lane heads the weights come from LDS, and 64 lanes reading one weight cost the LDS
// pipe 64 words: that, not the FMAs, bounds k_policy.)  Same features, same fmaf chains:
// bit-identical to k_policy.  (Stale MT19937 blocks are regenerated once per episode, by the
// reset kernel: see k_policy_mfma.)
template <int V>
__global__ void __launch_bounds__(TPB) k_policy_sorted(Cfg c, const float *__restrict__ Wc,
                                                       const float *__restrict__ Ww, float mean_c, float std_c,
                                                       float mean_w, float std_w, mhppo_rollout_bufs B, Bufs eb) {
  const int lane = threadIdx.x & 63;
  const int gw = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (TPB / 64) + (threadIdx.x >> 6)));
  const int R = c.N * c.nS * c.P;
  const int32_t *__restrict__ rows = B.rows;
  const int nc = __builtin_amdgcn_readfirstlane(rows[R]), nw = __builtin_amdgcn_readfirstlane(rows[R + 1]);
  const int wc = (nc + 63) / 64;
  int head, k0, kend;
  if (gw < wc) {
    head = 0, k0 = gw * 64, kend = nc;
  } else {
    const int w2 = gw - wc;
    if (w2 * 64 >= nw) return;
    head = 1, k0 = nc + w2 * 64, kend = nc + nw;
  }
  const int k = k0 + lane;
  if (k >= kend) return;
  const int r = rows[k];
  const ObsLayout L = obs_layout(c);
  const int p = r % c.P, i = (r / c.P) % c.nS;
  const int e = r / (c.P * c.nS);
  const float *o = B.obs + (size_t)e * L.obs_dim;
  float f[NF_C];
  float ex = obs_car_ped(o, L, i, p, f);
  const int64_t fr = feat_row<V>(B, c.P, r);
  if (fr >= 0) {
    float *fo = B.feat_c + fr * NF_C;
#pragma unroll
    for (int q = 0; q < NF_C; q++) fo[q] = f[q];
  }
  if (L.scalable && ex == 0.0f) return;  // `if exist:` gate of the scalable driver (:439)
  const float out = mlp_forward13_rows(head ? Ww : Wc, f);
  // Model_PPO type 1: tanh(x) * std + mean (:87-89), two roundings
  const float t = mhppo_tanhf(out) * (head ? std_w : std_c);
  B.out_c[r] = t + (head ? mean_w : mean_c);
}
#endif  // MHPPO_TEST_KERNELS

// ------------------------------------------------------- MFMA policy step
// k_policy_mfma: the head-sorted rows as 32-row tiles on f32 MFMA (v_mfma_f32_32x32x2_f32, the
// forward layout of mlp_train.hip: rows on the lanes, features in the 16 C registers), both
// actors' weights in LDS.  Bit-identical to mlp_forward13_rows: the f32 MFMA is a k-ordered
// fmaf chain (cdna_hip_programming.md §3), and the weight rows of layers 1-3 are staged
// permuted so that C register s of lane half kh holds neuron 2s + kh — k-step s of the next
// layer then feeds its inputs 2s, 2s + 1, i.e. every chain runs in ascending input order;
// the 32 -> 1 output is the same ascending fmaf chain over both lane halves.
#ifndef MHPPO_POLICY_BLOCKS_PER_CU
#define MHPPO_POLICY_BLOCKS_PER_CU 4  // k_policy_mfma blocks resident per CU (A/B builds override)
#endif
#ifndef MHPPO_POLICY_TPB
// k_policy_mfma block size: 4 waves share one LDS copy of the two actors (38.7 KB), four blocks per CU
// (the LDS bound) give four waves per SIMD (<= 128 VGPRs) to hide the MFMA chains' layer-to-layer
// latency.  r06: 256-thread blocks, more of them than fit at once at large N (below), against
// 512-thread blocks two per CU: cfg4 collect 10.85 -> 9.86 ms, cfg3 5.93 -> 5.80 ms
#define MHPPO_POLICY_TPB 256
#endif
constexpr int PTPB = MHPPO_POLICY_TPB;
namespace pol {
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int S1 = 15, S2 = 33, S3 = 65;  // odd LDS row strides: conflict-free operand reads
constexpr int O_W1 = 0, O_B1 = O_W1 + 32 * S1, O_W2 = O_B1 + 32, O_B2 = O_W2 + 64 * S2, O_W3 = O_B2 + 64,
              O_B3 = O_W3 + 32 * S3, O_W4 = O_B3 + 32, O_B4 = O_W4 + 32, HEAD = (O_B4 + 1 + 3) / 4 * 4;
// C-tile row i = (r & 3) + 8 (r >> 2) + 4 kh of register r carries neuron 2 r + kh
__device__ __forceinline__ int neuron_of_row(int i) { return 2 * ((i & 3) + 4 * (i >> 3)) + ((i >> 2) & 1); }
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; i++) z[i] = 0.0f;
  return z;
}
// v[r] = relu(v[r] + b[row(r)]) with the oracle's relu (x < 0 ? 0 : x)
__device__ __forceinline__ void bias_relu(f32x16 &v, const float *b, int kh) {
  const float4 *b4 = reinterpret_cast<const float4 *>(b);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const float4 c = b4[2 * q + kh];
    v[4 * q + 0] = relu(v[4 * q + 0] + c.x);
    v[4 * q + 1] = relu(v[4 * q + 1] + c.y);
    v[4 * q + 2] = relu(v[4 * q + 2] + c.z);
    v[4 * q + 3] = relu(v[4 * q + 3] + c.w);
  }
}
// LDS row holding neuron n (0..31) in the permuted staging above: the inverse of neuron_of_row
__device__ __forceinline__ int row_of_neuron(int n) {
  const int m = n >> 1;
  return (m & 3) + 8 * (m >> 2) + 4 * (n & 1);
}
// Both 13 -> 32 -> 64 -> 32 -> 1 actors (torch-packed W) into LDS, [2][HEAD], the weight rows
// of layers 1-3 permuted as above (LDS row i of a layer holds neuron neuron_of_row(i)), W1 rows
// zero-padded to S1.  Every global load of both nets is issued first (coalesced, in source
// order, none waiting on another), then the permuted LDS stores: one memory round trip per
// block (a strided load -> store loop per array costs ~20 dependent trips per net at the start
// of every policy launch).
template <int NT>
__device__ __forceinline__ void stage_both(float *L, const float *__restrict__ Wa, const float *__restrict__ Wb,
                                           int tid) {
  constexpr int NW1 = 32 * NF_C, N1 = (NW1 + NT - 1) / NT, N2 = 2048 / NT;
  static_assert(2048 % NT == 0 && NT >= 64, "stage_both: block size");
  const float *W[2] = {Wa, Wb};
  float v1[2][N1], v2[2][N2], v3[2][N2], vb1[2], vb2[2], vb3[2], vw4[2], vb4[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const float *w1 = W[h], *b1 = w1 + NW1, *w2 = b1 + 32, *b2 = w2 + 2048, *w3 = b2 + 64, *b3 = w3 + 2048,
                *w4 = b3 + 32, *b4 = w4 + 32;
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int x = tid + q * NT;
      v1[h][q] = x < NW1 ? w1[x] : 0.0f;
    }
#pragma unroll
    for (int q = 0; q < N2; q++) {
      v2[h][q] = w2[tid + q * NT];
      v3[h][q] = w3[tid + q * NT];
    }
    vb1[h] = tid < 32 ? b1[tid] : 0.0f;
    vb3[h] = tid < 32 ? b3[tid] : 0.0f;
    vw4[h] = tid < 32 ? w4[tid] : 0.0f;
    vb2[h] = tid < 64 ? b2[tid] : 0.0f;
    vb4[h] = tid == 0 ? b4[0] : 0.0f;
  }
#pragma unroll
  for (int h = 0; h < 2; h++) {
    float *Lh = L + h * HEAD;
#pragma unroll
    for (int q = 0; q < N1; q++) {
      const int x = tid + q * NT;
      if (x < NW1) {
        const int n = x / NF_C, k = x - n * NF_C;
        Lh[O_W1 + row_of_neuron(n) * S1 + k] = v1[h][q];
      }
    }
    if (tid < 64) Lh[O_W1 + (tid >> 1) * S1 + NF_C + (tid & 1)] = 0.0f;  // padding columns 13, 14
#pragma unroll
    for (int q = 0; q < N2; q++) {
      const int x = tid + q * NT;
      const int n2 = x >> 5, k2 = x & 31;  // W2 [64][32]
      Lh[O_W2 + ((n2 & 32) + row_of_neuron(n2 & 31)) * S2 + k2] = v2[h][q];
      const int n3 = x >> 6, k3 = x & 63;  // W3 [32][64]
      Lh[O_W3 + row_of_neuron(n3) * S3 + k3] = v3[h][q];
    }
    if (tid < 32) {
      Lh[O_B1 + row_of_neuron(tid)] = vb1[h];
      Lh[O_B3 + row_of_neuron(tid)] = vb3[h];
      Lh[O_W4 + tid] = vw4[h];
    }
    if (tid < 64) Lh[O_B2 + (tid & 32) + row_of_neuron(tid & 31)] = vb2[h];
    if (tid == 0) Lh[O_B4] = vb4[h];
  }
}
// One 32-row tile of one 13 -> 32 -> 64 -> 32 -> 1 actor (Wl: its LDS image above) on f32 MFMA:
// lane j of both halves holds row j's features f; returns the row's pre-tanh output in every
// lane — the oracle's ascending fmaf chains bit for bit (the permuted staging).
__device__ __forceinline__ float actor_tile(const float *Wl, const float (&f)[NF_C + 1], int j, int kh) {
  f32x16 h1 = zero16();
#pragma unroll
  for (int s = 0; s < 7; s++) {
    // both lane halves hold the row's features: the lower half takes f[2s], the upper f[2s + 1]
    // (one v_permlane32_swap; a lane-select of the two is folded into an indexed load of f,
    // which puts f in scratch memory)
    const auto x = __builtin_amdgcn_permlane32_swap(__float_as_uint(f[2 * s]), __float_as_uint(f[2 * s + 1]), false, false);
    h1 = mfma(Wl[O_W1 + j * S1 + 2 * s + kh], __uint_as_float(x[0]), h1);
  }
  bias_relu(h1, Wl + O_B1, kh);
  f32x16 h2a = zero16(), h2b = zero16();
#pragma unroll
  for (int s = 0; s < 16; s++) {
    h2a = mfma(Wl[O_W2 + j * S2 + 2 * s + kh], h1[s], h2a);
    h2b = mfma(Wl[O_W2 + (32 + j) * S2 + 2 * s + kh], h1[s], h2b);
  }
  bias_relu(h2a, Wl + O_B2, kh);
  bias_relu(h2b, Wl + O_B2 + 32, kh);
  f32x16 h3 = zero16();
#pragma unroll
  for (int s = 0; s < 16; s++) h3 = mfma(Wl[O_W3 + j * S3 + 2 * s + kh], h2a[s], h3);
#pragma unroll
  for (int s = 0; s < 16; s++) h3 = mfma(Wl[O_W3 + j * S3 + 32 + 2 * s + kh], h2b[s], h3);
  bias_relu(h3, Wl + O_B3, kh);
  float y = 0.0f;
#pragma unroll
  for (int s = 0; s < 16; s++) {
    // neuron 2s sits in register s of the lower lane half, 2s + 1 in the upper: one
    // v_permlane32_swap gives every lane both (r[0] = neuron 2s, r[1] = neuron 2s + 1 of its row)
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(h3[s]), __float_as_uint(h3[s]), false, false);
    y = fmaf(Wl[O_W4 + 2 * s], __uint_as_float(r[0]), y);
    y = fmaf(Wl[O_W4 + 2 * s + 1], __uint_as_float(r[1]), y);
  }
  return y + Wl[O_B4];
}
}  // namespace pol

// Registers for five waves per SIMD (88 VGPRs; 120 without the bound): the LDS holds four blocks per
// CU, and the fifth slot lets a policy wave share a SIMD with a cfg4 env wave of the other rollout part
// (k_sample_env_r<2, 8, 8, 1>: 404 VGPRs): collect cfg4 -0.9 %, cfg3 -0.6 %, cfg2 -1.4 %
// (profiles/r06_rollout/ab_policy_vgpr.txt)
#ifndef MHPPO_POLICY_WPE
#define MHPPO_POLICY_WPE 5
#endif
template <int V>
__global__ void __launch_bounds__(PTPB) __attribute__((amdgpu_waves_per_eu(MHPPO_POLICY_WPE)))
k_policy_mfma(Cfg c, const float *__restrict__ Wc,
                                                      const float *__restrict__ Ww, float mean_c, float std_c,
                                                      float mean_w, float std_w, mhppo_rollout_bufs B, Bufs eb,
                                                      int part, int nparts) {
  using namespace pol;
  extern __shared__ float lds[];  // [2][HEAD]: cross, wait
  const int tid = threadIdx.x, l = tid & 63, j = l & 31, kh = l >> 5;
  const int gw = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (PTPB / 64) + (tid >> 6)));
  const int nwaves = gridDim.x * (PTPB / 64);
  // No MT19937 refill here: the episode's reset kernel (k_env_reset) regenerates every stale block
  // of each env's 4-block ring (env_dev.h, MT_BLOCKS), so each env starts the episode with three
  // fresh 624-word blocks in reserve beyond its active one — more than an episode draws (reset
  // 24-61 words, a step 0-18) — and RngT twists in-lane in the (correct, never observed) case
  // that an env exhausts the whole ring within one episode.
  // A per-step refill here cost the policy step up to 25 us in the draw-heavy early steps (every
  // stale env a 624-word twist serialised in its wave) and its first step ~100 us.
  stage_both<PTPB>(lds, Wc, Ww, tid);
  __syncthreads();
  const int R = c.N * c.nS * c.P;
  const int32_t *__restrict__ rows = B.rows;
  const int nc = __builtin_amdgcn_readfirstlane(rows[R]), nw = __builtin_amdgcn_readfirstlane(rows[R + 1]);
  // this launch's rows: all of both lists, or part `part`'s run of each (k_part_bounds)
  int c0 = 0, ncp = nc, w0 = nc, nwp = nw;
  if (nparts > 1) {
    const int wb = R + 2 + nparts + 1;
    c0 = __builtin_amdgcn_readfirstlane(rows[R + 2 + part]);
    ncp = __builtin_amdgcn_readfirstlane(rows[R + 3 + part]) - c0;
    const int w0r = __builtin_amdgcn_readfirstlane(rows[wb + part]);
    w0 = nc + w0r;
    nwp = __builtin_amdgcn_readfirstlane(rows[wb + part + 1]) - w0r;
  }
  const int tc = (ncp + 31) / 32, ntiles = tc + (nwp + 31) / 32;
  const ObsLayout L = obs_layout(c);
  // software pipeline over this wave's tiles: row indices two tiles ahead, the rows'
  // observation values one tile ahead, so the gathers overlap the MFMA work
  auto tile_row = [&](int tl, bool &ok) {
    const int hd = tl >= tc;
    const int a0 = hd ? w0 + 32 * (tl - tc) : c0 + 32 * tl, a1 = hd ? w0 + nwp : c0 + ncp;
    ok = tl < ntiles && a0 + j < a1;
    return ok ? rows[a0 + j] : 0;
  };
  auto raw_of = [&](int rr) {
    const int pp = rr % c.P, ii = (rr / c.P) % c.nS, ee = rr / (c.P * c.nS);
    return feat_raw(B.obs + (size_t)ee * L.obs_dim, L, ii, pp);
  };
  bool ok_cur, ok_nxt;
  int r_cur = tile_row(gw, ok_cur);
  int r_nxt = tile_row(gw + nwaves, ok_nxt);
  FeatRaw raw_cur = raw_of(r_cur);
  for (int tile = gw; tile < ntiles; tile += nwaves) {
    bool ok_2;
    const int r_2 = tile_row(tile + 2 * nwaves, ok_2);
    const FeatRaw raw_nxt = raw_of(r_nxt);
    const int head = tile >= tc;
    const float *Wl = lds + head * HEAD;
    const bool valid = ok_cur;
    const int r = r_cur;
    float f[NF_C + 1];
    const float ex = obs_car_ped_raw(raw_cur, f);
    f[NF_C] = 0.0f;
    r_cur = r_nxt;
    ok_cur = ok_nxt;
    r_nxt = r_2;
    ok_nxt = ok_2;
    raw_cur = raw_nxt;
    const int64_t fr = valid ? feat_row<V>(B, c.P, r) : -1;
    if (fr >= 0 && kh == 0) {
      float *fo = B.feat_c + fr * NF_C;
#pragma unroll
      for (int q = 0; q < NF_C; q++) fo[q] = f[q];
    }
    const float out = actor_tile(Wl, f, j, kh);
    if (valid && kh == 0 && !(L.scalable && ex == 0.0f)) {  // `if exist:` gate (:439)
      const float t = mhppo_tanhf(out) * (head ? std_w : std_c);  // Model_PPO type 1 (:87-89)
      B.out_c[r] = t + (head ? mean_w : mean_c);
    }
  }
}

// Head lists for k_policy_sorted / k_policy_mfma (stable: each list in row order).  Pass 1 counts the
// cross rows of each 256-row block; pass 2 has every block sum the counts before it
// (and all of them, for the wait list's base), then place its rows by wave prefix.
// present: optional [R / P] segment flags (the compact record layout): rows of absent car slots join
// neither list — the policy skips them (their outputs are never read and they store no record).
// cnt[2 b] / cnt[2 b + 1]: block b's cross / wait rows.
__global__ void __launch_bounds__(TPB) k_head_count(const int32_t *a_d, int R, int32_t *cnt, const uint8_t *present,
                                                    int P) {
  __shared__ int wsum[2][TPB / 64];
  const int r = blockIdx.x * TPB + threadIdx.x;
  const bool valid = r < R && (!present || present[r / P]);
  const bool cross = valid && a_d[r] == 0;  // action_d = 2a - 1 <= 0 (:440-445)
  const uint64_t mc = __ballot(cross), mw = __ballot(valid && !cross);
  if ((threadIdx.x & 63) == 0) {
    wsum[0][threadIdx.x >> 6] = __popcll(mc);
    wsum[1][threadIdx.x >> 6] = __popcll(mw);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    int s = 0;
    for (int w = 0; w < TPB / 64; w++) s += wsum[threadIdx.x][w];
    cnt[2 * blockIdx.x + threadIdx.x] = s;
  }
}

__global__ void __launch_bounds__(TPB) k_head_place(const int32_t *a_d, int R, const int32_t *cnt, int nblk,
                                                    int32_t *rows, const uint8_t *present, int P) {
  __shared__ int red[4][TPB];
  __shared__ int wsum[2][TPB / 64];
  int cb = 0, ct = 0, wb = 0, wt = 0;  // cross / wait rows before this block and in all
  for (int b = threadIdx.x; b < nblk; b += TPB) {
    const int c = cnt[2 * b], w = cnt[2 * b + 1];
    ct += c;
    wt += w;
    if (b < (int)blockIdx.x) cb += c, wb += w;
  }
  red[0][threadIdx.x] = cb;
  red[1][threadIdx.x] = ct;
  red[2][threadIdx.x] = wb;
  red[3][threadIdx.x] = wt;
  __syncthreads();
  for (int st = TPB / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st)
      for (int k = 0; k < 4; k++) red[k][threadIdx.x] += red[k][threadIdx.x + st];
    __syncthreads();
  }
  const int cbase = red[0][0], nc = red[1][0], wbase = red[2][0], nwt = red[3][0];
  const int r = blockIdx.x * TPB + threadIdx.x;
  const bool valid = r < R && (!present || present[r / P]);
  const bool cross = valid && a_d[r] == 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t mc = __ballot(cross), mw = __ballot(valid && !cross);
  if (lane == 0) {
    wsum[0][w] = __popcll(mc);
    wsum[1][w] = __popcll(mw);
  }
  __syncthreads();
  int wc = 0, ww = 0;
  for (int q = 0; q < w; q++) wc += wsum[0][q], ww += wsum[1][q];
  const uint64_t lt = lane ? ((1ull << lane) - 1) : 0ull;
  const int ci = cbase + wc + __popcll(mc & lt);  // cross rows before r
  const int wi = wbase + ww + __popcll(mw & lt);  // wait rows before r
  if (valid) rows[cross ? ci : nc + wi] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    rows[R] = nc;
    rows[R + 1] = nwt;
  }
}

// The compact record layout (mhppo_rollout_bufs.rec_of): rank[s] = the number of flagged
// segments before s (flag[s] != 0), -1 for an unflagged one.  Two passes as the head lists:
// per-block counts, then every block sums the counts before it and ranks its rows by wave prefix.
__global__ void __launch_bounds__(TPB) k_flag_count(const uint8_t *flag, int R, int32_t *cnt) {
  __shared__ int wsum[TPB / 64];
  const int r = blockIdx.x * TPB + threadIdx.x;
  const uint64_t m = __ballot(r < R && flag[r] != 0);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int w = 0; w < TPB / 64; w++) s += wsum[w];
    cnt[blockIdx.x] = s;
  }
}
__global__ void __launch_bounds__(TPB) k_flag_rank(const uint8_t *flag, int R, const int32_t *cnt, int nblk,
                                                   int32_t *rank, int S, int32_t *pre) {
  __shared__ int red[TPB];
  __shared__ int wsum[TPB / 64];
  int before = 0;
  for (int b = threadIdx.x; b < (int)blockIdx.x && b < nblk; b += TPB) before += cnt[b];
  red[threadIdx.x] = before;
  __syncthreads();
  for (int st = TPB / 2; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  const int r = blockIdx.x * TPB + threadIdx.x;
  const bool f = r < R && flag[r] != 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t m = __ballot(f);
  if (lane == 0) wsum[w] = __popcll(m);
  __syncthreads();
  int wc = 0;
  for (int q = 0; q < w; q++) wc += wsum[q];
  const uint64_t below = lane ? (m & ((1ull << lane) - 1)) : 0ull;
  const int nbefore = red[0] + wc + __popcll(below);  // flagged segments before r
  if (r < R) rank[r] = f ? nbefore : -1;
  // pre[g] = flagged segments before segment g S (g = 0 .. R / S): per-group record ranges
  if (r < R && r % S == 0) pre[r / S] = nbefore;
  if (r == R - 1) pre[R / S] = nbefore + (f ? 1 : 0);
}

// The compact layout's step records of one full wave (the scalable env): its 64 envs' present
// segments are the records [R0, R0 + K) (R0 = the existing segments before its first env,
// mhppo_rollout_bufs.rec_of[N S + e]); each lane puts its slots' act / logp / rew at (record - R0)
// in the wave's LDS run, and the wave writes the run as lane-contiguous stores.  (Stored per lane,
// the records' 4- and 8-byte values land scattered over the run and leave as partial lines:
// +2 % HBM bytes and +4 % time for the step kernel at config 4.)
template <int CNS>
struct RecStage {
  float act[64 * CNS], logp[64 * CNS];
  double rew[64 * CNS];
};
template <int CNS>
__device__ __forceinline__ RecStage<CNS> *rec_stage_wave() {
  __shared__ RecStage<CNS> st[TPB / 64];
  return &st[(threadIdx.x >> 6) & (TPB / 64 - 1)];
}

// one lane per env: select/min over peds, MVN sample, buffers, env step, episodic min.
// All of this lane's rollout inputs are read before any buffer write so the loads
// issue as one batch; EV is the generic or the register env view.
template <class EV>
__device__ __forceinline__ void sample_env_body(EV &E, const float *__restrict__ eps, int t,
                                                const mhppo_rollout_bufs &B) {
  constexpr int V = EV::VAR;
  const Cfg &c = E.c;
  const int e = E.e;
  const ObsLayout L = obs_layout(c);
  const int S = E.nS(), P = E.nP(), T = B.T;
  PlainArr<double, 2 * EV::MAXAV> act;
  const float *o = B.obs + (size_t)e * L.obs_dim;
  // One pedestrian and a compile-time S that is a multiple of 4: this env's selected
  // feature rows are feat_c[e][0..S)[0] = S*13 contiguous floats on both sides, 16-B
  // aligned (S*52 B per env), copied as float4s.
  // With one pedestrian the selected feature row of every slot is THE row, so obs_c[t] is
  // feat_c verbatim: the host points feat_c at obs_c[t] for the policy step (rollout.py
  // collect) and nothing is copied here.  Otherwise each slot's selected row is copied.
  const bool feat_in_place = B.feat_c == B.obs_c + (size_t)t * c.N * S * NF_C && P == 1;
  // compile-time S multiple of 4: the step's act/logp/rew/ep_min records go out as vectors (the
  // identity record layout; the compact one stores each present segment's record at its index)
  constexpr bool REC_VEC = EV::CNS > 0 && EV::CNS % 4 == 0;
  // the compact layout on a full wave of the register-view step: records staged per wave (RecStage)
  constexpr bool STAGE = V == V_SCALABLE && REC_VEC;
  const int32_t *rec_of = rec_map<V>(B);
  const bool vec = REC_VEC && !rec_of;
  const int lane = threadIdx.x & 63;
  const int e0 = __builtin_amdgcn_readfirstlane(e - lane);
  const bool staged = STAGE && rec_of && e0 + 64 <= c.N;
  int R0 = 0, K = 0;
  if (staged) {  // the wave's record run (uniform loads, issued with the other inputs)
    R0 = rec_of[(size_t)c.N * S + e0];
    K = rec_of[(size_t)c.N * S + e0 + 64] - R0;
  }
  // this env's records: its present slots (exist, set by mhppo_rollout_begin) in slot order from
  // the env's first record (one prefix load and the S exist bytes, not S rank loads)
  int64_t rbase = 0;
  uint32_t emask = 0;
  if (rec_of) {
    rbase = rec_of[(size_t)c.N * S + e];
    MHPPO_UNROLL
    for (int i = 0; i < S; i++) emask |= (uint32_t)(B.exist[(size_t)e * S + i] != 0) << i;
  }
  float av[REC_VEC ? EV::CNS : 1], lv[REC_VEC ? EV::CNS : 1];
  int64_t rix[EV::CNS > 0 ? EV::CNS : EV::MAXAV];  // this step's record of each slot (-1: none)
  MHPPO_UNROLL
  for (int i = 0; i < S; i++) {
    size_t row0 = ((size_t)e * S + i) * P;
    float loc = 2.0f;  // torch.tensor(car_b[1,0]) (:435)
    int sel = 0;
    MHPPO_UNROLL
    for (int p = 0; p < P; p++) {
      // scalable `if exist:` gate (:439) on the observation's exist field; the register view
      // reads the same flag from its state (pedestrian existence never changes in a step, and
      // get_data writes exactly that flag there), not a 4-B gather of the obs row
      if constexpr (V == V_SCALABLE) {
        if (EV::CNP > 0 ? !(E.pflag(p) & F_EXIST) : o[L.ped_off + p * 9 + 7] == 0.0f) continue;
      }
      float out = B.out_c[row0 + p];
      loc = t_minimum(loc, out);
      if (out == loc) sel = p;
    }
    if (loc != loc && B.status) atomicOr(B.status, 2u);  // MultivariateNormal raises on a NaN loc
    float z = eps[(size_t)e * S + i];
    float a = loc + MVN_L * z;
    rix[i] = !rec_of ? (int64_t)e * S + i
                       : (((emask >> i) & 1u) ? rbase + __builtin_popcount(emask & ((1u << i) - 1u)) : -1);
    const int64_t bt = (int64_t)t * c.N * S + rix[i];  // time-major records [T][N S]
    if (REC_VEC && (vec || staged)) {
      av[i] = a;
      lv[i] = mvn_logp(a, loc);
    } else if (rix[i] >= 0) {
      B.act[bt] = a;
      B.logp[bt] = mvn_logp(a, loc);
    }
    if (!feat_in_place && rix[i] >= 0) {
      const float *fs = B.feat_c + (row0 + sel) * NF_C;
      float *fo = B.obs_c + bt * NF_C;
#pragma unroll
      for (int k = 0; k < NF_C; k++) fo[k] = fs[k];
    }
    act[i] = (double)a;
    // closest_ped_d starts at pedestrian 0 and only moves to another one: with one (compile-time)
    // pedestrian it is 0, and the a_d gather below does not wait on the closest[] load
    const int cp = EV::CNP == 1 ? 0 : B.closest[(size_t)e * S + i];
    act[S + i] = (double)(2 * B.a_d[row0 + cp] - 1);  // action_d_light (:423-424)
  }
  if (REC_VEC && vec) {  // this env's S records of step t are contiguous and 16-B aligned
    const size_t b0 = ((size_t)t * c.N + e) * S;
#pragma unroll
    for (int q = 0; q < (REC_VEC ? EV::CNS / 4 : 0); q++) {
      reinterpret_cast<float4 *>(B.act + b0)[q] = make_float4(av[4 * q], av[4 * q + 1], av[4 * q + 2], av[4 * q + 3]);
      reinterpret_cast<float4 *>(B.logp + b0)[q] = make_float4(lv[4 * q], lv[4 * q + 1], lv[4 * q + 2], lv[4 * q + 3]);
    }
  }
  // the episodic minima are read with the other inputs, not behind the env step's stores
  // (which the compiler may not reorder them across): no memory round trip at the end
  PlainArr<double, EV::MAXAV> epm;
  MHPPO_UNROLL
  for (int i = 0; i < S; i++) epm[i] = B.ep_min[(size_t)e * S + i];
  MHPPO_MARK(3);
  env_step_body(E, act, B.obs, nullptr);
  MHPPO_UNROLL
  for (int i = 0; i < S; i++) {
    double m = epm[i];
    double x = E.rl[i];
    epm[i] = (m != m) ? m : ((x != x) ? x : (x < m ? x : m));  // np.minimum: NaN-propagating
  }
  if constexpr (STAGE) {
    if (staged) {
      RecStage<EV::CNS> *st = rec_stage_wave<EV::CNS>();
      MHPPO_UNROLL
      for (int i = 0; i < S; i++) {
        if (rix[i] >= 0) {
          const int o = (int)(rix[i] - R0);
          st->act[o] = av[i];
          st->logp[o] = lv[i];
          st->rew[o] = E.rw[i];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int64_t base = (int64_t)t * c.N * S + R0;
      for (int j = lane; j < K; j += 64) {
        B.act[base + j] = st->act[j];
        B.logp[base + j] = st->logp[j];
        B.rew[base + j] = st->rew[j];
      }
#pragma unroll
      for (int q = 0; q < EV::CNS / 2; q++)
        reinterpret_cast<double2 *>(B.ep_min + (size_t)e * S)[q] = make_double2(epm[2 * q], epm[2 * q + 1]);
      MHPPO_MARK(10);
      MHPPO_MARK_FLUSH();
      return;
    }
  }
  if (REC_VEC && vec) {
    const size_t b0 = ((size_t)t * c.N + e) * S;
#pragma unroll
    for (int q = 0; q < (REC_VEC ? EV::CNS / 2 : 0); q++) {
      reinterpret_cast<double2 *>(B.rew + b0)[q] = make_double2(E.rw[2 * q], E.rw[2 * q + 1]);
      reinterpret_cast<double2 *>(B.ep_min + (size_t)e * S)[q] = make_double2(epm[2 * q], epm[2 * q + 1]);
    }
  } else {
    MHPPO_UNROLL
    for (int i = 0; i < S; i++) {
      if (rix[i] >= 0) B.rew[(int64_t)t * c.N * S + rix[i]] = E.rw[i];
      B.ep_min[(size_t)e * S + i] = epm[i];
    }
  }
  MHPPO_MARK(10);
  MHPPO_MARK_FLUSH();
}

template <int V>
__global__ void __launch_bounds__(TPB)
    k_sample_env(Cfg c, Bufs eb, const float *eps, int t, mhppo_rollout_bufs B, int e_lo, int e_hi) {
  int e = e_lo + blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(eb, c.N, e, e < e_hi);
  if (e >= e_hi) return;
  Env<V> E(c, eb, e);
  sample_env_body(E, eps, t, B);
}

// No MT refill in the register-view step kernel: the episode's reset kernel regenerated every stale block
// (see k_policy_mfma), and a block exhausted twice within one episode is twisted in-lane by RngT
#ifdef MHPPO_WAVE_TIMES
// A/B builds only (tools/env_waves.py): each wave's shader-clock start / end of the last launch
__device__ unsigned long long g_wave_times[2 * 8192];
#endif
template <int V, int NC, int NAV, int NP>
__global__ void __launch_bounds__(TPB)
    k_sample_env_r(Cfg c, Bufs eb, const float *eps, int t, mhppo_rollout_bufs B, int e_lo, int e_hi) {
  // envs [e_lo, e_hi) (e_lo a multiple of 64: the observation rows leave as whole wave blocks)
  const int e = e_lo + blockIdx.x * TPB + threadIdx.x;
#ifdef MHPPO_WAVE_TIMES
  const unsigned long long wt0 = __builtin_amdgcn_s_memtime();
#endif
  MHPPO_MARK(0);
  MHPPO_MARK(1);
  if (e >= e_hi) return;
  EnvR<V, NC, NAV, NP> E(c, eb, e);
  MHPPO_MARK(2);
  sample_env_body(E, eps, t, B);
#ifdef MHPPO_WAVE_TIMES
  __builtin_amdgcn_s_waitcnt(0);  // the wave's stores issued: it ends here
  const unsigned long long wt1 = __builtin_amdgcn_s_memtime();
  const int wv = e >> 6;
  if ((e & 63) == 0 && wv < 8192) {
    g_wave_times[2 * wv] = wt0;
    g_wave_times[2 * wv + 1] = wt1;
  }
#endif
}

// -------------------------------------------------------------- evaluation
// Env_rollout.iterations (:152-252; the routine Algo_PPO.evaluate runs), one lane per env
// and step: deterministic choice (argmax) when a decision is due, mean actions with the
// left-lane override and the (10 - V)/dt cap, the flat-index light quirk, env step,
// episodic min, re-decision test and saves.  Weights of the three heads in LDS.
template <int V>
__global__ void __launch_bounds__(TPB) k_eval_step(Cfg c, Bufs eb, mhppo_mlp mc, mhppo_mlp mw, mhppo_mlp md,
                                                   int t, mhppo_eval_bufs E) {
  extern __shared__ float lds[];
  const int szc = mlp_size(NF_C, 1), dc = choice_dim(c), szd = mlp_size(dc, 2);
  float *Wc = lds, *Ww = lds + szc, *Wd = lds + 2 * szc;
  for (int i = threadIdx.x; i < szc; i += blockDim.x) {
    Wc[i] = mc.packed[i];
    Ww[i] = mw.packed[i];
  }
  for (int i = threadIdx.x; i < szd; i += blockDim.x) Wd[i] = md.packed[i];
  __syncthreads();
  const int e = blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(eb, c.N, e, e < c.N);
  if (e >= c.N) return;
  const ObsLayout L = obs_layout(c);
  const int S = c.nS, P = c.P, N = c.N;
  float *o = E.obs + (size_t)e * L.obs_dim;
  int32_t *ad = E.a_d + (size_t)e * S * P;
  double *epm = E.ep_min + (size_t)e * S;
  if (t == 0 || E.trig[e]) {  // need_new_d (:175-188)
    for (int i = 0; i < S; i++) epm[i] = 0.0;
    for (int i = 0; i < S; i++)
      for (int p = 0; p < P; p++) {
        float fd[2 + 6 * (MAXS - 1) + 10], pr[2];
        obs_car_ped_d(o, L, i, p, fd);
        mlp_forward<0, 2>(Wd, dc, fd, pr);
        float mx = pr[0] > pr[1] ? pr[0] : pr[1];
        float e0 = mhppo_expf(pr[0] - mx), e1 = mhppo_expf(pr[1] - mx);
        float sm = e0 + e1;
        ad[i * P + p] = (e1 / sm > e0 / sm) ? 1 : 0;  // torch.argmax: first maximum
      }
  }
  const size_t te = (size_t)t * N + e;
  float *oh = E.obs_hist + te * L.obs_dim;
  for (int k = 0; k < L.obs_dim; k++) oh[k] = o[k];
  double act[2 * MAXS], rw[MAXS], rl[MAXS];
  for (int i = 0; i < S; i++) {
    double a = c.b10;  // np.array(car_b[1,0]) (:193)
    for (int p = 0; p < P; p++) {
      float f[NF_C];
      obs_car_ped(o, L, i, p, f);
      double cand;
      if (f[7] != 0.0f) {  // left the lane: speed-limit tracking, clamped (:196-197)
        double x = (10.0 - (double)f[0]) / c.dt;
        double m = (c.b10 < x) ? c.b10 : x;
        cand = (c.b00 > m) ? c.b00 : m;
      } else {
        const bool wait = (2 * ad[i * P + p] - 1) > 0;
        float out;
        mlp_forward<NF_C, 1>(wait ? Ww : Wc, NF_C, f, &out);
        const mhppo_mlp &m = wait ? mw : mc;
        float tt = mhppo_tanhf(out) * m.std;
        cand = (double)(tt + m.mean);
      }
      if (cand < a) a = cand;  // Python min keeps the first on ties (:205-206)
      double lim = (10.0 - (double)f[0]) / c.dt;
      if (lim < a) a = lim;
    }
    act[i] = a;
    E.acts[te * S + i] = (float)a;
  }
  for (int i = 0; i < S; i++) act[S + i] = (double)(2 * ad[i] - 1);  // action_d_light: flat index (:188, :210)
  const float prev1 = o[L.env_off + 1];
  env_step_one<V>(c, eb, e, act, E.obs, rw, rl, E.saved + (size_t)t * N);  // writes done into saved[t][e]
  const uint8_t done = E.saved[te];
  for (int i = 0; i < S; i++) {
    E.rews_c[te * S + i] = (float)rw[i];
    double m = epm[i], x = rl[i];
    epm[i] = (m != m) ? m : ((x != x) ? x : (x < m ? x : m));  // np.minimum
  }
  const float cur1 = o[L.env_off + 1];
  const uint8_t trig = L.scalable ? (cur1 != (float)P) : (cur1 != prev1);  // (:218-220)
  const uint8_t saved = trig || done;
  E.saved[te] = saved;
  E.trig[e] = trig;
  if (saved) {  // (:224-229)
    for (int i = 0; i < S; i++) E.rews_d[te * S + i] = (float)epm[i];
    for (int p = 0; p < P; p++) E.waiting[te * P + p] = (float)eb.ped[sidx(P_NF * P, P_WT * P + p, e)];
  }
}

__global__ void __launch_bounds__(TPB) k_fill_f64(double *p, size_t n, double v) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i < n) p[i] = v;
}

// --------------------------------------------------------------- noise
__global__ void __launch_bounds__(TPB) k_philox(uint64_t seed, uint64_t off, float *out, int64_t n, int normal) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  uint64_t ctr = off + (uint64_t)i;
  uint32_t c4[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x6d687070u, 0u};
  philox(c4, (uint32_t)seed, (uint32_t)(seed >> 32));
  if (normal) {
    float u1 = ((float)(c4[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
    float u2 = (float)(c4[1] >> 8) * (1.0f / 16777216.0f);
    out[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795865f * u2);
  } else {
    out[i] = (float)(c4[0] >> 8) * (1.0f / 16777216.0f);
  }
}

// The policy heads' glibc-exact transcendentals (libm_glibc.h) over float bit patterns
// first .. first + n - 1 (mod 2^32): the device side of their exhaustive pin (mhppo_libm_eval)
__global__ void __launch_bounds__(TPB) k_libm_eval(int fn, uint64_t first, int64_t n, float *out) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= n) return;
  const float x = __uint_as_float((uint32_t)(first + (uint64_t)i));
  out[i] = fn == 0 ? mhppo_tanhf(x) : (fn == 1 ? mhppo_expm1f(x) : mhppo_expf(x));
}

// rows x cols standard normals, element (r, c) from counter off + r * stride + c (one
// launch for a whole rollout's per-step MVN noise: bit-identical to `rows` 1-D calls)
__global__ void __launch_bounds__(TPB) k_philox_normal_2d(uint64_t seed, uint64_t off, uint64_t stride, float *out,
                                                          int64_t rows, int64_t cols) {
  const int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= rows * cols) return;
  const int64_t r = i / cols, cc = i - r * cols;
  const uint64_t ctr = off + (uint64_t)r * stride + (uint64_t)cc;
  uint32_t c4[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x6d687070u, 0u};
  philox(c4, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = ((float)(c4[0] >> 8) + 1.0f) * (1.0f / 16777216.0f);  // (0, 1]
  const float u2 = (float)(c4[1] >> 8) * (1.0f / 16777216.0f);
  out[i] = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853071795865f * u2);
}

// ------------------------------------------------------------ returns
// futur_rewards (:668-672): episodic_reward = rew + 0.99*episodic_reward, float64,
// then torch.tensor(..., dtype=float) -> float32
__global__ void __launch_bounds__(TPB) k_returns(const double *rew, float *ret, int64_t B, int T, double gamma) {
  int64_t b = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (b >= B) return;
  const double *r = rew + b * T;
  float *o = ret + b * T;
  double g = 0.0;
  for (int t = T - 1; t >= 0; t--) {
    g = r[t] + gamma * g;
    o[t] = (float)g;
  }
}

// time-major records [T][B]: lane b scans column b (coalesced across the wave)
// Segment-major buckets (bucket_segments; the reference's per-episode concatenation,
// Coop-MH-PPO-scalable.py:489-507), both buckets in one pass over the time-major records:
// record (t, s) of a segment s in bucket b = bucket[s] (pos[s] >= 0) goes to row pos[s]*T + t
// of bucket b.  A block owns 64 segments x 16 steps: coalesced loads of the records (64
// consecutive segments per step) into LDS, then each segment's 16 rows leave as contiguous
// runs — every record read once and every bucket row written once, in full lines.
namespace bk {
constexpr int SEGS = 64, STEPS = 16;
// LDS strides per segment, padded by one word: phase 1 writes one step of 64 consecutive
// segments per instruction, and unpadded strides (208 / 16 words) put those 64 lanes on 4
// banks (16-way conflicts on every record field)
constexpr int OBS_SEG = STEPS * NF_C + 1, V_SEG = STEPS + 1;
#ifndef MHPPO_BK_TPB
#define MHPPO_BK_TPB 1024  // 16 waves: two blocks (75 KB of LDS each) fill a CU
#endif
constexpr int BTPB = MHPPO_BK_TPB;
}
__global__ void __launch_bounds__(bk::BTPB)
    k_bucket_scatter(const int64_t *__restrict__ pos, const int8_t *__restrict__ bucket, int64_t NS, int T,
                     const float *__restrict__ obs, const float *__restrict__ act, const float *__restrict__ logp,
                     const float *__restrict__ ret, const double *__restrict__ rew, mhppo_bucket_dst d0,
                     mhppo_bucket_dst d1) {
  using namespace bk;
  __shared__ float s_obs[SEGS * OBS_SEG];
  __shared__ float s_v[3][SEGS * V_SEG];
  __shared__ double s_rew[SEGS * V_SEG];
  __shared__ int64_t s_pos[SEGS];
  __shared__ int8_t s_b[SEGS];
  const int64_t s0 = (int64_t)blockIdx.x * SEGS;
  const int t0 = blockIdx.y * STEPS;
  const int nseg = (int)min((int64_t)SEGS, NS - s0), nt = min(STEPS, T - t0);
  const int tid = threadIdx.x;
  if (tid < SEGS) {
    s_pos[tid] = tid < nseg ? pos[s0 + tid] : -1;
    s_b[tid] = tid < nseg ? bucket[s0 + tid] : 0;
  }
  __syncthreads();
  // the observation records of one step of the block's 64 segments are 64 x 13 consecutive
  // floats: lanes read them as one flat run (every load instruction on two 128-byte lines), all
  // of a lane's loads issued before its first LDS store.  Only records of bucketed segments are
  // loaded (exec-masked): the scalable env's non-existent slots (pos < 0) cost no fetch unless a
  // bucketed neighbour shares their 128-byte line.
  {
    constexpr int NQ = SEGS * NF_C * STEPS / BTPB;
    static_assert(SEGS * NF_C * STEPS % BTPB == 0, "bucket scatter: block size");
    float v[NQ];
    int at[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const int i = tid + q * BTPB, tl = i / (SEGS * NF_C), k = i - tl * (SEGS * NF_C), sg = k / NF_C;
      const bool in = sg < nseg && tl < nt;
      at[q] = in && s_pos[sg] >= 0 ? sg * OBS_SEG + tl * NF_C + (k - sg * NF_C) : -1;
      v[q] = 0.0f;
      if (at[q] >= 0) v[q] = obs[((int64_t)(t0 + tl) * NS + s0) * NF_C + k];
    }
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (at[q] >= 0) s_obs[at[q]] = v[q];
  }
#pragma unroll
  for (int i = tid; i < SEGS * STEPS; i += BTPB) {  // i = step * SEGS + seg: lanes on consecutive segments
    const int sg = i % SEGS, tl = i / SEGS;
    if (sg >= nseg || tl >= nt || s_pos[sg] < 0) continue;
    const int64_t rec = (int64_t)(t0 + tl) * NS + s0 + sg;
    const int o = sg * V_SEG + tl;  // LDS: segment-major
    s_v[0][o] = act[rec];
    s_v[1][o] = logp[rec];
    s_v[2][o] = ret[rec];
    s_rew[o] = rew[rec];
  }
  __syncthreads();
  // the waves take the segments in turn: segment sg's rows pos*T + t0 .. + nt leave as one run
  const int w = tid >> 6, l = tid & 63;
  for (int sg = w; sg < nseg; sg += BTPB / 64) {
    const int64_t p = s_pos[sg];
    if (p < 0) continue;
    const mhppo_bucket_dst &D = s_b[sg] ? d1 : d0;
    const int64_t r0 = p * T + t0;
    float *oo = D.obs + r0 * NF_C;
    for (int j = l; j < nt * NF_C; j += 64) oo[j] = s_obs[sg * OBS_SEG + j];
    if (l < nt) {
      const int o = sg * V_SEG + l;
      D.act[r0 + l] = s_v[0][o];
      D.logp[r0 + l] = s_v[1][o];
      D.ret[r0 + l] = s_v[2][o];
      D.rew[r0 + l] = s_rew[o];
    }
  }
}

__global__ void __launch_bounds__(TPB) k_returns_tm(const double *rew, float *ret, int64_t B, int T, double gamma) {
  int64_t b = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (b >= B) return;
  double g = 0.0;
  for (int t = T - 1; t >= 0; t--) {
    g = rew[(int64_t)t * B + b] + gamma * g;
    ret[(int64_t)t * B + b] = (float)g;
  }
}

// ------------------------------------------------- deterministic reductions
// Pass 1 writes one partial per block (fixed in-block tree order); pass 2 sums the
// partials in index order into out[k] (+=).  NP = partial arrays per call.
template <int NP>
__device__ inline void block_reduce_store(double (&v)[NP], double *partials, int nblocks) {
  __shared__ double sh[NP][TPB];
#pragma unroll
  for (int k = 0; k < NP; k++) sh[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int s = TPB / 2; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < NP; k++) sh[k][threadIdx.x] += sh[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NP; k++) partials[(size_t)k * nblocks + blockIdx.x] = sh[k][0];
}

// one block per partial array: each thread sums a fixed strided subset, then a fixed
// tree — the summation order depends only on nblocks, never on scheduling
__global__ void __launch_bounds__(TPB) k_sum_partials(const double *partials, int nblocks, int np, double *out) {
  __shared__ double sh[TPB];
  int k = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < nblocks; b += TPB) s += partials[(size_t)k * nblocks + b];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int w = TPB / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[k] += sh[0];
}

__global__ void __launch_bounds__(TPB) k_adv_stats(const float *ret, const float *val, int64_t M, double *partials) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double v[2] = {0.0, 0.0};
  if (i < M) {
    float a = ret[i] - val[i];  // rtgs_batch - V_batch (float32, :786)
    v[0] = a;
    v[1] = (double)a * (double)a;
  }
  block_reduce_store<2>(v, partials, gridDim.x);
}

// (A - mean) / (std + 1e-10), torch.std unbiased (:787)
__global__ void __launch_bounds__(TPB)
    k_adv_norm(const float *ret, const float *val, int64_t M, const double *stats, double mg, float *adv) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= M) return;
  double mean = stats[0] / mg;
  double var = (stats[1] - stats[0] * mean) / (mg - 1.0);
  float meanf = (float)mean, stdf = (float)sqrt(var > 0 ? var : 0.0);
  float a = ret[i] - val[i];
  adv[i] = (a - meanf) / (stdf + 1e-10f);
}

__global__ void __launch_bounds__(TPB)
    k_ppo_cont(const float *mu, const float *act, const float *lp_old, const float *adv, int64_t M, double inv_m,
               float *dmu, double *partials) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double v[1] = {0.0};
  if (i < M) {
    // log_prob(action f64) (:800): diff in float64 then float32 solve, float32 tail
    float diff = (float)((double)act[i] - (double)mu[i]);
    float x = diff * MVN_INV_L;
    float lp = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HALF_LOGDET;
    double r = exp((double)lp - (double)lp_old[i]);  // float64 ratio (:803)
    double dfdr;
    double f = surr_and_grad(r, (double)adv[i], dfdr);
    v[0] = f;
    // dlogp/dmu = x / L  (d/dmu of -0.5 ((a - mu)/L)^2)
    dmu[i] = (float)(inv_m * dfdr * r * (double)x * (double)MVN_INV_L);
  }
  block_reduce_store<1>(v, partials, gridDim.x);
}

// O(M) form of the M x M Categorical broadcast (:834-842)
__global__ void __launch_bounds__(TPB)
    k_ppo_choice(const float *probs, const float *lp_old, const float *adv, int64_t M, const double *counts,
                 double inv_m2, float *dprobs, double *partials) {
  int64_t j = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double v[1] = {0.0};
  if (j < M) {
    const float eps = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
    float p0 = probs[2 * j], p1 = probs[2 * j + 1];
    float s = p0 + p1;
    float pn[2] = {p0 / s, p1 / s};
    double A = adv[j], old = lp_old[j];
    double dlp[2];
    double f = 0.0;
    for (int k = 0; k < 2; k++) {
      float pc = pn[k] < eps ? eps : (pn[k] > hi ? hi : pn[k]);
      float lp = logf(pc);
      double r = exp((double)lp - old);
      double dfdr;
      double fk = surr_and_grad(r, A, dfdr);
      f += counts[k] * fk;
      double pass = (pn[k] >= eps && pn[k] <= hi) ? 1.0 : 0.0;
      dlp[k] = inv_m2 * counts[k] * dfdr * r * pass / (double)pc;  // dL/dpn_k
    }
    v[0] = f;
    // pn_k = p_k / (p0 + p1)
    double sd = (double)s;
    double g0 = (dlp[0] * (1.0 - pn[0]) - dlp[1] * pn[1]) / sd;
    double g1 = (dlp[1] * (1.0 - pn[1]) - dlp[0] * pn[0]) / sd;
    dprobs[2 * j] = (float)g0;
    dprobs[2 * j + 1] = (float)g1;
  }
  block_reduce_store<1>(v, partials, gridDim.x);
}

__global__ void __launch_bounds__(TPB)
    k_mse(const float *val, const float *ret, int64_t M, double inv_m, float *dv, double *partials) {
  int64_t i = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double v[1] = {0.0};
  if (i < M) {
    float d = val[i] - ret[i];
    v[0] = (double)d * (double)d;
    dv[i] = (float)(2.0 * inv_m * (double)d);
  }
  block_reduce_store<1>(v, partials, gridDim.x);
}

// scratch for partial sums (per device, grown on demand, stream-ordered use)
struct Scratch {
  double *p = nullptr;
  size_t n = 0;
};
Scratch g_scratch[16];

double *scratch(size_t n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= mhppo::MAX_DEVICES) return nullptr;
  Scratch &s = g_scratch[dev];
  if (s.n < n) {
    if (s.p) (void)hipFree(s.p);
    if (hipMalloc(&s.p, n * sizeof(double)) != hipSuccess) {
      s.p = nullptr;
      s.n = 0;
      return nullptr;
    }
    s.n = n;
  }
  return s.p;
}

#define VLAUNCH(kern, variant, grid, shm, stream, ...) VLAUNCHB(kern, variant, grid, dim3(TPB), shm, stream, __VA_ARGS__)
#define VLAUNCHB(kern, variant, grid, block, shm, stream, ...)                                               \
  do {                                                                                                       \
    switch (variant) {                                                                                       \
      case V_COOP: hipLaunchKernelGGL(kern<V_COOP>, grid, block, shm, stream, __VA_ARGS__); break;           \
      case V_4CARS: hipLaunchKernelGGL(kern<V_4CARS>, grid, block, shm, stream, __VA_ARGS__); break;         \
      case V_SCALABLE: hipLaunchKernelGGL(kern<V_SCALABLE>, grid, block, shm, stream, __VA_ARGS__); break;   \
      case V_NAIF: hipLaunchKernelGGL(kern<V_NAIF>, grid, block, shm, stream, __VA_ARGS__); break;           \
      case V_STOP: hipLaunchKernelGGL(kern<V_STOP>, grid, block, shm, stream, __VA_ARGS__); break;           \
      default:                                                                                               \
        return set_error(MHPPO_EINVAL, "the rollout/evaluation drivers do not support variant %d (4cars2: "    \
                         "the reference has no driver and its followers earn no reward)", variant);          \
    }                                                                                                        \
  } while (0)

inline dim3 grid_for(size_t n) { return dim3((unsigned)((n + TPB - 1) / TPB)); }

// Dispatch-attached timing of the env-step launches (mhppo_kernel_timing_begin/_end): the
// next n launches of the calling thread on the device current at _begin record a start/stop
// pair with their dispatch.  The events belong to that device (recreated when _begin runs on
// another one) and are reused across begin/end pairs (2 * the largest n, per thread).
struct KernelTiming {
  std::vector<hipEvent_t> ev;  // [2 * cap]
  int cap = 0, used = 0, dev = -1;
  bool on = false;
};
thread_local KernelTiming g_ktime;
inline bool ktime_next(hipEvent_t &a, hipEvent_t &b) {
  KernelTiming &k = g_ktime;
  if (!k.on || k.used >= k.cap) return false;
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev != k.dev) return false;  // a launch on another device: untimed
  a = k.ev[2 * k.used];
  b = k.ev[2 * k.used + 1];
  k.used++;
  return true;
}

// register-view rollout step for a compiled shape (4cars2 has no rollout driver)
template <int V, int NC, int NAV, int NP>
bool launch_sample_reg(const Cfg &c, const Bufs &eb, const float *eps, int t, const mhppo_rollout_bufs &B,
                       hipStream_t s, int e_lo, int e_hi) {
  if constexpr (V == V_4CARS2) {
    return false;
  } else {
    if (!use_reg_view(c, V, NC, NAV, NP)) return false;
    const dim3 g = grid_for((size_t)(e_hi - e_lo));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (ktime_next(e0, e1))  // same launch, with the timing events attached to its dispatch
      hipExtLaunchKernelGGL((k_sample_env_r<V, NC, NAV, NP>), g, dim3(TPB), 0, s, e0, e1, 0, c, eb, eps, t, B, e_lo,
                            e_hi);
    else
      hipLaunchKernelGGL((k_sample_env_r<V, NC, NAV, NP>), g, dim3(TPB), 0, s, c, eb, eps, t, B, e_lo, e_hi);
    return true;
  }
}

// Env range of part `part` of `nparts` (the two-stream rollout, RolloutGPU(parts=2)): boundaries at
// multiples of 64 envs (whole waves), the last part ends at N
__host__ __device__ inline int part_env(const Cfg &c, int part, int nparts) {
  if (part >= nparts) return c.N;
  const int64_t b = ((int64_t)part * c.N / nparts + 63) / 64 * 64;
  return (int)std::min<int64_t>(b, c.N);
}

// Per part, where its rows start in the head lists: rows[R + 2 + p] = cross rows of envs before part
// p's first env, rows[R + 2 + nparts + 1 + p] = wait rows likewise (p = 0 .. nparts).  The lists
// are in row order, so a part's rows are one contiguous run of each list (binary search).
__global__ void k_part_bounds(Cfg c, int32_t *rows, int nparts) {
  const int p = threadIdx.x;
  if (p > nparts) return;
  const int R = c.N * c.nS * c.P, nc = rows[R];
  const int rb = part_env(c, p, nparts) * c.nS * c.P;
  int lo = 0, hi = nc;  // first cross index with rows[k] >= rb
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (rows[m] < rb) lo = m + 1;
    else hi = m;
  }
  rows[R + 2 + p] = lo;
  lo = nc, hi = nc + rows[R + 1];  // the wait list (absent rows, if skipped, join neither list)
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (rows[m] < rb) lo = m + 1;
    else hi = m;
  }
  rows[R + 2 + nparts + 1 + p] = lo - nc;
}

}  // namespace

extern "C" {

#ifdef MHPPO_WAVE_TIMES
extern "C" int mhppo_debug_wave_times(unsigned long long *out) {  // [2 * 8192]: start, end per wave
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_times), sizeof(unsigned long long) * 2 * 8192));
  return MHPPO_OK;
}
#endif
#ifdef MHPPO_TIMING
// A/B timing builds only (not part of include/mhppo.h): copy out and clear g_timing
int mhppo_debug_timing(unsigned long long *out16) {
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_timing), sizeof(unsigned long long) * 16));
  unsigned long long z[32] = {0};
  CHECK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_timing), z, sizeof(z)));
  return MHPPO_OK;
}
// the per-phase slowest-wave cycles (g_timing[16 + k]); read before mhppo_debug_timing clears them
int mhppo_debug_timing_max(unsigned long long *out16) {
  CHECK_HIP(hipDeviceSynchronize());
  CHECK_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_timing), sizeof(unsigned long long) * 16,
                                sizeof(unsigned long long) * 16));
  return MHPPO_OK;
}
#endif

int mhppo_choice_dim(const mhppo_env *env) { return env ? choice_dim(env_cfg(env)) : MHPPO_EINVAL; }

int mhppo_rollout_begin(mhppo_env *env, const mhppo_mlp *actor_choice, const float *u, const int32_t *forced_a,
                        mhppo_rollout_bufs *bufs, void *stream) {
  if (!env || !actor_choice || !bufs || (!u && !forced_a)) return set_error(MHPPO_EINVAL, "null argument");
  if (bufs->parts < 0 || bufs->parts > 63) return set_error(MHPPO_EINVAL, "parts %d outside [0, 63]", bufs->parts);
  if (bufs->parts > 1 && !bufs->rows) return set_error(MHPPO_EINVAL, "parts > 1 needs the head lists (rows)");
  GUARD_DEVICE(env_device(env));
  const Cfg &c = env_cfg(env);
  if (actor_choice->n_in != choice_dim(c) || actor_choice->n_out != 2)
    return set_error(MHPPO_EINVAL, "choice actor must be %d -> 2 (got %d -> %d)", choice_dim(c), actor_choice->n_in,
                     actor_choice->n_out);
  hipStream_t s = (hipStream_t)stream;
  // the NaN flags cover this episode only (a flag left by an unchecked earlier collect must not
  // surface at a later, clean iteration's mhppo_rollout_check)
  if (bufs->status) CHECK_HIP(hipMemsetAsync(bufs->status, 0, sizeof(uint32_t), s));
  int rc = mhppo_env_reset(env, bufs->obs, stream);
  if (rc) return rc;
  size_t R = (size_t)c.N * c.nS * c.P;
  size_t shm = sizeof(float) * choice_lds_floats(c, actor_choice->n_in);
  if (shm > 160 * 1024) return set_error(MHPPO_EINVAL, "choice kernel LDS %zu B (obs_dim %d, dc %d)", shm, c.obs_dim, choice_dim(c));
  VLAUNCH(k_choice, c.variant, grid_for(R), shm, s, c, actor_choice->packed, u, forced_a, *bufs);
  size_t NS = (size_t)c.N * c.nS;
  if (bufs->rec_of) {  // the compact record layout: present segments ranked in (env, slot) order
    if (c.variant != V_SCALABLE) return set_error(MHPPO_EINVAL, "rec_of: the scalable env's layout only");
    if (!bufs->exist) return set_error(MHPPO_EINVAL, "rec_of needs exist");
    const int nblk = (int)grid_for(NS).x;
    int32_t *cnt = reinterpret_cast<int32_t *>(scratch((nblk + 1) / 2));
    if (!cnt) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
    hipLaunchKernelGGL(k_flag_count, grid_for(NS), dim3(TPB), 0, s, bufs->exist, (int)NS, cnt);
    hipLaunchKernelGGL(k_flag_rank, grid_for(NS), dim3(TPB), 0, s, bufs->exist, (int)NS, cnt, nblk, bufs->rec_of,
                       c.nS, bufs->rec_of + NS);
  }
  if (bufs->rows) {  // head lists for k_policy_mfma (the choice is fixed for the episode)
    const int nblk = (int)grid_for(R).x;
    int32_t *cnt = reinterpret_cast<int32_t *>(scratch(nblk));
    if (!cnt) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
    // every row: a car slot absent at t = 0 (no record) can be present later in the episode, and its
    // action then drives the env (skipping those rows diverged the scalable reference rollout)
    const uint8_t *present = nullptr;
    hipLaunchKernelGGL(k_head_count, grid_for(R), dim3(TPB), 0, s, bufs->a_d, (int)R, cnt, present, c.P);
    hipLaunchKernelGGL(k_head_place, grid_for(R), dim3(TPB), 0, s, bufs->a_d, (int)R, cnt, nblk, bufs->rows, present,
                       c.P);
    if (bufs->parts > 1) hipLaunchKernelGGL(k_part_bounds, dim3(1), dim3(64), 0, s, c, bufs->rows, (int)bufs->parts);
  }
  hipLaunchKernelGGL(k_fill_f64, grid_for(NS), dim3(TPB), 0, s, bufs->ep_min, NS, 0.0);  // np.array([0.]*S) (:383)
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

static int rollout_policy(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                          mhppo_rollout_bufs *bufs, int part, int nparts, void *stream);

int mhppo_rollout_policy(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                         mhppo_rollout_bufs *bufs, void *stream) {
  return rollout_policy(env, actor_cross, actor_wait, bufs, 0, 1, stream);
}

int mhppo_rollout_policy_part(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                              mhppo_rollout_bufs *bufs, int part, void *stream) {
  if (!bufs) return set_error(MHPPO_EINVAL, "null argument");
  const int np = bufs->parts > 1 ? bufs->parts : 1;
  if (part < 0 || part >= np) return set_error(MHPPO_EINVAL, "part %d outside [0, %d)", part, np);
  if (np > 1 && (bufs->flags & MHPPO_ROLLOUT_VALU_POLICY))
    return set_error(MHPPO_EINVAL, "parts > 1: MFMA policy only");
  return rollout_policy(env, actor_cross, actor_wait, bufs, part, np, stream);
}

static int rollout_policy(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                          mhppo_rollout_bufs *bufs, int part, int nparts, void *stream) {
  if (!env || !actor_cross || !actor_wait || !bufs) return set_error(MHPPO_EINVAL, "null argument");
  if (actor_cross->n_in != NF_C || actor_wait->n_in != NF_C || actor_cross->n_out != 1 || actor_wait->n_out != 1)
    return set_error(MHPPO_EINVAL, "continuous actors must be 13 -> 1");
  GUARD_DEVICE(env_device(env));
  const Cfg &c = env_cfg(env);
  size_t R = (size_t)c.N * c.nS * c.P;
  if (R > (size_t)INT32_MAX - 2) return set_error(MHPPO_EINVAL, "N*S*P too large");
  if (!bufs->rows) return set_error(MHPPO_EINVAL, "the policy step needs the head lists (bufs->rows)");
  if (!(bufs->flags & MHPPO_ROLLOUT_VALU_POLICY)) {
    // persistent 32-row MFMA tiles (grid below)
    static int cus[mhppo::MAX_DEVICES] = {0};
    const int dev = env_device(env);
    if (dev < 0 || dev >= mhppo::MAX_DEVICES) return set_error(MHPPO_EINVAL, "device %d >= %d", dev, mhppo::MAX_DEVICES);
    if (!cus[dev]) {
      int n = 256;
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      cus[dev] = n;
    }
    constexpr size_t WPB = PTPB / 64;  // waves per block
    const size_t tiles = R / (32 * (size_t)nparts) + 2;
    // at least the blocks that fit at once (this part's share of them), at most one tile per wave, and
    // beyond the resident blocks ~2 tiles per wave: the waiting blocks start as the first ones drain
    // (cfg4's 8 192 tiles per part: 1 024 blocks, collect -9 %; cfg3: 513, -2 %; cfg2: 65 at one tile
    // per wave, -7 %; profiles/r06_rollout/ab_policy_grid.txt)
    const size_t resident = (size_t)MHPPO_POLICY_BLOCKS_PER_CU * cus[dev] / nparts + 1;
    const size_t blocks = std::min<size_t>(std::max<size_t>(resident, (tiles + 2 * WPB - 1) / (2 * WPB)),
                                           (tiles + WPB - 1) / WPB);
    VLAUNCHB(k_policy_mfma, c.variant, dim3((unsigned)blocks), dim3(PTPB), 2 * pol::HEAD * sizeof(float),
             (hipStream_t)stream, c, actor_cross->packed, actor_wait->packed, actor_cross->mean, actor_cross->std,
             actor_wait->mean, actor_wait->std, *bufs, env_bufs(env), part, nparts);
    CHECK_HIP(hipGetLastError());
    return MHPPO_OK;
  }
#ifdef MHPPO_TEST_KERNELS
  // the VALU reference: one wave per 64 rows of one head (at most R/64 + 2 waves), or with
  // MHPPO_ROLLOUT_VALU_POLICY | 2 the unsorted one-lane-per-row kernel
  if (bufs->flags & 2) {
    size_t shm = 2 * sizeof(float) * mlp_size(NF_C, 1);
    VLAUNCH(k_policy, c.variant, grid_for(R), shm, (hipStream_t)stream, c, *actor_cross, *actor_wait, *bufs);
  } else {
    const size_t waves = (R + 63) / 64 + 2;
    const dim3 grid((unsigned)((waves + TPB / 64 - 1) / (TPB / 64)));
    VLAUNCH(k_policy_sorted, c.variant, grid, 0, (hipStream_t)stream, c, actor_cross->packed, actor_wait->packed,
            actor_cross->mean, actor_cross->std, actor_wait->mean, actor_wait->std, *bufs, env_bufs(env));
  }
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
#else
  return set_error(MHPPO_EINVAL, "MHPPO_ROLLOUT_VALU_POLICY: the VALU policy kernels are in the test build only");
#endif
}

int mhppo_kernel_timing_begin(int n) {
  if (n < 0) return set_error(MHPPO_EINVAL, "kernel timing: n < 0");
  KernelTiming &k = g_ktime;
  k.on = false;
  k.used = 0;
  int dev = 0;
  CHECK_HIP(hipGetDevice(&dev));
  if (dev != k.dev) {  // events of another device: replace them
    for (hipEvent_t e : k.ev) (void)hipEventDestroy(e);
    k.ev.clear();
    k.cap = 0;
    k.dev = dev;
  }
  while ((int)k.ev.size() < 2 * n) {
    hipEvent_t e;
    CHECK_HIP(hipEventCreate(&e));
    k.ev.push_back(e);
  }
  if (n > k.cap) k.cap = n;
  k.on = n > 0;
  return MHPPO_OK;
}

static int kernel_timing_collect(double *ms_total, float *ms_each, int cap, int *launches) {
  KernelTiming &k = g_ktime;
  const int used = k.used;
  k.on = false;  // off before anything can fail: later launches are untimed either way
  k.used = 0;
  double tot = 0.0;
  for (int i = 0; i < used; i++) {
    CHECK_HIP(hipEventSynchronize(k.ev[2 * i + 1]));
    float ms = 0.f;
    CHECK_HIP(hipEventElapsedTime(&ms, k.ev[2 * i], k.ev[2 * i + 1]));
    tot += ms;
    if (ms_each && i < cap) ms_each[i] = ms;
  }
  if (ms_total) *ms_total = tot;
  if (launches) *launches = used;
  return MHPPO_OK;
}

int mhppo_kernel_timing_end(double *ms_total, int *launches) {
  return kernel_timing_collect(ms_total, nullptr, 0, launches);
}

int mhppo_kernel_timing_end_each(float *ms_each, int cap, int *launches) {
  if (cap < 0 || (cap > 0 && !ms_each)) return set_error(MHPPO_EINVAL, "kernel timing: bad output buffer");
  return kernel_timing_collect(nullptr, ms_each, cap, launches);
}

static int rollout_sample_env(mhppo_env *env, const float *eps, int t, mhppo_rollout_bufs *bufs, int part,
                              int nparts, void *stream) {
  if (!env || !eps || !bufs) return set_error(MHPPO_EINVAL, "null argument");
  if (t < 0 || t >= bufs->T) return set_error(MHPPO_EINVAL, "step %d outside [0, %d)", t, bufs->T);
  GUARD_DEVICE(env_device(env));
  const Cfg &c = env_cfg(env);
  // the compact layout with one pedestrian: the policy wrote each row's features at its record index,
  // which only the in-place record (feat_c = obs_c[t]) reads back at the right place
  if (bufs->rec_of && c.P == 1 && bufs->feat_c != bufs->obs_c + (size_t)t * c.N * c.nS * NF_C)
    return set_error(MHPPO_EINVAL, "rec_of with one pedestrian: feat_c must point at obs_c[t]");
  const int e_lo = part_env(c, part, nparts), e_hi = part_env(c, part + 1, nparts);
  if (e_hi <= e_lo) return MHPPO_OK;  // an empty part (N < 64 nparts)
#define SAMPLE_REG(V_, NC_, NAV_, NP_)                                                                      \
  if (launch_sample_reg<V_, NC_, NAV_, NP_>(c, env_bufs(env), eps, t, *bufs, (hipStream_t)stream, e_lo, e_hi)) { \
    CHECK_HIP(hipGetLastError());                                                                           \
    return MHPPO_OK;                                                                                        \
  }
  MHPPO_REG_SHAPES(SAMPLE_REG)
#undef SAMPLE_REG
  VLAUNCH(k_sample_env, c.variant, grid_for((size_t)(e_hi - e_lo)), 0, (hipStream_t)stream, c, env_bufs(env), eps, t,
          *bufs, e_lo, e_hi);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_rollout_sample_env(mhppo_env *env, const float *eps, int t, mhppo_rollout_bufs *bufs, void *stream) {
  return rollout_sample_env(env, eps, t, bufs, 0, 1, stream);
}

int mhppo_rollout_sample_env_part(mhppo_env *env, const float *eps, int t, mhppo_rollout_bufs *bufs, int part,
                                  void *stream) {
  if (!bufs) return set_error(MHPPO_EINVAL, "null argument");
  const int np = bufs->parts > 1 ? bufs->parts : 1;
  if (part < 0 || part >= np) return set_error(MHPPO_EINVAL, "part %d outside [0, %d)", part, np);
  return rollout_sample_env(env, eps, t, bufs, part, np, stream);
}

int mhppo_rollout_step(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait, const float *eps,
                       int t, mhppo_rollout_bufs *bufs, void *stream) {
  int rc = mhppo_rollout_policy(env, actor_cross, actor_wait, bufs, stream);
  if (rc) return rc;
  return mhppo_rollout_sample_env(env, eps, t, bufs, stream);
}

int mhppo_rollout_check(mhppo_rollout_bufs *bufs, void *stream) {
  if (!bufs) return set_error(MHPPO_EINVAL, "null argument");
  if (!bufs->status) return MHPPO_OK;
  hipStream_t s = (hipStream_t)stream;
  uint32_t st = 0;
  CHECK_HIP(hipMemcpyAsync(&st, bufs->status, sizeof(st), hipMemcpyDeviceToHost, s));
  CHECK_HIP(hipStreamSynchronize(s));
  if (!st) return MHPPO_OK;
  CHECK_HIP(hipMemsetAsync(bufs->status, 0, sizeof(uint32_t), s));
  return set_error(MHPPO_ENAN, "NaN policy output sampled (%s%s%s): the reference raises ValueError here",
                   (st & 1u) ? "Categorical probs of the choice actor, :409" : "", (st & 3u) == 3u ? "; " : "",
                   (st & 2u) ? "MultivariateNormal loc of the continuous actors, :451" : "");
}

int mhppo_eval_step(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                    const mhppo_mlp *actor_choice, int t, mhppo_eval_bufs *bufs, void *stream) {
  if (!env || !actor_cross || !actor_wait || !actor_choice || !bufs) return set_error(MHPPO_EINVAL, "null argument");
  const Cfg &c = env_cfg(env);
  if (actor_cross->n_in != NF_C || actor_wait->n_in != NF_C || actor_cross->n_out != 1 || actor_wait->n_out != 1)
    return set_error(MHPPO_EINVAL, "continuous actors must be 13 -> 1");
  if (actor_choice->n_in != choice_dim(c) || actor_choice->n_out != 2)
    return set_error(MHPPO_EINVAL, "choice actor must be %d -> 2", choice_dim(c));
  if (t < 0 || t >= bufs->T || t >= c.max_episode)
    return set_error(MHPPO_EINVAL, "step %d outside [0, %d)", t, bufs->T < c.max_episode ? bufs->T : c.max_episode);
  GUARD_DEVICE(env_device(env));
  size_t shm = sizeof(float) * (2 * mlp_size(NF_C, 1) + mlp_size(choice_dim(c), 2));
  VLAUNCH(k_eval_step, c.variant, grid_for(c.N), shm, (hipStream_t)stream, c, env_bufs(env), *actor_cross,
          *actor_wait, *actor_choice, t, *bufs);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_philox_normal(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream) {
  if (!out || n < 0) return set_error(MHPPO_EINVAL, "bad argument");
  if (n == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_philox, grid_for(n), dim3(TPB), 0, (hipStream_t)stream, seed, offset, out, n, 1);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_philox_normal_2d(uint64_t seed, uint64_t offset, uint64_t stride, float *out, int64_t rows, int64_t cols,
                           void *stream) {
  if (!out || rows < 0 || cols < 0) return set_error(MHPPO_EINVAL, "bad argument");
  if (rows == 0 || cols == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_philox_normal_2d, grid_for((size_t)(rows * cols)), dim3(TPB), 0, (hipStream_t)stream, seed,
                     offset, stride, out, rows, cols);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_philox_uniform(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream) {
  if (!out || n < 0) return set_error(MHPPO_EINVAL, "bad argument");
  if (n == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_philox, grid_for(n), dim3(TPB), 0, (hipStream_t)stream, seed, offset, out, n, 0);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_libm_eval(int fn, uint64_t first, int64_t n, float *out, void *stream) {
  if (!out || n < 0 || fn < 0 || fn > 2) return set_error(MHPPO_EINVAL, "bad argument (fn 0 tanhf, 1 expm1f, 2 expf)");
  if (n == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_libm_eval, grid_for(n), dim3(TPB), 0, (hipStream_t)stream, fn, first, n, out);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_returns_scan(const double *rew, float *ret, int64_t B, int32_t T, double gamma, void *stream) {
  if (!rew || !ret || B < 0 || T <= 0) return set_error(MHPPO_EINVAL, "bad argument");
  if (B == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_returns, grid_for(B), dim3(TPB), 0, (hipStream_t)stream, rew, ret, B, T, gamma);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_returns_scan_tm(const double *rew, float *ret, int64_t B, int32_t T, double gamma, void *stream) {
  if (!rew || !ret || B < 0 || T <= 0) return set_error(MHPPO_EINVAL, "bad argument");
  if (B == 0) return MHPPO_OK;
  hipLaunchKernelGGL(k_returns_tm, grid_for(B), dim3(TPB), 0, (hipStream_t)stream, rew, ret, B, T, gamma);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_bucket_scatter(const int64_t *pos, const int8_t *bucket, int64_t NS, int32_t T, const float *obs_tm,
                         const float *act_tm, const float *logp_tm, const float *ret_tm, const double *rew_tm,
                         const mhppo_bucket_dst *dst, void *stream) {
  if (NS < 0 || T <= 0 || !dst) return set_error(MHPPO_EINVAL, "bad argument");
  if (NS == 0) return MHPPO_OK;
  if (!pos || !bucket || !obs_tm || !act_tm || !logp_tm || !ret_tm || !rew_tm)
    return set_error(MHPPO_EINVAL, "null pointer");
  const int64_t nb = (NS + bk::SEGS - 1) / bk::SEGS;
  if (nb > 0x7fffffff) return set_error(MHPPO_EINVAL, "too many segments");
  dim3 g((unsigned)nb, (unsigned)((T + bk::STEPS - 1) / bk::STEPS));
  hipLaunchKernelGGL(k_bucket_scatter, g, dim3(bk::BTPB), 0, (hipStream_t)stream, pos, bucket, NS, (int)T, obs_tm,
                     act_tm, logp_tm, ret_tm, rew_tm, dst[0], dst[1]);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_adv_stats(const float *ret, const float *value, int64_t M, double *stats, void *stream) {
  if (M == 0) return MHPPO_OK;  // an empty shard (data parallel) adds nothing; its pointers may be NULL
  if (!ret || !value || !stats || M < 0) return set_error(MHPPO_EINVAL, "bad argument");
  dim3 g = grid_for(M);
  double *part = scratch(2 * (size_t)g.x);
  if (!part) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_adv_stats, g, dim3(TPB), 0, s, ret, value, M, part);
  hipLaunchKernelGGL(k_sum_partials, dim3(2), dim3(TPB), 0, s, part, (int)g.x, 2, stats);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_adv_normalize(const float *ret, const float *value, int64_t M, const double *stats, double m_global,
                        float *adv, void *stream) {
  if (M == 0) return MHPPO_OK;
  if (!ret || !value || !stats || !adv || M < 0) return set_error(MHPPO_EINVAL, "bad argument");
  hipLaunchKernelGGL(k_adv_norm, grid_for(M), dim3(TPB), 0, (hipStream_t)stream, ret, value, M, stats, m_global,
                     adv);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_ppo_cont_fwd_bwd(const float *mu, const float *act, const float *logp_old, const float *adv, int64_t M,
                           double inv_m, float *dmu, double *loss, void *stream) {
  if (M == 0) return MHPPO_OK;
  if (!mu || !act || !logp_old || !adv || !dmu || !loss || M < 0) return set_error(MHPPO_EINVAL, "bad argument");
  dim3 g = grid_for(M);
  double *part = scratch(g.x);
  if (!part) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ppo_cont, g, dim3(TPB), 0, s, mu, act, logp_old, adv, M, inv_m, dmu, part);
  hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(TPB), 0, s, part, (int)g.x, 1, loss);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_ppo_choice_fwd_bwd(const float *probs, const float *logp_old, const float *adv, int64_t M,
                             const double *counts, double inv_m2, float *dprobs, double *loss, void *stream) {
  if (M == 0) return MHPPO_OK;
  if (!probs || !logp_old || !adv || !counts || !dprobs || !loss || M < 0)
    return set_error(MHPPO_EINVAL, "bad argument");
  dim3 g = grid_for(M);
  double *part = scratch(g.x);
  if (!part) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_ppo_choice, g, dim3(TPB), 0, s, probs, logp_old, adv, M, counts, inv_m2, dprobs, part);
  hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(TPB), 0, s, part, (int)g.x, 1, loss);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_mse_fwd_bwd(const float *value, const float *ret, int64_t M, double inv_m, float *dv, double *loss,
                      void *stream) {
  if (M == 0) return MHPPO_OK;
  if (!value || !ret || !dv || !loss || M < 0) return set_error(MHPPO_EINVAL, "bad argument");
  dim3 g = grid_for(M);
  double *part = scratch(g.x);
  if (!part) return set_error(MHPPO_ENOMEM, "scratch allocation failed");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_mse, g, dim3(TPB), 0, s, value, ret, M, inv_m, dv, part);
  hipLaunchKernelGGL(k_sum_partials, dim3(1), dim3(TPB), 0, s, part, (int)g.x, 1, loss);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

}  // extern "C"
