// rollout_dev.h — rollout featurizers and policy MLP (host+device).
//
// The reference featurizers (Env_rollout.obs_car_ped / obs_car_ped_d /
// closest_ped_d, Coop-MH-PPO-scalable.py:526-627; coop driver
// Coop-MH-PPO.ipynb cell 0) index the float32 flat observation and do their
// arithmetic on numpy float32 scalars (NEP 50: python scalars are weak), so
// every feature is computed here in float32 from the same observation row,
// operation by operation.
//
// Two driver families:
//   scalable driver (Coop-MH-PPO-scalable.py): car rows of 7, env of 4, lines =
//     env[3], pedestrian `exist` gates the actor call and the closest-ped search,
//     choice features carry the own-car exist flag (6 per other slot);
//   coop driver (Coop-MH-PPO.ipynb; also MH-PPO.ipynb for naif, and the
//     build-defined 4cars featurization that reads the AV `car` block by key):
//     car rows of 6, env of 3, lines = env[2], 5 per other car, closest-ped
//     search seeded with pedestrian 0's distance.
#pragma once
#include "env_dev.h"

namespace mhppo {

constexpr int NF_C = 13;  // obs_car_ped width (2 + 9 + 2)

struct ObsLayout {
  int cw, env_off, ped_off, lines_idx, S, P, obs_dim, scalable;
};

MHPPO_HD inline ObsLayout obs_layout(const Cfg &c) {
  ObsLayout L;
  L.scalable = c.variant == V_SCALABLE;
  L.cw = L.scalable ? 7 : 6;
  L.S = c.nS;
  L.P = c.P;
  L.env_off = L.cw * c.nS + (c.variant == V_4CARS ? 6 * c.nS : 0);
  int ne = L.scalable ? 4 : 3;
  L.ped_off = L.env_off + ne;
  L.lines_idx = L.scalable ? 3 : 2;
  L.obs_dim = c.obs_dim;
  return L;
}

// choice feature width: scalable 2+6(S-1)+8+2, coop 2+5(S-1)+8+2
MHPPO_HD inline int choice_dim(const Cfg &c) {
  return c.variant == V_SCALABLE ? 2 + 6 * (c.nS - 1) + 10 : 2 + 5 * (c.nS - 1) + 10;
}

// Env_rollout.is_in_cross (:526-530)
MHPPO_HD inline void is_in_cross(float car_line, float ped_pos, float ped_dir, float cross_lines, float lines,
                                 float &crossing, float &dist_to_start) {
  float cross = (cross_lines * 2.0f) / lines;
  float line_start = (-cross_lines) + cross * car_line;
  float line_end = (-cross_lines) + cross * (car_line + 1.0f);
  dist_to_start = (ped_pos - line_start) * (float)(ped_dir > 0) + (line_end - ped_pos) * (float)(ped_dir < 0);
  crossing = (ped_pos > line_start && ped_pos < line_end) ? 1.0f : 0.0f;
}

// Env_rollout.leave_cross (:532-539)
MHPPO_HD inline void leave_cross(float car_line, float ped_pos, float ped_dir, float cross_lines, float lines,
                                 float &end_cross, float &dist_end) {
  float cross = (cross_lines * 2.0f) / lines;
  float line_start = (-cross_lines) + cross * car_line;
  float line_end = (-cross_lines) + cross * (car_line + 1.0f);
  if (ped_dir == -1.0f) {
    end_cross = (ped_pos < line_start) ? 1.0f : 0.0f;
    dist_end = line_start - ped_pos;
  } else {
    end_cross = (ped_pos > line_end) ? 1.0f : 0.0f;
    dist_end = ped_pos - line_end;
  }
}

// The 13 observation values obs_car_ped reads for (car i, ped p), gathered apart from the
// arithmetic so a kernel can issue the loads of the next row ahead of time.
struct FeatRaw {
  float car[6], ped[9], cl, lines;  // car[0,4] and ped[5,6] unused
};
MHPPO_HD inline FeatRaw feat_raw(const float *o, const ObsLayout &L, int i, int p) {
  const float *car = o + i * L.cw;
  const float *ped = o + L.ped_off + p * 9;
  const float *env = o + L.env_off;
  FeatRaw R;
  R.car[0] = 0.f; R.car[1] = car[1]; R.car[2] = car[2]; R.car[3] = car[3]; R.car[4] = 0.f; R.car[5] = car[5];
  R.ped[0] = ped[0]; R.ped[1] = ped[1]; R.ped[2] = ped[2]; R.ped[3] = ped[3]; R.ped[4] = ped[4];
  R.ped[5] = 0.f; R.ped[6] = 0.f; R.ped[7] = ped[7]; R.ped[8] = ped[8];
  R.cl = env[0];
  R.lines = env[L.lines_idx];
  return R;
}
MHPPO_HD inline float obs_car_ped_from(const float *car, const float *ped, float cl, float lines, float *f);

// Env_rollout.obs_car_ped (:541-572): 13 features of (car i, ped p); returns ped exist
MHPPO_HD inline float obs_car_ped(const float *o, const ObsLayout &L, int i, int p, float *f) {
  const float *car = o + i * L.cw;
  const float *ped = o + L.ped_off + p * 9;
  const float *env = o + L.env_off;
  return obs_car_ped_from(car, ped, env[0], env[L.lines_idx], f);
}
MHPPO_HD inline float obs_car_ped_raw(const FeatRaw &R, float *f) { return obs_car_ped_from(R.car, R.ped, R.cl, R.lines, f); }

MHPPO_HD inline float obs_car_ped_from(const float *car, const float *ped, float cl, float lines, float *f) {
  float crossing, dist_start, end_cross, dist_end;
  is_in_cross(car[5], ped[3], ped[8], cl, lines, crossing, dist_start);
  leave_cross(car[5], ped[3], ped[8], cl, lines, end_cross, dist_end);
  float d = ped[2] - car[3];
  float den = car[1] - ped[0];
  if (0.01f > den) den = 0.01f;  // max(car_V - ped_vx, 0.01)
  float q = d / den;
  float t = (q < 10.0f) ? q : 10.0f;  // min(10.0, q)
  float ttc = (ped[2] > car[3]) ? t : 10.0f;
  f[0] = car[1];
  f[1] = car[2];
  f[2] = ped[1];
  f[3] = (ped[2] > car[3]) ? 1.0f : 0.0f;
  f[4] = d;
  f[5] = ped[4];
  f[6] = crossing;
  f[7] = end_cross;
  f[8] = dist_start;
  f[9] = dist_end;
  f[10] = ttc;
  f[11] = cl;
  f[12] = lines;
  return ped[7];
}

// Env_rollout.obs_car_ped_d (:574-611): choice features of (car i, ped p)
MHPPO_HD inline void obs_car_ped_d(const float *o, const ObsLayout &L, int i, int p, float *f) {
  const float *car = o + i * L.cw;
  const float *ped = o + L.ped_off + p * 9;
  const float *env = o + L.env_off;
  int k = 0;
  f[k++] = car[1];
  f[k++] = car[2];
  for (int j = 0; j < L.S; j++) {
    if (j == i) continue;
    const float *c2 = o + j * L.cw;
    f[k++] = c2[1];
    f[k++] = (ped[2] > c2[3]) ? 1.0f : 0.0f;
    f[k++] = ped[2] - c2[3];
    f[k++] = c2[4];
    f[k++] = c2[5] - car[5];
    if (L.scalable) f[k++] = car[6];
  }
  float cl = env[0], lines = env[L.lines_idx];
  float crossing, dist_start, end_cross, dist_end;
  is_in_cross(car[5], ped[3], ped[8], cl, lines, crossing, dist_start);
  leave_cross(car[5], ped[3], ped[8], cl, lines, end_cross, dist_end);
  f[k++] = ped[1];
  f[k++] = (ped[2] > car[3]) ? 1.0f : 0.0f;
  f[k++] = ped[2] - car[3];
  f[k++] = ped[4];
  f[k++] = crossing;
  f[k++] = end_cross;
  f[k++] = dist_start;
  f[k++] = dist_end;
  f[k++] = cl;
  f[k++] = lines;
}

// Env_rollout.closest_ped_d (:614-627)
MHPPO_HD inline int closest_ped_d(const float *o, const ObsLayout &L, int i) {
  const float *car = o + i * L.cw;
  int min_ped = 0;
  if (L.scalable) {
    float min_d = 1000000.f;
    for (int p = 0; p < L.P; p++) {
      const float *ped = o + L.ped_off + p * 9;
      float d = ped[2] - car[3];
      if (d < min_d && ped[7] != 0.0f) { min_d = d; min_ped = p; }
    }
  } else {
    float min_d = o[L.ped_off + 2] - car[3];
    for (int p = 0; p < L.P; p++) {
      const float *ped = o + L.ped_off + p * 9;
      float d = ped[2] - car[3];
      if (d < min_d) { min_d = d; min_ped = p; }
    }
  }
  return min_ped;
}

// ------------------------------------------------------------ Model_PPO MLP
// packed torch layout: W1[32][in] b1[32] W2[64][32] b2[64] W3[32][64] b3[32] W4[out][32] b4[out]
MHPPO_HD inline int mlp_size(int n_in, int n_out) {
  return 32 * n_in + 32 + 64 * 32 + 64 + 32 * 64 + 32 + n_out * 32 + n_out;
}

MHPPO_HD inline float relu(float x) { return (x < 0.0f) ? 0.0f : x; }

// Each output accumulates its products in ascending input order with one fused
// multiply-add per term, starting from 0, the bias added last — a fixed order the
// C oracle (oracle/rollout_oracle.c) repeats bit for bit.  Layers 2 and 3 are
// fused: hidden-2 unit o2 is finished and immediately folded into the layer-3
// accumulators, which keeps layer 3's ascending-o2 order and ~70 live VGPRs.
// NIN > 0: compile-time input width (x fully in registers); NIN == 0: n_in at run
// time, x streamed from memory.
template <int NIN, int NOUT>
MHPPO_HD inline void mlp_forward(const float *W, int n_in, const float *x, float *out) {
  if (NIN > 0) n_in = NIN;
  const float *w1 = W, *b1 = w1 + 32 * n_in, *w2 = b1 + 32, *b2 = w2 + 64 * 32, *w3 = b2 + 64, *b3 = w3 + 32 * 64,
              *w4 = b3 + 32, *b4 = w4 + NOUT * 32;
  float h1[32];
#pragma unroll
  for (int o = 0; o < 32; o++) h1[o] = 0.0f;
  if (NIN > 0) {
#pragma unroll
    for (int k = 0; k < (NIN > 0 ? NIN : 1); k++) {
      float xk = x[k];
#pragma unroll
      for (int o = 0; o < 32; o++) h1[o] = fmaf(w1[o * NIN + k], xk, h1[o]);
    }
  } else {
    for (int k = 0; k < n_in; k++) {
      float xk = x[k];
#pragma unroll
      for (int o = 0; o < 32; o++) h1[o] = fmaf(w1[o * n_in + k], xk, h1[o]);
    }
  }
#pragma unroll
  for (int o = 0; o < 32; o++) h1[o] = relu(h1[o] + b1[o]);
  float h3[32];
#pragma unroll
  for (int o = 0; o < 32; o++) h3[o] = 0.0f;
  for (int o2 = 0; o2 < 64; o2++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; k++) acc = fmaf(w2[o2 * 32 + k], h1[k], acc);
    float h2 = relu(acc + b2[o2]);
#pragma unroll
    for (int o = 0; o < 32; o++) h3[o] = fmaf(w3[o * 64 + o2], h2, h3[o]);
  }
#pragma unroll
  for (int o = 0; o < 32; o++) h3[o] = relu(h3[o] + b3[o]);
#pragma unroll
  for (int j = 0; j < NOUT; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; k++) acc = fmaf(w4[j * 32 + k], h3[k], acc);
    out[j] = acc + b4[j];
  }
}

// mlp_forward's arithmetic (every output's fmaf chain in the same ascending order from 0, the bias
// added last) for a compile-time input width, output-major: with a wave-uniform W each output's
// weight row is contiguous and streams through the scalar cache (the choice actor, k_choice; hidden
// 2 kept whole before layer 3).  The per-output chains unrolled, the output loops not: fully
// unrolled, the hoisted scalar loads spilled 516 SGPRs (k_choice at cfg4 247 us, unrolled by 4:
// 252 us, rolled: 221 us; the LDS-staged generic forward before: 437 us,
// profiles/r06_rollout/k_choice_variants.txt)
template <int NIN, int NOUT>
MHPPO_HD inline void mlp_forward_rows(const float *__restrict__ W, const float *x, float *out) {
  const float *w1 = W, *b1 = w1 + 32 * NIN, *w2 = b1 + 32, *b2 = w2 + 64 * 32, *w3 = b2 + 64, *b3 = w3 + 32 * 64,
              *w4 = b3 + 32, *b4 = w4 + NOUT * 32;
  float xr[NIN], h1[32], h2[64], h3[32];
#pragma unroll
  for (int k = 0; k < NIN; k++) xr[k] = x[k];
#pragma unroll 1
  for (int o = 0; o < 32; o++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < NIN; k++) acc = fmaf(w1[o * NIN + k], xr[k], acc);
    h1[o] = relu(acc + b1[o]);
  }
#pragma unroll 1
  for (int o2 = 0; o2 < 64; o2++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; k++) acc = fmaf(w2[o2 * 32 + k], h1[k], acc);
    h2[o2] = relu(acc + b2[o2]);
  }
#pragma unroll 1
  for (int o = 0; o < 32; o++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k++) acc = fmaf(w3[o * 64 + k], h2[k], acc);
    h3[o] = relu(acc + b3[o]);
  }
#pragma unroll
  for (int j = 0; j < NOUT; j++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; k++) acc = fmaf(w4[j * 32 + k], h3[k], acc);
    out[j] = acc + b4[j];
  }
}

// The same arithmetic (every output's fmaf chain in the same ascending order, bias
// last) with the loops output-major, so each output reads its weights contiguously:
// with a wave-uniform W they stream through the scalar cache as SGPR operands.
// Hidden 2 is kept whole (64 registers) before layer 3.
MHPPO_HD inline float mlp_forward13_rows(const float *__restrict__ W, const float *x) {
  constexpr int NIN = NF_C;
  const float *w1 = W, *b1 = w1 + 32 * NIN, *w2 = b1 + 32, *b2 = w2 + 64 * 32, *w3 = b2 + 64, *b3 = w3 + 32 * 64,
              *w4 = b3 + 32, *b4 = w4 + 32;
  float h1[32], h2[64];
#pragma unroll
  for (int o = 0; o < 32; o++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < NIN; k++) acc = fmaf(w1[o * NIN + k], x[k], acc);
    h1[o] = relu(acc + b1[o]);
  }
#pragma unroll
  for (int o2 = 0; o2 < 64; o2++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; k++) acc = fmaf(w2[o2 * 32 + k], h1[k], acc);
    h2[o2] = relu(acc + b2[o2]);
  }
  float y = 0.0f;
#pragma unroll
  for (int o = 0; o < 32; o++) {
    float acc = 0.0f;
#pragma unroll
    for (int k = 0; k < 64; k++) acc = fmaf(w3[o * 64 + k], h2[k], acc);
    y = fmaf(w4[o], relu(acc + b3[o]), y);
  }
  return y + b4[0];
}

// MVN(loc, diag(0.5)) in float32, the arithmetic torch performs
// (multivariate_normal.py rsample/log_prob; pinned in tests/test_rollout_math.py):
//   sample a = loc + L*eps;  x = (a - loc) * (1/L);  logp = -0.5*(log(2 pi) + x*x) - log(L)
constexpr float MVN_L = 0x1.6a09e6p-1f;        // cholesky([[0.5]]) in float32
// PPO clipped surrogate f = -min(r A, clamp(r, .8, 1.2) A) and df/dr, with torch's tie
// rule (minimum splits the gradient evenly on ties; clamp passes it on [0.8, 1.2]
// inclusive) — Coop-MH-PPO-scalable.py:803-806, :838-841
MHPPO_HD inline double surr_and_grad(double r, double A, double &dfdr) {
  double rc = r < 0.8 ? 0.8 : (r > 1.2 ? 1.2 : r);
  double s1 = r * A, s2 = rc * A;
  double in = (r >= 0.8 && r <= 1.2) ? 1.0 : 0.0;
  double g;
  if (s1 < s2)
    g = A;
  else if (s2 < s1)
    g = in * A;
  else
    g = 0.5 * A + 0.5 * in * A;
  dfdr = -g;
  return -(s1 < s2 ? s1 : s2);
}
// The same with the ratio's magnitude in float32 and its clip branch decided in float64 (the
// split-precision train kernel's continuous actor).  r = expf(lp - lp_old) carries ~2 float32
// roundings; which branch the reference's float64 ratio takes depends only on
// d = lp - lp_old in float64 (exact: a difference of two floats), against ln 0.8 / ln 1.2:
//   A > 0: -min(rA, clamp(r)A) follows r up to r = 1.2 (dfdr = -A), then is constant;
//   A < 0: it follows r from r = 0.8 on, and is constant below.
// (At r in [0.8, 1.2] the two terms tie and torch's minimum splits the gradient evenly between
// them, 0.5 A + 0.5 A.)  d is a multiple of 2^-24 for log-densities below -0.5, whose grid points lie
// >= 8e-9 from ln 0.8 and ln 1.2, far outside a float64 rounding of them: the decision is the float64 ratio's
// (tests/test_update_scale_gpu.py counts the rows a float32 decision would flip).
constexpr double LN_0_8 = -0x1.c8ff7c79a9a20p-3, LN_1_2 = 0x1.7565011e49675p-3;  // float64 log(0.8), log(1.2)
MHPPO_HD inline float surr_and_grad_fd(float r, double d, float A, float &dfdr) {
  const bool lo = d < LN_0_8, hi = d > LN_1_2;  // r < 0.8, r > 1.2 in float64
  const float rc = lo ? 0.8f : (hi ? 1.2f : r);
  const bool follow = A > 0.0f ? !hi : (A < 0.0f && !lo);
  dfdr = follow ? -A : 0.0f;
  const float s1 = r * A, s2 = rc * A;
  return -(s1 < s2 ? s1 : s2);
}

constexpr float MVN_INV_L = 0x1.6a09e6p+0f;    // float32(1/L) as torch's triangular solve uses
constexpr float MVN_LOG2PI = 0x1.d67f1cp+0f;   // float32(1 * math.log(2*math.pi))
constexpr float MVN_HALF_LOGDET = -0x1.62e432p-2f;  // float32 log(L)

MHPPO_HD inline float mvn_logp(float a, float loc) {
  float x = (a - loc) * MVN_INV_L;
  float m = x * x;
  return (-0.5f * (MVN_LOG2PI + m)) - MVN_HALF_LOGDET;
}

// torch.minimum (NaN-propagating) in float32
MHPPO_HD inline float t_minimum(float a, float b) {
  if (a != a) return a;
  if (b != b) return b;
  return (b < a) ? b : a;
}

// Philox-4x32-10 (perf-mode noise)
MHPPO_HD inline void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; r++) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0, hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

}  // namespace mhppo
