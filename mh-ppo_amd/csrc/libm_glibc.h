// libm_glibc.h — the float transcendentals of the rollout's policy heads, returning exactly
// what this image's glibc (2.35, x86-64) returns, on the GPU and on the host.
//
// Why: the C oracle (oracle/rollout_oracle.c) restates the rollout's policy heads
// (Env_rollout.iterations_rand, Coop-MH-PPO-scalable.py:430-453; Model_PPO :87-89) with glibc
// tanhf/expf, and the full-scale discrete parity tests compare the device with that oracle:
// the action feeds env.step, so a one-ulp difference moves a car by an ulp and can, downstream,
// flip a gap-acceptance decision or the Categorical draw u >= p0 / (p0 + p1).  These
// restatements make the device return glibc's bits, so device and oracle agree bit for bit.
// They do NOT make the device equal to torch's CPU forward: in this container (torch 2.10,
// AVX512 capability) ATen evaluates even a one-element tanh/exp in its vectorised (Sleef)
// kernel, which differs from glibc in the last bit on ~20 % of inputs, and torch's Linear sums
// in MKL's order, not the fmaf chain's.  Against the reference's own batch-1 forward the policy
// outputs therefore agree to float32 rounding (tests/test_policy_torch_gpu.py: probabilities
// within 1e-5 relative, actions within 1e-5, every Categorical draw identical on 4 096 rows).
//   mhppo_tanhf  — sysdeps/ieee754/flt-32/s_tanhf.c (fdlibm): |x| >= 1: 1 - 2 / (expm1f(2|x|) + 2),
//                  else -t / (t + 2) with t = expm1f(-2|x|); |x| >= 22: +-1; |x| < 2^-55: x (1 + x)
//   mhppo_expm1f — sysdeps/ieee754/flt-32/s_expm1f.c (fdlibm): reduction x = k ln2 + r (ln2 split
//                  hi/lo), rational approximation of degree 5 in hxs = r^2 / 2, reconstruction by k
//   mhppo_expf   — sysdeps/ieee754/flt-32/e_expf.c (ARM optimized-routines), as the x86-64 IFUNC
//                  selects it on an FMA + AVX2 host (e_expf-fma.c: GCC contracts every multiply
//                  whose uses are all additions into an fma): 2^(k/32) from a 32-entry table
//                  times a cubic in r, in double precision, rounded once to float.
// Every operation is written out in the order (and with the fma / no-fma choice) the glibc
// object code uses; the translation units that include this are built with -ffp-contract=off.
// Pinned exhaustively — all 2^32 float inputs — against the host's glibc by
// tests/test_libm_glibc.py (tools/libm_check.cpp).
// Sources and licences of the restated algorithms (third-party, not the reference):
//   s_expm1f.c, s_tanhf.c — glibc sysdeps/ieee754/flt-32, from FreeBSD/fdlibm:
//     "Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//      Developed at SunPro, a Sun Microsystems, Inc. business.
//      Permission to use, copy, modify, and distribute this software is freely granted,
//      provided that this notice is preserved."
//     (float versions by Ian Lance Taylor, Cygnus Support.)
//   e_expf.c + e_exp2f_data.c (__exp2f_data, the 32-entry 2^(k/32) table below) — glibc
//     sysdeps/ieee754/flt-32, from ARM optimized-routines:
//     "Copyright (c) 2017-2018 Arm Ltd.  SPDX-License-Identifier: MIT OR Apache-2.0 WITH
//      LLVM-exception" (glibc carries it under the LGPL-2.1-or-later).
// The code below is a restatement of those algorithms, operation for operation.
#pragma once
#include <stdint.h>

#ifndef MHPPO_LIBM_HD
#ifdef __HIP__
#define MHPPO_LIBM_HD __host__ __device__ __attribute__((always_inline)) inline
#else
#define MHPPO_LIBM_HD __attribute__((always_inline)) inline
#endif
#endif

namespace mhppo {
namespace glibc {
MHPPO_LIBM_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
MHPPO_LIBM_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
MHPPO_LIBM_HD uint64_t d2u(double x) { return __builtin_bit_cast(uint64_t, x); }
MHPPO_LIBM_HD double u2d(uint64_t u) { return __builtin_bit_cast(double, u); }
MHPPO_LIBM_HD double fma_d(double a, double b, double c) { return __builtin_fma(a, b, c); }
}  // namespace glibc

// expm1f (fdlibm s_expm1f.c).  Non-finite and overflow handling kept for completeness.
MHPPO_LIBM_HD float mhppo_expm1f(float x) {
  using namespace glibc;
  const float one = 1.0f, huge = 1.0e+30f, tiny = 1.0e-30f;
  const float o_threshold = u2f(0x42b17180u), ln2_hi = u2f(0x3f317180u), ln2_lo = u2f(0x3717f7d1u),
              invln2 = u2f(0x3fb8aa3bu);
  const float Q1 = u2f(0xbd088889u), Q2 = u2f(0x3ad00d01u), Q3 = u2f(0xb8a670cdu), Q4 = u2f(0x36867e54u),
              Q5 = u2f(0xb457edbbu);
  float y, hi, lo, c = 0.0f, t, e, hxs, hfx, r1;
  int32_t k;
  uint32_t hx = f2u(x);
  const uint32_t xsb = hx & 0x80000000u;
  y = xsb == 0 ? x : -x;
  (void)y;
  hx &= 0x7fffffffu;
  if (hx >= 0x4195b844u) {    // |x| >= 27 ln2
    if (hx >= 0x42b17218u) {  // |x| >= 88.721...
      if (hx > 0x7f800000u) return x + x;                // NaN
      if (hx == 0x7f800000u) return xsb == 0 ? x : -1.0f;  // exp(+-inf) - 1
      if (x > o_threshold) return huge * huge;           // overflow
    }
    if (xsb != 0) return tiny - one;  // x < -27 ln2: -1 (inexact)
  }
  if (hx > 0x3eb17218u) {    // |x| > 0.5 ln2
    if (hx < 0x3F851592u) {  // and |x| < 1.5 ln2
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      } else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    } else {
      const float kf = invln2 * x + (xsb == 0 ? 0.5f : -0.5f);
      k = (int32_t)kf;
      t = (float)k;
      hi = x - t * ln2_hi;  // t * ln2_hi is exact here
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  } else if (hx < 0x33000000u) {  // |x| < 2^-25: x
    t = huge + x;
    return x - (t - (huge + x));
  } else {
    k = 0;
  }
  // x is now in the primary range
  hfx = 0.5f * x;
  hxs = x * hfx;
  r1 = one + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
  t = 3.0f - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0f - x * t));
  if (k == 0) return x - (x * e - hxs);
  e = (x * (e - c) - c);
  e -= hxs;
  if (k == -1) return 0.5f * (x - e) - 0.5f;
  if (k == 1) {
    if (x < -0.25f) return -2.0f * (e - (x + 0.5f));
    return one + 2.0f * (x - e);
  }
  if (k <= -2 || k > 56) {  // exp(x) - 1 suffices
    y = one - (e - x);
    if (k == 128) {
      y = y * 2.0f * u2f(0x7f000000u);  // 0x1p127f
    } else {
      y = u2f(f2u(y) + ((uint32_t)k << 23));  // add k to y's exponent
    }
    return y - one;
  }
  if (k < 23) {
    t = u2f(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
    y = t - (e - x);
    y = u2f(f2u(y) + ((uint32_t)k << 23));
  } else {
    t = u2f((uint32_t)(0x7f - k) << 23);  // 2^-k
    y = x - (e + t);
    y += one;
    y = u2f(f2u(y) + ((uint32_t)k << 23));
  }
  return y;
}

// tanhf (fdlibm s_tanhf.c)
MHPPO_LIBM_HD float mhppo_tanhf(float x) {
  using namespace glibc;
  const float one = 1.0f, two = 2.0f, tiny = 1.0e-30f;
  const int32_t jx = (int32_t)f2u(x);
  const uint32_t ix = (uint32_t)jx & 0x7fffffffu;
  if (ix >= 0x7f800000u) {  // inf or NaN
    if (jx >= 0) return one / x + one;
    return one / x - one;
  }
  float z;
  if (ix < 0x41b00000u) {  // |x| < 22
    if (ix == 0) return x;
    if (ix < 0x24000000u) return x * (one + x);  // |x| < 2^-55
    const float ax = u2f(ix);
    if (ix >= 0x3f800000u) {  // |x| >= 1
      const float t = mhppo_expm1f(two * ax);
      z = one - two / (t + two);
    } else {
      const float t = mhppo_expm1f(-two * ax);
      z = -t / (t + two);
    }
  } else {
    z = one - tiny;  // |x| >= 22: +-1
  }
  return jx >= 0 ? z : -z;
}

// expf (e_expf.c, EXP2F_TABLE_BITS 5, as compiled into e_expf-fma.c)
MHPPO_LIBM_HD float mhppo_expf(float x) {
  using namespace glibc;
  // T[i] = asuint64(2^(i/32)) - (i << 52) / 32 (__exp2f_data.tab)
  constexpr uint64_t T[32] = {
      0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
      0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
      0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
      0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
      0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
      0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
      0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
      0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};
  const double InvLn2N = 0x1.71547652b82fep+0 * 32, SHIFT = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-5 / 32 / 32 / 32, C1 = 0x1.ebfce50fac4f3p-3 / 32 / 32,
               C2 = 0x1.62e42ff0c52d6p-1 / 32;
  const uint32_t abstop = (f2u(x) >> 20) & 0x7ff;
  if (abstop >= ((f2u(88.0f) >> 20) & 0x7ff)) {  // |x| >= 88 or NaN
    if (f2u(x) == 0xff800000u) return 0.0f;        // -inf
    if (abstop >= ((0x7f800000u >> 20) & 0x7ff)) return x + x;
    if (x > 0x1.62e42ep6f) return u2f(0x7f800000u);  // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;             // underflow
  }
  const double xd = (double)x;
  // z = InvLn2N * xd has only additive uses (z + SHIFT, z - kd): both fused
  double kd = fma_d(InvLn2N, xd, SHIFT);
  const uint64_t ki = d2u(kd);
  kd -= SHIFT;
  const double r = fma_d(InvLn2N, xd, -kd);
  uint64_t t = T[ki % 32];
  t += ki << (52 - 5);
  const double s = u2d(t);
  const double z = fma_d(C0, r, C1);
  const double r2 = r * r;
  double y = fma_d(C2, r, 1.0);
  y = fma_d(z, r2, y);
  y = y * s;
  return (float)y;
}
}  // namespace mhppo
