// env_dev.h — device-side crosswalk env for gfx950: one env per lane.
//
// State lives in HBM as structure-of-arrays blocked by 64 envs ([N/64][field][slot][64],
// sidx), so every per-lane access of a wave is one coalesced 512-B transaction and a
// wave's whole state is one contiguous block.  Each env draws from its own CPython-compatible
// MT19937 stream (two blocks [N][2][624] u32 + cursor), so trajectories are the
// reference's on `random.seed(seed_base + env_id)` and invariant to how envs
// are sharded over GPUs.
//
// Semantics follow the reference statement by statement (file:line under
// /root/reference/Environments, coop file unless noted):
//   pedestrian.__init__ :15-103, choix_pedestrian :138-173 (naif :129-174,
//   4cars no shuffle), detection :175-259 (scalable :176-264, naif :176-215),
//   ped.step :292-401 (+ scalable mid-cross stop :371-380), CG_score :403-412,
//   get_data/is_in_front/is_crossing_in_front/new_reward_wait_safety/
//   delta_l* :433-511, car :515-622, IDM follow_action scalable :604-624,
//   car_follower 4cars :13-129, env.step :745-832, env.reset :838-893.
// Python's two-argument min/max keep the FIRST argument unless the second is
// strictly smaller/greater; pymin/pymax reproduce that (NaN included).
// Built with -ffp-contract=off: no FMA contraction, Python's rounding order.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

// Every env routine is __host__ __device__: the kernels run it on gfx950 and
// tools/hostsim.cpp runs the identical source on the CPU for debugging.
// Always inlined: an env view passed by reference to an outlined call would have to
// live in memory (scratch), defeating the register view below.
#define MHPPO_HD __host__ __device__ __attribute__((always_inline))
// full unroll of slot/pedestrian loops: compile-time trip counts in the register view
#define MHPPO_UNROLL _Pragma("unroll")

namespace mhppo {

// Phase timing, A/B builds only (tools/ab_build.sh <name> -DMHPPO_TIMING): lane 0 of every
// wave adds the shader-clock cycles since its previous mark to its phase-k slot (mark 0
// starts the clock); MHPPO_MARK_FLUSH adds the wave's slots 1-13 to g_timing[k], the largest
// wave total to g_timing[14] (max) and counts the wave in g_timing[15]; tools/env_phases.py / train_phases.py read them.  Loads are
// asynchronous, so a phase is charged with the wait for the data it first consumes.
#if defined(MHPPO_TIMING) && defined(__HIP_DEVICE_COMPILE__)
static __device__ unsigned long long g_timing[32];  // [16 + k]: the slowest wave's phase k
// per-wave accumulators in LDS (one global atomic per phase and wave, at MHPPO_MARK_FLUSH)
__device__ __forceinline__ unsigned long long *timing_slots() {
  // [wave][phase 1..14 at 1..14, last stamp at 15]: 2 KB, within the train kernel's LDS slack
  __shared__ unsigned long long t_acc[16][16];
  return &t_acc[threadIdx.x >> 6][0];
}
// MHPPO_MARK_MASK (A/B timing builds): only the marks whose bit is set stamp (mark 0 always), so a
// block can be timed between two stamps with the rest of the kernel unperturbed by the others
#ifndef MHPPO_MARK_MASK
#define MHPPO_MARK_MASK 0xffff
#endif
__device__ __forceinline__ void timing_mark(int k) {
  if (k > 0 && !((MHPPO_MARK_MASK >> k) & 1)) return;
  unsigned long long *a = timing_slots();
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long now = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  if ((threadIdx.x & 63) == 0) {
    if (k > 0) {
      a[k] += now - a[15];
    } else {
      for (int q = 0; q < 15; q++) a[q] = 0;
    }
    a[15] = now;
  }
}
__device__ __forceinline__ void timing_flush() {
  unsigned long long *a = timing_slots();
  if ((threadIdx.x & 63) == 0) {
    unsigned long long tot = 0;
    for (int q = 1; q < 14; q++) {
      if (a[q]) {
        atomicAdd(&g_timing[q], a[q]);
        atomicMax(&g_timing[16 + q], a[q]);
      }
      tot += a[q];
    }
    atomicMax(&g_timing[14], tot);  // the slowest wave's phases 1-13 (a launch lasts as long as it)
    atomicAdd(&g_timing[15], 1ull);
  }
}
#define MHPPO_MARK(k) ::mhppo::timing_mark(k)
#define MHPPO_MARK_FLUSH() ::mhppo::timing_flush()
#elif defined(MHPPO_TIMING) && defined(__HIP__)
static __device__ unsigned long long g_timing[32];
#define MHPPO_MARK(k)
#define MHPPO_MARK_FLUSH()
#else
#define MHPPO_MARK(k)
#define MHPPO_MARK_FLUSH()
#endif

enum { V_COOP = 0, V_4CARS = 1, V_SCALABLE = 2, V_NAIF = 3, V_4CARS2 = 4, V_STOP = 5 };
// 4cars / 4cars2: nb_car AVs, each followed by an IDM car (4cars2: PPO-driven follower)
constexpr bool has_followers(int v) { return v == V_4CARS || v == V_4CARS2; }

// car fields (double) [C_NF][nC] per env (env-blocked, see sidx).  The reference's two-step
// acceleration history (car.step's discount_array = [1, 0, 0], :550, :643-645) enters the
// acceleration only as 0 * h, i.e. only through whether h is finite: it is kept
// as one non-finite bit per car and history step (envi EI_H0NF / EI_H1NF, bit s = car slot s).
enum { C_AC, C_VC, C_SC, C_LIGHT, C_PA, C_ES, C_TS, C_LINE, C_EXIST, C_NF };
// ped fields (double) [P_NF][P] per env
enum { P_SX, P_SY, P_VX, P_VY, P_T0, P_WT, P_CT, P_WDL, P_DELTA, P_LPOS, P_IVX, P_IVY, P_RATIO,
       P_CSTOP, P_A, P_B, P_W, P_NF };
// ped flag word bits [P] per env (u32)
enum : uint32_t {
  F_DECISION = 1u << 0, F_ATCROSS = 1u << 1, F_LEFT = 1u << 2, F_INCROSS = 1u << 3,
  F_ACCIDENT = 1u << 4, F_STOP = 1u << 5, F_WSA = 1u << 6, F_NEEDSTOP = 1u << 7,
  F_EXIST = 1u << 8, F_ISCROSS = 1u << 9, F_FOLLOW = 1u << 10, F_DIRNEG = 1u << 11,
  F_DIRPOS = 1u << 12, F_GENDER = 1u << 13, F_SIN = 1u << 14,
  F_PNW = 1u << 15,  // ped_not_waiting (:35, :224-226): only gates the "Pedestrian is not waiting" print
  F_AGE_SHIFT = 16, F_AGE_MASK = 3u << 16,
  F_TSTOP_SHIFT = 20, F_TSTOP_MASK = 0xFFu << 20,
};
// env scalars
enum { E_CROSS, E_TIME, E_ND };
enum { EI_PEDTRAF, EI_CARTRAF, EI_MTI, EI_MTB, EI_H0NF, EI_H1NF, EI_NI };
// Per-env event counters: the reference's only run-time diagnostics are prints inside
// pedestrian.detection (scalable :186, :200, :222, :227, :236; 4cars :293-334); each print
// here increments this env's counter, cleared by reset.  Order = include/mhppo.h MHPPO_EV_*.
enum { EV_ACCIDENT, EV_POSSIBLE, EV_SMALL, EV_NOTWAIT, EV_GREEN, EV_N };
constexpr int MAX_CAR_SLOTS = 32;  // the history bit words (AV slots + 4cars followers)

// +1 on an env's event counter (one lane per env: no contention).  A plain read-modify-write: the
// no-return-atomic form (-DMHPPO_ATOMIC_EVENTS) takes the counter load off the detection phase
// but the atomics' completion then holds the step's final stores, 2 % slower end to end (r04,
// profiles/r04_env_steps/).
MHPPO_HD inline void ev_inc(uint32_t *p) {
#if defined(__HIP_DEVICE_COMPILE__) && defined(MHPPO_ATOMIC_EVENTS)
  (void)__hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p += 1u;
#endif
}

struct Cfg {
  // nS: action slots (acc + light each); nAV: AV slots with rewards/detection (= nS except
  // 4cars2, whose followers take actions but earn none); nC: all car slots (+ followers)
  int variant, N, nb_car, nb_ped, nb_lines, nS, nC, P, max_episode, sin_model, obs_dim, nAV;
  double dt, dt2, b00, b10, pb[2][4], xb0, xb1, idm_den, ep_len;
  // car.__init__ position bounds (:549-560): low/high_car_range, mean_speed_ped (host-computed)
  double car_low, car_high, mean_speed_ped;
  // host-computed constants of the step: car.time_braking at speed_limit (:564), and the braking
  // distance's divisor -2 b00 (:508-514) — when it is a power of two (b00 = -4: 8) its exact
  // reciprocal, so v^2 / (-2 b00) is one multiply with the same bits instead of a float64 division
  double tb, brake_inv;
  uint64_t seed_base, env_off;
  int flags, brake_p2;  // MHPPO_FIX_* (include/mhppo.h); brake_inv is exact
};

struct Bufs {
  double *car;    // [N/EB][C_NF][nC][EB]  (env-blocked: index with sidx)
  double *ped;    // [N/EB][P_NF][P][EB]
  uint32_t *pfl;  // [N/EB][P][EB]
  double *envd;   // [N/EB][E_ND][EB]
  int32_t *envi;  // [N/EB][EI_NI][EB]
  uint32_t *mt;   // [N][2][624] (active + next block, see RngT)
  uint32_t *ev;   // [N/EB][EV_N][EB] event counters (touched only when an event fires)
  // [N][2][nC] bytes: every car slot's line and existence, the static car fields (the step never
  // writes them; reset and choix_test do, through Env::set_line / set_exist, which keep car's
  // C_LINE / C_EXIST doubles and these bytes equal).  The register view reads only the bytes:
  // 2 nC bytes per env and step instead of 16 nC (one 16-B load per lane at nC = 8)
  uint8_t *carb;
};
MHPPO_HD __forceinline__ size_t carb_idx(int nC, int f, int s, int e) { return ((size_t)e * 2 + f) * nC + s; }

// Env-blocked state layout: every field array ([rows] per env: car C_NF*nC, ped P_NF*P,
// flags P, envd E_ND, envi EI_NI) is stored [ceil(N/EB)][rows][EB], so one wave's 64 envs
// own one contiguous block (a few KB) instead of rows 8*N bytes apart: the same 512-B
// coalesced access per field, but a wave's state load touches one DRAM/TLB region.
constexpr int EB = 64;
MHPPO_HD __forceinline__ size_t sidx(int rows, int row, int e) {
  return ((size_t)(e >> 6) * (size_t)rows + (size_t)row) * EB + (size_t)(e & (EB - 1));
}
MHPPO_HD __forceinline__ size_t npad(int N) { return ((size_t)N + EB - 1) / EB * EB; }

MHPPO_HD __forceinline__ double pymin(double a, double b) { return (b < a) ? b : a; }
MHPPO_HD __forceinline__ double pymax(double a, double b) { return (b > a) ? b : a; }

// x**2 and x**4 (CPython float_pow -> glibc pow, <= 0.52 ulp, i.e. the correctly rounded
// power but for rare near-midpoint cases).  The device computes the correctly rounded square
// and a double-double fourth power (one rounding) instead of ocml's general pow (~130
// instructions through an extended-precision log/exp); the host build (tools/hostsim.cpp)
// keeps glibc's pow, so the simulator stays bit-identical to the oracle.
MHPPO_HD __forceinline__ double pow_2(double x) {
#ifdef __HIP_DEVICE_COMPILE__
  return x * x;
#else
  return pow(x, 2.0);
#endif
}
MHPPO_HD __forceinline__ double pow_4(double x) {
#ifdef __HIP_DEVICE_COMPILE__
  const double x2 = x * x, r = x2 * x2;
  if (!(fabs(r) < 0x1p1000) || fabs(x2) < 0x1p-400) return r;  // inf/NaN/overflow, tiny: plain
  const double e = fma(x, x, -x2);                                // x^2 == x2 + e exactly
  return fma(x2, x2, 2.0 * x2 * e);  // x2^2 + 2 x2 e (+ e^2 < 2^-106 x^4), rounded once
#else
  return pow(x, 4.0);
#endif
}

static constexpr double PI = 0x1.921fb54442d18p+1;
static constexpr double NV_MAGICCONST = 0x1.b72cd3f331398p+0;  // 4*exp(-0.5)/sqrt(2.0)

// ------------------------------------------------------------ CPython random
// Each env owns a RING of four 624-word MT19937 blocks, [N][4][624]: the active block (the
// CPython state, consumed at cursor mti) and, ahead of it in ring order, the next three
// blocks = successive twists of it, kept ready ahead of time.  Exhausting the active block
// just moves to the next one; the old block is marked stale.  The episode's reset kernel
// regenerates every stale block (mt_refill_wave: coalesced loads, three LDS phases, coalesced
// stores, in ring order), so an episode can draw 3 x 624 words beyond its active block — the
// draw-heavy envs (a pedestrian waiting in front of several cars re-draws its normalvariate
// gap acceptance every step, up to ~20 words a step) stay within it — and the 624-step twist
// never sits on one lane's critical path during the rollout; RngT twists in-lane only if an
// env exhausts the whole ring in one episode.
// envi[EI_MTB]: bits 0-1 = active block, bit 2 + k = block k is stale.
enum : int { MT_N = 624, MT_BLOCKS = 4, MT_PAD = 64 };  // MT_PAD: words after the last env's blocks
MHPPO_HD inline int mt_active(int mtb) { return mtb & 3; }
MHPPO_HD inline bool mt_stale(int mtb, int k) { return (mtb >> (2 + k)) & 1; }

MHPPO_HD inline uint32_t mt_mix(uint32_t a, uint32_t b) {  // one twist term of (a, successor b)
  uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// dst = twist(src), out of place (CPython genrand_uint32's in-place loop restated:
// terms 0..226 read src only, 227..622 the new words 227 behind, 623 new[396] and new[0])
__host__ __device__ __attribute__((noinline)) inline void mt_twist_into(const uint32_t *src, uint32_t *dst) {
  for (int kk = 0; kk < 227; kk++) dst[kk] = src[kk + 397] ^ mt_mix(src[kk], src[kk + 1]);
  for (int kk = 227; kk < 623; kk++) dst[kk] = dst[kk - 227] ^ mt_mix(src[kk], src[kk + 1]);
  dst[623] = dst[396] ^ mt_mix(src[623], dst[0]);
}

#ifndef MHPPO_RNG_MULTI
#define MHPPO_RNG_MULTI 1  // RngT::genrand_n's one-shift window path (A/B builds override)
#endif
// K > 0: the next K words of the active block are read ahead in one batch (independent
// loads) and consumed in order; an empty window is refilled with one batch, so a run
// of draws costs one HBM round trip per K words.
template <int K>
struct RngT {
  uint32_t *base;  // this env's two blocks
  uint32_t *mt;    // the active block
  int mti, mtb;
  uint32_t win[K > 0 ? K : 1];  // win[0 .. nwin) == mt[mti .. mti + nwin)
  int nwin = 0;

  MHPPO_HD void attach(uint32_t *env_blocks, int mti_, int mtb_) {
    base = env_blocks;
    mti = mti_;
    mtb = mtb_;
    mt = base + mt_active(mtb) * MT_N;
  }
  MHPPO_HD void prefetch() {
    if (K == 0) return;
    nwin = (MT_N - mti) < K ? (MT_N - mti) : K;
#pragma unroll
    // unconditional loads (one batch, no branches): words past the active block read the
    // next block or the allocation's tail padding (MT_PAD) and are never consumed
    for (int k = 0; k < (K > 0 ? K : 1); k++) win[k] = mt[mti + k];
  }
  MHPPO_HD uint32_t genrand() {
    if (mti >= MT_N) {
      const int a = mt_active(mtb), n = (a + 1) & 3;
      uint32_t *next = base + n * MT_N;
      if (mt_stale(mtb, n)) mt_twist_into(mt, next);  // ring exhausted within one episode
      mtb = n | (((mtb >> 2) | (1 << a)) & ~(1 << n)) << 2;  // switch; the old block is now stale
      mt = next;
      mti = 0;
      nwin = 0;
    }
    uint32_t y;
    if (K > 0) {
      if (nwin == 0) prefetch();
      y = win[0];
#pragma unroll
      for (int k = 0; k + 1 < (K > 0 ? K : 1); k++) win[k] = win[k + 1];
      nwin--;
    } else {
      y = mt[mti];
    }
    mti++;
    return temper(y);
  }
  MHPPO_HD static uint32_t temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // the next n words (= n genrand() calls): with a window, one shift of it by n (n genrand()s shift
  // it n times by one, ~K moves each); a run that crosses the active block's end takes genrand()
  template <int n>
  MHPPO_HD void genrand_n(uint32_t (&y)[n]) {
    if (!MHPPO_RNG_MULTI || K < n || mti + n > MT_N) {
#pragma unroll
      for (int k = 0; k < n; k++) y[k] = genrand();
      return;
    }
    if (nwin < n) prefetch();  // then nwin = min(MT_N - mti, K) >= n
#pragma unroll
    for (int k = 0; k < n; k++) y[k] = temper(win[k]);
#pragma unroll
    for (int k = 0; k + n < (K > 0 ? K : 1); k++) win[k] = win[k + n];
    nwin -= n;
    mti += n;
  }
  MHPPO_HD static double random53(uint32_t a, uint32_t b) {  // CPython random() of two words
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
  }
  MHPPO_HD double random() {
    uint32_t w[2];
    genrand_n<2>(w);
    return random53(w[0], w[1]);
  }
  MHPPO_HD uint32_t randbelow(uint32_t n) {
    if (!n) return 0;
    int k = 0;
    for (uint32_t t = n; t; t >>= 1) k++;
    uint32_t v = genrand() >> (32 - k);
    while (v >= n) v = genrand() >> (32 - k);
    return v;
  }
  MHPPO_HD int randint(int a, int b) { return a + (int)randbelow((uint32_t)(b - a + 1)); }
  MHPPO_HD double uniform(double a, double b) { return a + (b - a) * random(); }
  MHPPO_HD double normalvariate(double mu, double sigma) {
    double t, u2;
    for (;;) {
      uint32_t w[4];  // the round's two random() calls, in order
      genrand_n<4>(w);
      const double u1 = random53(w[0], w[1]);
      u2 = 1.0 - random53(w[2], w[3]);
      t = NV_MAGICCONST * (u1 - 0.5);  // CPython: z = t / u2, zz = z * z / 4, accept iff zz <= -log(u2)
      // Squeeze around that test (same decisions, same draws): with r = 1 - u2 (exact: the second
      // random()), r < -log(u2) < r / u2, and for r >= 2^-40 both gaps are >= r^2 / 2, i.e.
      // >= 2^-41 relative.  zz is t^2 / (4 u2^2) within a few ulps, so q = t^2 / 4 against r u2^2
      // and r u2 with a 2^-40 relative margin decides zz <= r (accept) and zz > r / u2 (reject)
      // without a division; only a draw inside a margin (or r < 2^-40) takes the exact test.
      const double r = 1.0 - u2;
      if (r >= 0x1p-40) {
        const double q = t * t * 0.25, ru = r * u2;
        if (q <= ru * u2 * (1.0 - 0x1p-40)) break;
        if (q > ru * (1.0 + 0x1p-40)) continue;
      }
      const double z = t / u2;
      if (z * z / 4.0 <= -log(u2)) break;
    }
    return mu + (t / u2) * sigma;
  }
};
using Rng = RngT<0>;

// init_by_array([seed lo, seed hi]) exactly as CPython's random.seed(int)
MHPPO_HD inline void rng_seed(uint32_t *mt, uint64_t seed) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  int klen = key[1] ? 2 : 1;
  mt[0] = 19650218u;
  for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
  int i = 1, j = 0;
  for (int k = 624; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
    i++; j++;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
    if (j >= klen) j = 0;
  }
  for (int k = 623; k; k--) {
    mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
    i++;
    if (i >= 624) { mt[0] = mt[623]; i = 1; }
  }
  mt[0] = 0x80000000u;
}

// fmod is exact (the remainder is always representable).  The device's ocml fmod reduces
// the exponent difference in a loop; with a small quotient (|x/y| < 2^52, the env's lane
// index) the remainder is one fma away: q = trunc(|x|/|y|) is the true quotient or one too
// large (the division rounds up onto an integer), and |x| - q|y| is then the exact
// remainder, which fma returns unrounded.  Same bits as fmod, NaN/inf/zero cases included.
MHPPO_HD __forceinline__ double fmod_exact(double x, double y) {
#ifdef __HIP_DEVICE_COMPILE__
  const double ax = fabs(x), ay = fabs(y);
  const double q = trunc(ax / ay);
  if (!(q < 0x1p52) || !(ay > 0.0) || !isfinite(ax) || !isfinite(ay)) return fmod(x, y);
  double r = fma(-q, ay, ax);
  if (r < 0.0) r = fma(-(q - 1.0), ay, ax);
  return copysign(r, x);
#else
  return fmod(x, y);
#endif
}

// CPython float floor division (Objects/floatobject.c _float_div_mod)
MHPPO_HD inline double py_floordiv(double vx, double wx) {
  double mod = fmod_exact(vx, wx);
  double div = (vx - mod) / wx;
  if (mod) {
    if ((wx < 0) != (mod < 0)) { mod += wx; div -= 1.0; }
  }
  double fl;
  if (div) {
    fl = floor(div);
    if (div - fl > 0.5) fl += 1.0;
  } else {
    fl = copysign(0.0, vx / wx);
  }
  return fl;
}

// ---------------------------------------------------------- small arrays
template <class T, int N>
struct PlainArr {
  T v[N];
  MHPPO_HD T &operator[](int i) { return v[i]; }
  MHPPO_HD const T &operator[](int i) const { return v[i]; }
};

// ---------------------------------------------------------------- env views
// Every env routine below is written against an "env view" EV: VAR (the variant),
// shape queries nC()/nAV()/nS()/nP(), MAXAV (capacity of per-AV scratch arrays),
// accessors car(f, s) / pedf(f, p) / pflag(p), the RNG stream, cross/cl, and
// commit() (end of a step).  Two views exist:
//
// Env<V>: generic shapes.  Car/ped fields are read and written in place in HBM
// (coalesced across the wave); used by reset, state dumps and every shape the
// register view is not instantiated for.
template <int V>
struct Env {
  static constexpr int VAR = V;
  static constexpr int MAXAV = 16;
  static constexpr int CNS = 0, CNP = 0;  // compile-time action slots / pedestrians: not known
  static constexpr int OBS_DIM = 0;       // compile-time observation width: not known
  using AvArr = PlainArr<double, MAXAV>;
  AvArr rw, rl;  // step outputs per AV: reward, reward_light
  const Cfg &c;
  const Bufs &b;
  int e;
  Rng rng;
  double cross, cl;  // crosswalk lane width, cross_lines = nb_lines * cross

  MHPPO_HD Env(const Cfg &c_, const Bufs &b_, int e_) : c(c_), b(b_), e(e_) {
    rng.attach(b.mt + (size_t)e * (MT_BLOCKS * MT_N), b.envi[sidx(EI_NI, EI_MTI, e)], b.envi[sidx(EI_NI, EI_MTB, e)]);
    cross = b.envd[sidx(E_ND, E_CROSS, e)];
    cl = (double)c.nb_lines * cross;
  }
  MHPPO_HD void save_rng() {
    b.envi[sidx(EI_NI, EI_MTI, e)] = rng.mti;
    b.envi[sidx(EI_NI, EI_MTB, e)] = rng.mtb;
  }
  MHPPO_HD void commit_cars() {}  // in place: nothing staged
  MHPPO_HD void commit_peds() {}
  MHPPO_HD void commit_det() {}
  MHPPO_HD void commit() { save_rng(); }
  MHPPO_HD int nC() const { return c.nC; }
  MHPPO_HD int nAV() const { return c.nAV; }
  MHPPO_HD int nS() const { return c.nS; }
  MHPPO_HD int nP() const { return c.P; }
  MHPPO_HD int ped_traffic() const { return b.envi[sidx(EI_NI, EI_PEDTRAF, e)]; }
  MHPPO_HD int car_traffic() const { return b.envi[sidx(EI_NI, EI_CARTRAF, e)]; }
  MHPPO_HD int32_t &hist_nf(int k) const { return b.envi[sidx(EI_NI, EI_H0NF + k, e)]; }

  MHPPO_HD double &car(int f, int s) const { return b.car[sidx(C_NF * c.nC, f * c.nC + s, e)]; }
  // the static car fields: read here from the doubles, written to the doubles and the byte mirror
  MHPPO_HD double line(int s) const { return car(C_LINE, s); }
  MHPPO_HD double exists(int s) const { return car(C_EXIST, s); }
  MHPPO_HD void set_line(int s, double v) const {
    car(C_LINE, s) = v;
    b.carb[carb_idx(c.nC, 0, s, e)] = (uint8_t)v;
  }
  MHPPO_HD void set_exist(int s, double v) const {
    car(C_EXIST, s) = v;
    b.carb[carb_idx(c.nC, 1, s, e)] = (uint8_t)v;
  }
  MHPPO_HD double &pedf(int f, int p) const { return b.ped[sidx(P_NF * c.P, f * c.P + p, e)]; }
  MHPPO_HD uint32_t &pflag(int p) const { return b.pfl[sidx(c.P, p, e)]; }
  MHPPO_HD void event(int k) const { ev_inc(&b.ev[sidx(EV_N, k, e)]); }
};

#ifdef __HIP__
// One observation row per lane, obs [N][OD] f32: the wave's 64 rows are one contiguous
// 256*OD-byte block, but row-per-lane stores put each instruction's 64 lanes 4*OD bytes
// apart (64 partial cache lines per instruction, OD instructions).  The register view
// builds its row straight into this wave's LDS image of the block ([64][OD], the block's
// exact memory image; obs_lds_row), and store_obs_wave writes the block out as
// lane-contiguous 16-B stores: OD/4 fully coalesced instructions.  Every lane of a full
// wave must call it (convergent); a partial wave (or a misaligned caller buffer) copies its
// rows out one per lane.  Workgroups of 4 waves (TPB = 256 in every register-view kernel).
template <int OD>
__device__ __forceinline__ float *obs_lds_wave() {
  __shared__ float sh_obs[4][64 * OD];
  return sh_obs[(threadIdx.x >> 6) & 3];
}
template <int OD>
__device__ __forceinline__ float *obs_lds_row() { return obs_lds_wave<OD>() + (threadIdx.x & 63) * OD; }
template <int OD>
__device__ __forceinline__ void store_obs_wave(float *obs, int e, int N) {
  const int lane = threadIdx.x & 63;
  const int e0 = e - lane;
  const float *s = obs_lds_wave<OD>();
  float *wbase = obs + (size_t)e0 * OD;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (e0 + 64 > N || ((uintptr_t)wbase & 15) != 0) {
#pragma unroll
    for (int k = 0; k < OD; k++) obs[(size_t)e * OD + k] = s[lane * OD + k];
    return;
  }
  constexpr int NCH = 16 * OD;  // 16-B chunks of the wave's block: OD/4 per lane (+ a tail)
  const float4 *src = reinterpret_cast<const float4 *>(s) + lane;
  float4 *dst = reinterpret_cast<float4 *>(wbase) + lane;
  // all reads first, into distinct registers, then the stores (no store waits on the
  // previous one's data registers)
  float4 v[NCH / 64];
#pragma unroll
  for (int j = 0; j < NCH / 64; j++) v[j] = src[64 * j];
#pragma unroll
  for (int j = 0; j < NCH / 64; j++) dst[64 * j] = v[j];
  if constexpr (NCH % 64 != 0) {
    if (lane < NCH % 64) dst[64 * (NCH / 64)] = src[64 * (NCH / 64)];
  }
}
#endif

// EnvR<V, NC, NAV, NP>: compile-time shape (NC car slots, NAV AVs, NP pedestrians).
// The whole env state is loaded into registers in one batch of independent loads at
// construction (plus a 16-word RNG window), the step runs on registers with fully
// unrolled slot/ped loops (every index a compile-time constant after unrolling and
// inlining, so the arrays below live in VGPRs/AGPRs, never in scratch), and commit()
// writes the dynamic fields back.  With one env
// per lane and 65 536 envs the GPU holds one wave per SIMD, so the in-place HBM view
// serialises ~100 dependent memory round trips per step; this view needs ~3.
#ifndef MHPPO_RNG_WIN
#define MHPPO_RNG_WIN 16  // words of the register view's RNG window (A/B builds override)
#endif
static_assert(MHPPO_RNG_WIN <= MT_PAD, "the window's unconsumed tail stays inside the allocation");
template <int V, int NC, int NAV, int NP>
struct EnvR {
  static constexpr int VAR = V;
  static constexpr int MAXAV = NAV;
  static constexpr int CNS = V == V_4CARS2 ? 2 * NAV : NAV, CNP = NP;
  static constexpr int OBS_DIM = (V == V_SCALABLE ? 7 * NC + 4 : 6 * NC + 3) + 9 * NP;
  using AvArr = PlainArr<double, NAV>;
  AvArr rw, rl;  // step outputs per AV: reward, reward_light
  const Cfg &c;
  const Bufs &b;
  int e;
  RngT<MHPPO_RNG_WIN> rng;
  double cross, cl;
  mutable double car_[C_LINE][NC];  // the dynamic car fields (C_LINE and C_EXIST come from carb)
  static constexpr int NCB = (2 * NC + 3) / 4;
  double st_[2][NC];  // line, exist of every slot, decoded once from carb's 2 NC bytes
  mutable double ped_[P_NF][NP];
  mutable uint32_t pfl_[NP];
  mutable int32_t hnf_[2];
  int ptraf, ctraf;

  MHPPO_HD EnvR(const Cfg &c_, const Bufs &b_, int e_) : c(c_), b(b_), e(e_) {
    const size_t N = (size_t)c.N;
    rng.attach(b.mt + (size_t)e * (MT_BLOCKS * MT_N), b.envi[sidx(EI_NI, EI_MTI, e)], b.envi[sidx(EI_NI, EI_MTB, e)]);
    cross = b.envd[sidx(E_ND, E_CROSS, e)];
    cl = (double)c.nb_lines * cross;
    ptraf = b.envi[sidx(EI_NI, EI_PEDTRAF, e)];
    ctraf = b.envi[sidx(EI_NI, EI_CARTRAF, e)];
    hnf_[0] = b.envi[sidx(EI_NI, EI_H0NF, e)];
    hnf_[1] = b.envi[sidx(EI_NI, EI_H1NF, e)];
#pragma unroll
    for (int f = 0; f < C_LINE; f++)
#pragma unroll
      for (int s = 0; s < NC; s++) car_[f][s] = b.car[sidx(C_NF * NC, f * NC + s, e)];
    uint32_t cb[NCB];  // packed: line of slot s = byte s, exist = byte NC + s
    if constexpr ((2 * NC) % 4 == 0) {  // whole dwords (one 16-B load at NC = 8)
      const uint32_t *cw = reinterpret_cast<const uint32_t *>(b.carb + carb_idx(NC, 0, 0, e));
#pragma unroll
      for (int k = 0; k < NCB; k++) cb[k] = cw[k];
    } else {
#pragma unroll
      for (int k = 0; k < NCB; k++) cb[k] = 0u;
#pragma unroll
      for (int k = 0; k < 2 * NC; k++) cb[k / 4] |= (uint32_t)b.carb[carb_idx(NC, 0, k, e)] << (8 * (k % 4));
    }
#pragma unroll
    for (int k = 0; k < 2 * NC; k++) st_[k / NC][k % NC] = (double)((cb[k / 4] >> (8 * (k % 4))) & 0xffu);
#pragma unroll
    for (int f = 0; f < P_NF; f++)
#pragma unroll
      for (int p = 0; p < NP; p++) ped_[f][p] = b.ped[sidx(P_NF * NP, f * NP + p, e)];
#pragma unroll
    for (int p = 0; p < NP; p++) pfl_[p] = b.pfl[sidx(NP, p, e)];
    // the RNG window is fetched at the start of the step (env_step_body): its address
    // depends on the cursor loaded here, and the car steps cover the round trip
  }
  // Dynamic fields only (line/exist and the pedestrian's static draws never change in a
  // step), each group stored as soon as env_step_body is done with it, so the stores drain
  // while the rest of the step computes instead of in one burst at the end: the cars'
  // kinematics and history bits after the car steps (commit_cars), the pedestrians'
  // kinematics and the RNG cursor after the pedestrian step (commit_peds; no later phase
  // draws), the detection fields after detection (commit_det), the rest in commit().
  MHPPO_HD void commit_cars() {
    constexpr int dyn_car[4] = {C_AC, C_VC, C_SC, C_LIGHT};
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int s = 0; s < NC; s++) b.car[sidx(C_NF * NC, dyn_car[k] * NC + s, e)] = car_[dyn_car[k]][s];
    b.envi[sidx(EI_NI, EI_H0NF, e)] = hnf_[0];
    b.envi[sidx(EI_NI, EI_H1NF, e)] = hnf_[1];
  }
  MHPPO_HD void commit_peds() {
    constexpr int kin_ped[8] = {P_SX, P_SY, P_VX, P_VY, P_T0, P_WT, P_CT, P_LPOS};
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int p = 0; p < NP; p++) b.ped[sidx(P_NF * NP, kin_ped[k] * NP + p, e)] = ped_[kin_ped[k]][p];
    b.envi[sidx(EI_NI, EI_MTI, e)] = rng.mti;
    b.envi[sidx(EI_NI, EI_MTB, e)] = rng.mtb;
  }
  MHPPO_HD void commit_det() {
    constexpr int det_car[3] = {C_PA, C_ES, C_TS};
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
      for (int s = 0; s < NAV; s++) b.car[sidx(C_NF * NC, det_car[k] * NC + s, e)] = car_[det_car[k]][s];
  }
  MHPPO_HD void commit() {  // after rewards (P_WDL) and the observation (P_DELTA, flags)
#pragma unroll
    for (int p = 0; p < NP; p++) {
      b.ped[sidx(P_NF * NP, P_WDL * NP + p, e)] = ped_[P_WDL][p];
      b.ped[sidx(P_NF * NP, P_DELTA * NP + p, e)] = ped_[P_DELTA][p];
      b.pfl[sidx(NP, p, e)] = pfl_[p];
    }
  }
  // env_observe builds this env's observation row in obs_stage() (device: the wave's LDS
  // image) and store_obs_row writes it to obs [N][OBS_DIM]
#ifdef __HIP_DEVICE_COMPILE__
  MHPPO_HD float *obs_stage() const { return obs_lds_row<OBS_DIM>(); }
  MHPPO_HD void store_obs_row(float *obs) const { store_obs_wave<OBS_DIM>(obs, e, c.N); }
#else
  mutable float obs_h[OBS_DIM];
  float *obs_stage() const { return obs_h; }
  void store_obs_row(float *obs) const {
    for (int k = 0; k < OBS_DIM; k++) obs[(size_t)e * OBS_DIM + k] = obs_h[k];
  }
#endif
  static constexpr int nC() { return NC; }
  static constexpr int nAV() { return NAV; }
  static constexpr int nS() { return V == V_4CARS2 ? 2 * NAV : NAV; }
  static constexpr int nP() { return NP; }
  MHPPO_HD int ped_traffic() const { return ptraf; }
  MHPPO_HD int car_traffic() const { return ctraf; }

  MHPPO_HD double &car(int f, int s) const { return car_[f][s]; }
  MHPPO_HD double line(int s) const { return st_[0][s]; }
  MHPPO_HD double exists(int s) const { return st_[1][s]; }
  MHPPO_HD int32_t &hist_nf(int k) const { return hnf_[k]; }
  MHPPO_HD double &pedf(int f, int p) const { return ped_[f][p]; }
  MHPPO_HD uint32_t &pflag(int p) const { return pfl_[p]; }
  // a lane increments its env's counter in HBM only when one fires (no-return atomic)
  MHPPO_HD void event(int k) const { ev_inc(&b.ev[sidx(EV_N, k, e)]); }
};

struct Ped {
  double Sx, Sy, Vx, Vy, t0, wt, ct, wdl, delta, lpos, ivx, ivy, ratio, cstop, A, B, W;
  uint32_t fl;
  int dir, tstop;
  MHPPO_HD bool has(uint32_t f) const { return (fl & f) != 0; }
  MHPPO_HD void set(uint32_t f, bool v) { fl = v ? (fl | f) : (fl & ~f); }
};

template <class EV>
MHPPO_HD inline Ped load_ped(const EV &E, int p) {
  constexpr int V = EV::VAR;
  Ped q;
  q.Sx = E.pedf(P_SX, p); q.Sy = E.pedf(P_SY, p); q.Vx = E.pedf(P_VX, p); q.Vy = E.pedf(P_VY, p);
  q.t0 = E.pedf(P_T0, p); q.wt = E.pedf(P_WT, p); q.ct = E.pedf(P_CT, p); q.wdl = E.pedf(P_WDL, p);
  q.delta = E.pedf(P_DELTA, p); q.lpos = E.pedf(P_LPOS, p); q.ivx = E.pedf(P_IVX, p);
  q.ivy = E.pedf(P_IVY, p); q.ratio = E.pedf(P_RATIO, p); q.cstop = E.pedf(P_CSTOP, p);
  q.A = E.pedf(P_A, p); q.B = E.pedf(P_B, p); q.W = E.pedf(P_W, p);
  q.fl = E.pflag(p);
  q.dir = (q.fl & F_DIRNEG) ? -1 : ((q.fl & F_DIRPOS) ? 1 : 0);
  q.tstop = (int)((q.fl & F_TSTOP_MASK) >> F_TSTOP_SHIFT);
  return q;
}

template <class EV>
MHPPO_HD inline void store_ped(const EV &E, int p, Ped &q, bool dyn_only) {
  constexpr int V = EV::VAR;
  E.pedf(P_SX, p) = q.Sx; E.pedf(P_SY, p) = q.Sy; E.pedf(P_VX, p) = q.Vx; E.pedf(P_VY, p) = q.Vy;
  E.pedf(P_T0, p) = q.t0; E.pedf(P_WT, p) = q.wt; E.pedf(P_CT, p) = q.ct; E.pedf(P_WDL, p) = q.wdl;
  E.pedf(P_DELTA, p) = q.delta; E.pedf(P_LPOS, p) = q.lpos;
  if (!dyn_only) {
    E.pedf(P_IVX, p) = q.ivx; E.pedf(P_IVY, p) = q.ivy; E.pedf(P_RATIO, p) = q.ratio;
    E.pedf(P_CSTOP, p) = q.cstop; E.pedf(P_A, p) = q.A; E.pedf(P_B, p) = q.B; E.pedf(P_W, p) = q.W;
  }
  uint32_t fl = q.fl & ~(F_TSTOP_MASK | F_DIRNEG | F_DIRPOS);
  fl |= ((uint32_t)q.tstop << F_TSTOP_SHIFT) & F_TSTOP_MASK;
  if (q.dir < 0) fl |= F_DIRNEG;
  if (q.dir > 0) fl |= F_DIRPOS;
  E.pflag(p) = fl;
}

// ------------------------------------------------------- pedestrian geometry
template <class EV>
MHPPO_HD inline bool is_in_front(const EV &E, const Ped &q, double car_line, double next_line) {
  constexpr int V = EV::VAR;
  double line_1 = (-E.cl / 2) + E.cross * (car_line - 0.5 * next_line + 1);
  double line_2 = (E.cl / 2) - E.cross * ((double)E.c.nb_lines - 0.5 * next_line - car_line);
  if (q.dir == -1) return q.Sy >= line_2 - 0.001;
  return q.Sy <= line_1 + 0.001;
}

template <class EV>
MHPPO_HD inline bool is_crossing_in_front(const EV &E, const Ped &q, double car_line, double prev_line) {
  constexpr int V = EV::VAR;
  double line_1 = (-E.cl / 2) + E.cross * (car_line - prev_line);
  double line_2 = (E.cl / 2) - E.cross * ((double)E.c.nb_lines - car_line - 1 - prev_line);
  if (q.dir == -1) return q.Sy < line_2;
  return q.Sy > line_1;
}

// which car slots the pedestrians see: mode 0 = reset observation (all AV slots),
// mode 1 = step (existing AVs [+ followers for 4cars])
template <class EV>
MHPPO_HD inline bool in_view(const EV &E, int s, int mode) {
  constexpr int V = EV::VAR;
  if (has_followers(V)) return mode == 1 || s < E.nAV();
  if (V == V_SCALABLE) return mode == 0 || E.exists(s) != 0.0;
  return true;
}

template <class EV>
MHPPO_HD inline double CG_score(EV &E, const Ped &q, double crossing_size) {
  constexpr int V = EV::VAR;
  if (!q.has(F_ISCROSS)) return 0.;
  const double fem = 0.0369, child = -0.0355, midage = -0.0221, old = -0.1810;
  const double alpha = 0.09, sigma = 0.09;
  int age = (int)((q.fl & F_AGE_MASK) >> F_AGE_SHIFT);
  double gamma = log10(crossing_size / fabs(q.ivy + 10e-3));
  double log_val = alpha + gamma + fem * (double)(q.has(F_GENDER)) + child * (double)(age == 0) +
                   midage * (double)(age == 1) + old * (double)(age == 2);
  log_val = log_val + E.rng.normalvariate(0.0, sigma);
#ifdef __HIP_DEVICE_COMPILE__
  // 10^x: ocml exp10 (~66 instructions) instead of the general pow (~238): the value only ever
  // meets `car_time + light < CG`, where a last-bit difference (both are ~1 ulp from glibc's
  // pow(10, x), which the oracle calls) flips the decision only on an exact tie; the full-scale
  // parity tests still see 0 diverging envs
  return exp10(log_val);
#else
  return pow(10.0, log_val);
#endif
}

template <class EV>
MHPPO_HD inline bool choix_pedestrian(EV &E, const Ped &q, int mode) {
  constexpr int V = EV::VAR;
  const double car_size = 4;
  int n = 0;
  MHPPO_UNROLL
  for (int s = 0; s < E.nC(); s++) n += in_view(E, s, mode);
  if (q.has(F_FOLLOW)) {
    if (V == V_NAIF) {
      // random.shuffle(cars): real permutation, nibble-packed (n <= 16)
      uint64_t perm = 0;
      for (int i = 0; i < n; i++) perm |= (uint64_t)i << (4 * i);
      if (n > 1) {
        for (int i = n - 1; i >= 1; i--) {
          int j = (int)E.rng.randbelow((uint32_t)(i + 1));
          uint64_t xi = (perm >> (4 * i)) & 15u, xj = (perm >> (4 * j)) & 15u;
          perm &= ~((15ull << (4 * i)) | (15ull << (4 * j)));
          perm |= (xj << (4 * i)) | (xi << (4 * j));
        }
      }
      // naif: view == all slots, in order
      for (int k = 0; k < n; k++) {
        int i = (int)((perm >> (4 * k)) & 15u);
        double pos = E.car(C_SC, i), line = E.line(i);
        if (is_crossing_in_front(E, q, line, 0.5) && is_in_front(E, q, line, 1.0) &&
            (pos < car_size + q.Sx) && (pos > q.Sx))
          return false;
      }
      for (int k = 0; k < n; k++) {
        int i = (int)((perm >> (4 * k)) & 15u);
        if (E.car(C_SC, i) < q.Sx && E.car(C_LIGHT, i) < 0) return false;
      }
    } else {
      if (!has_followers(V) && n > 1)
        for (int i = n - 1; i >= 1; i--) (void)E.rng.randbelow((uint32_t)(i + 1));
      MHPPO_UNROLL
      for (int s = 0; s < E.nC(); s++) {
        if (!in_view(E, s, mode)) continue;
        double pos = E.car(C_SC, s), line = E.line(s);
        if (is_crossing_in_front(E, q, line, 0.5) && is_in_front(E, q, line, 1.0)) {
          if ((pos < car_size + q.Sx) && (pos > q.Sx)) return false;
        }
      }
      MHPPO_UNROLL
      for (int s = 0; s < E.nC(); s++) {
        if (!in_view(E, s, mode)) continue;
        double light = E.car(C_LIGHT, s);
        if (E.car(C_SC, s) < q.Sx && light != 0) return light > 0.;
      }
    }
  }
  // Gap acceptance (:162-172): over the in-view cars in slot order, a car in front within
  // car_size ahead refuses; a car behind the pedestrian draws a CG_score and refuses if its
  // time gap is shorter; otherwise the next car.  Restated as a loop over the CG draws with a
  // single CG_score site: each round selects the first slot >= from that blocks or draws.
  // (Unrolled over slots, a wave would run one inlined CG_score per slot any lane reaches.)
  int from = 0;
  for (;;) {
    int hit = -1;
    double pos = 0, spd = 0, line = 0, light = 0;
    MHPPO_UNROLL
    for (int s = E.nC() - 1; s >= 0; s--) {  // descending: the lowest qualifying slot wins
      if (s < from || !in_view(E, s, mode)) continue;
      const double ln = E.line(s), ps = E.car(C_SC, s);
      if (!is_in_front(E, q, ln, 1.0)) continue;
      if (((ps < car_size + q.Sx) && (ps > q.Sx)) || (ps < q.Sx)) {
        hit = s;
        pos = ps;
        spd = E.car(C_VC, s);
        line = ln;
        light = E.car(C_LIGHT, s);
      }
    }
    if (hit < 0) return true;
    if (pos > q.Sx) return false;  // blocking car (pos < car_size + Sx held)
    double car_time = fabs((pos - q.Sx) / (spd + 10e-3));
    double CG = CG_score(E, q, fabs(q.lpos - line) * E.cross);
    if (car_time + light < CG) return false;
    from = hit + 1;
  }
}

template <class EV>
MHPPO_HD inline double brake_dist(const EV &E, double spd) {  // spd^2 / (-2 b00), correctly rounded
  const double v2 = spd * spd;
  return E.c.brake_p2 ? v2 * E.c.brake_inv : v2 / (-2.0 * E.c.b00);
}

template <class EV>
MHPPO_HD inline double worst_delta_l(const EV &E, const Ped &q, double pos, double spd, double line) {
  constexpr int V = EV::VAR;
  if (pos > q.Sx || q.has(F_LEFT) || !is_in_front(E, q, line, 0)) return V == V_SCALABLE ? 100.0 : 0.0;
  return fabs(pos - q.Sx) - brake_dist(E, spd);
}

template <class EV>
MHPPO_HD inline double delta_l(const EV &E, const Ped &q, double pos, double spd, double line) {
  constexpr int V = EV::VAR;
  if (pos > q.Sx || q.has(F_LEFT) || !is_in_front(E, q, line, 0)) return 0.0;
  return fabs(pos - q.Sx) - brake_dist(E, spd) - 1.0 * (spd);
}

template <class EV>
MHPPO_HD inline double delta_l_all(const EV &E, const Ped &q, int mode) {
  constexpr int V = EV::VAR;
  double dl = V == V_SCALABLE ? 100.0 : 0.0;
  MHPPO_UNROLL
  for (int s = 0; s < E.nC(); s++) {
    if (!in_view(E, s, mode)) continue;
    double pos = E.car(C_SC, s), spd = E.car(C_VC, s);
    if ((pos <= q.Sx) && is_in_front(E, q, E.line(s), 0) && (!q.has(F_LEFT)) && (E.car(C_LIGHT, s) >= 0)) {
      double nd = fabs(pos - q.Sx) - brake_dist(E, spd) - 1.0 * (spd);
      dl = pymin(dl, nd);
    }
  }
  return dl;
}

// pedestrian.get_data (:433-444); updates the running-min `delta`
template <class EV>
MHPPO_HD inline void ped_get_data(const EV &E, Ped &q, int mode, double out[9]) {
  constexpr int V = EV::VAR;
  if (!q.has(F_EXIST)) {
    for (int k = 0; k < 9; k++) out[k] = 0.;
    return;
  }
  q.delta = pymin(delta_l_all(E, q, mode) * (double)q.has(F_ISCROSS) * (double)(!q.has(F_LEFT)), q.delta);
  out[0] = q.Vx; out[1] = q.Vy; out[2] = q.Sx; out[3] = q.Sy; out[4] = q.delta;
  out[5] = q.has(F_LEFT); out[6] = q.has(F_INCROSS); out[7] = 1.0; out[8] = (double)q.dir;
}

template <class EV>
MHPPO_HD inline double new_reward_wait_safety(const EV &E, Ped &q, double spd, double pos, double line) {
  constexpr int V = EV::VAR;
  if ((!q.has(F_LEFT)) && q.has(F_ISCROSS) && (pos < q.Sx) && is_in_front(E, q, line, 0)) {
    double exp_dl;
    if (spd < (V == V_STOP ? 0.01 : 0.05)) {  // stop :478
      exp_dl = 0.;
    } else {
      double dl = delta_l(E, q, pos, spd, line) / (spd);
      if (dl >= -1.) exp_dl = pymax(-20. * exp(-4. * (dl)-4.), -20.0);
      else exp_dl = 20. * dl;
    }
    exp_dl = exp_dl - (double)(q.has(F_ACCIDENT) ? 20 : 0);
    if (exp_dl < q.wdl) q.wdl = exp_dl;
  }
  return q.wdl + 0.0;
}

// --------------------------------------------------------- pedestrian.step
template <class EV>
MHPPO_HD inline void function_step(const EV &E, const Ped &q, double time, double &pos, double &spd) {
  constexpr int V = EV::VAR;
  if (q.has(F_SIN)) {
    double t = time + E.c.dt;
    double sn, cs;
#ifdef __HIP_DEVICE_COMPILE__
    sincos(q.W * (t - q.t0), &sn, &cs);  // one range reduction: ocml sin/cos/sincos share it (same bits)
#else
    sn = sin(q.W * (t - q.t0));
    cs = cos(q.W * (t - q.t0));
#endif
    const double z = q.W * 0.0;
    const double c0 = z == 0.0 ? 1.0 : cos(z);  // cos(+-0) == 1 exactly; NaN/inf W still go through cos
    double speed_p = (q.A * sn + q.B);
    double pos_p = ((-E.cl / 2.) + (q.A * (-cs + c0) / q.W));
    if (!(pos_p >= 0.0 && speed_p < fabs(q.ivy))) {
      pos = (double)q.dir * pos_p;
      spd = (double)q.dir * speed_p;
      return;
    }
  }
  pos = q.Sy + q.ivy * E.c.dt;
  spd = q.ivy;
}

template <class EV>
MHPPO_HD inline void ped_step(EV &E, Ped &q, double time) {
  constexpr int V = EV::VAR;
  const double dt = E.c.dt, cl = E.cl;
  double pp_y = q.Sy + q.ivy * dt;
  {  // boolean_ped_position (:261-274)
    double ds = (double)q.dir * q.Sy;
    if (ds >= cl / 2) { q.set(F_INCROSS, false); q.set(F_LEFT, true); }
    else if (ds > -cl / 2) { q.set(F_INCROSS, true); q.set(F_LEFT, false); }
    else { q.set(F_INCROSS, false); q.set(F_LEFT, false); }
  }
  if (!q.has(F_ISCROSS)) return;
  bool choose = true;
  if (!q.has(F_DECISION) && q.has(F_ATCROSS)) {
    choose = choix_pedestrian(E, q, 1);
    if (choose) {
      q.lpos = (double)((E.c.nb_lines - 1) * (q.dir < 0));
      q.set(F_ATCROSS, false);
    }
    q.set(F_DECISION, true);
    q.t0 = time;
  }
  const double dir = (double)q.dir;
  if ((q.Sy * dir < -cl / 2.) && (pp_y * dir > -cl / 2.) && !q.has(F_DECISION)) {
    double pos_p_x = (q.Vx * dt) * (fabs(-cl / 2. - q.Sy * dir) / fabs(q.Vy * dt + 10e-3));
    q.Vx = pos_p_x / dt;
    q.Sx = q.Sx + pos_p_x;
    q.Vy = dir * fabs(-q.Sy * dir - (cl / 2.)) / dt;
    q.Sy = -dir * cl / 2.;
    q.tstop = 0;
    q.set(F_ATCROSS, true);
  } else if ((fabs(q.Sy) <= cl / 2) || q.has(F_DECISION)) {
    if (q.tstop != 0) {
      q.Vx = 0.0;
      q.Vy = 0.0;
      q.tstop = q.tstop - 1;
      q.t0 = q.t0 + dt;
    } else if ((E.rng.uniform(0, 1) < 0.98) && choose) {
      q.set(F_DECISION, false);
      double new_spy, new_vpy;
      function_step(E, q, time, new_spy, new_vpy);
      bool change_line = false;
      // new_spy's lane (:278, and apply_change_line :287 on the same value): one floordiv
      const bool spy_in = fabs(new_spy) < cl / 2;
      const double new_line = spy_in ? py_floordiv(new_spy + cl / 2, E.cross) : 0.0;
      if (spy_in) {  // will_change_line (:276-281)
        if (new_line != q.lpos && fabs(q.Sy) < cl / 2) change_line = true;
      }
      double dtc = ((double)E.c.nb_lines - q.lpos - 1) * E.cross * (double)(q.dir > 0);
      dtc += (q.lpos) * E.cross * (double)(q.dir < 0);
      bool new_choice;
      if (change_line && (dtc > 0. && dtc < cl)) {
        new_choice = choix_pedestrian(E, q, 1);
        if (new_choice && q.has(F_STOP)) q.set(F_STOP, false);
      } else {
        new_choice = false;
      }
      if (q.has(F_STOP)) {
        q.Vx = 0.0;
        q.Vy = 0.0;
        q.t0 = q.t0 + dt;
        if (change_line) q.wt = q.wt + dt;
      } else if ((V == V_SCALABLE || V == V_4CARS2 || V == V_STOP) && q.has(F_NEEDSTOP) && q.Sy < q.cstop &&
                 pp_y > q.cstop) {  // mid-crossing stop (scalable :371-381, 4cars2 :448, stop :366)
        q.tstop = V == V_STOP ? E.rng.randint(2, 15) : E.rng.randint(5, 35);
        q.set(F_NEEDSTOP, false);
        if (!choose) {
          q.set(F_DECISION, false);
          q.tstop = 0;
          q.wt = q.wt + dt;
        }
        q.Vx = 0.0;
        q.Vy = 0.0;
        q.t0 = q.t0 + dt;
      } else if ((!change_line) || (change_line && new_choice)) {
        q.Sy = new_spy;
        q.Vy = new_vpy;
        double nsx = q.Sx + q.Vy * q.ratio * dt, nvx = q.Vy * q.ratio;
        q.Sx = nsx;
        q.Vx = nvx;
        q.ct = q.ct + dt;
        if (change_line && new_choice) {  // apply_change_line (:283-289)
          if (!spy_in) {
            q.lpos = (double)(E.c.nb_lines * (q.dir < 0) - 1 * (q.dir > 0));
          } else {
            if (new_line != q.lpos) q.lpos = new_line;
          }
        }
      } else {  // change_line && !new_choice
        q.set(F_STOP, true);
        double distance = fabs(dir * (cl - dtc) - dir * cl / 2. - q.Sy);
        double pos_p_x = (q.Vx) * (distance) / fabs(q.Vy + 10e-3);
        q.Vx = pos_p_x / dt;
        q.Sx = q.Sx + pos_p_x;
        q.Vy = dir * distance / dt;
        q.Sy = dir * ((cl - dtc) - cl / 2.);
      }
    } else {
      q.tstop = V == V_4CARS2 ? E.rng.randint(5, 35) : (V == V_STOP ? E.rng.randint(2, 15) : E.rng.randint(2, 5));
      if (!choose) {
        q.set(F_DECISION, false);
        q.tstop = 0;
        q.wt = q.wt + dt;
      }
      q.Vx = 0.0;
      q.Vy = 0.0;
      q.t0 = q.t0 + dt;
    }
  } else {
    double nsx = q.Sx + q.ivx * dt, nsy = q.Sy + q.ivy * dt;
    q.Sx = nsx;
    q.Vx = q.ivx;
    q.Sy = nsy;
    q.Vy = q.ivy;
  }
}

// ------------------------------------------------------- pedestrian.detection
// accumulates this ped's per-slot danger into acc[] (caller passes registers)
template <class EV, class AV>
MHPPO_HD inline void ped_detection(EV &E, Ped &q, const AV &prev, AV &acc, bool add) {
  constexpr int V = EV::VAR;
  const int nS = E.nAV();  // detection runs over the AVs (followers excluded, :845)
  // green lights of existing AVs behind the pedestrian (:229-233): the loop below never writes
  // light, position or existence, so the count is the same for every i
  double clw = 0;
  if (V != V_NAIF) {
    MHPPO_UNROLL
    for (int k = 0; k < nS; k++)
      if (E.car(C_LIGHT, k) > 0. && E.car(C_SC, k) < q.Sx && (V != V_SCALABLE || E.exists(k) != 0.0))
        clw += 1.0;
  }
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) {
    bool cond = is_in_front(E, q, E.line(i), 0);
    if (V == V_SCALABLE) cond = cond && (E.exists(i) != 0.0);
    if (!cond) continue;
    double Sc = E.car(C_SC, i), Vc = E.car(C_VC, i), line = E.line(i);
    int ped_accident;
    if (V == V_NAIF) {
      q.set(F_WSA, worst_delta_l(E, q, Sc, Vc, line) < 0);
      ped_accident = (!q.has(F_ACCIDENT)) && q.has(F_WSA);
    } else {
      ped_accident = (!q.has(F_ACCIDENT)) && q.has(F_WSA);
      q.set(F_WSA, worst_delta_l(E, q, Sc, Vc, line) < 0);
    }
    bool cif = is_crossing_in_front(E, q, line, 0);
    if (ped_accident && (cif && (prev[i] < q.Sx) && (Sc > q.Sx))) {
      q.set(F_ACCIDENT, true);
      E.event(EV_ACCIDENT);  // "Accident! : " (:186)
    }
    if (cif) {
      double dl;
      if ((Vc) < 0.05) dl = (V == V_SCALABLE) ? 100. : 0.;
      else dl = worst_delta_l(E, q, Sc, Vc, line) / (Vc);
      double pa;
      if (dl > 0) pa = -1. * exp(-4. * (dl));
      else pa = (V == V_NAIF || V == V_STOP) ? -1. * dl - 1 : 1. * dl - 1;
      if (pa < -1. && E.car(C_PA, i) >= -1.) E.event(EV_POSSIBLE);  // "Possible accident! " (:199-200)
      E.car(C_PA, i) = pymin(E.car(C_PA, i), pa);
    }
    double Ts = E.car(C_TS, i);
    const double tb = E.c.tb;  // car.time_braking (:564), Vc = speed_limit at init
    if (V == V_NAIF) {
      if (Sc < q.Sx) Ts = pymax(q.wt + 10. * q.ct - tb + 1., Ts);
    } else {
      if (Sc < q.Sx) Ts = pymax((1. + clw) * q.wt + 2. * q.ct - tb + 1., Ts);
    }
    E.car(C_TS, i) = Ts;
    double light = E.car(C_LIGHT, i);
    // red (:250-253) and green (:254-257) light are exclusive: one exp site serves both
    if (light < 0.0 || light > 0.0) {
      const bool red = light < 0.0;
      const bool ex = red ? (Ts < 0) : (q.Sx - Sc > 0);
      double ne;
      if (ex) ne = -1. * exp(red ? 4. * (Ts) : -4. * (q.Sx - Sc));
      else ne = red ? -1. * (1 + Ts) : -1. * (1 + Sc - q.Sx);
      // "Small mistake - priority ? " (:221-222) / "Mauvais signal vert " (:235-236)
      if (E.car(C_ES, i) >= -1. && ne < -1.) E.event(red ? EV_SMALL : EV_GREEN);
      // "Pedestrian is not waiting " (:224-227): once per pedestrian (naif: every time, :223-224)
      if (red && cif && Sc < q.Sx && (V == V_NAIF || !q.has(F_PNW))) {
        q.set(F_PNW, true);
        E.event(EV_NOTWAIT);
      }
      E.car(C_ES, i) = pymin(ne, E.car(C_ES, i));
    }
  }
  if (!add) return;
  double green = 0;
  MHPPO_UNROLL
  for (int k = 0; k < nS; k++)
    if (E.car(C_LIGHT, k) > 0. && (V != V_SCALABLE || E.exists(k) != 0.0)) green += 1.0;
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) {
    double res = E.car(C_PA, i) + E.car(C_ES, i);
    double term = 0.5 * green * (double)(E.car(C_LIGHT, i) < 0.) * (double)(E.car(C_TS, i) > 0);
    if (V == V_COOP || V == V_4CARS2 || V == V_STOP) res = res + term;
    else if (V == V_4CARS || V == V_SCALABLE) res = res - term;
    if (V == V_SCALABLE && E.exists(i) == 0.0) res = 0.;
    acc[i] += res;
  }
}

// ---------------------------------------------------------------- car.step
template <class EV>
MHPPO_HD inline double car_follow_action(const EV &E, int s, double lead_V, double lead_S) {
  constexpr int V = EV::VAR;
  double speed_car = E.car(C_VC, s);
  double diff_dist = lead_S - E.car(C_SC, s);
  double delta_v = speed_car - lead_V;
  double sm = 2. + (speed_car * 2.0) + (speed_car * delta_v) / E.c.idm_den;
  return E.c.b10 * (1 - pow_4(speed_car / 10.) - pow_2(sm / diff_dist));
}

template <class EV>
MHPPO_HD inline void car_step(const EV &E, int s, double action, double light) {
  constexpr int V = EV::VAR;
  const double dt = E.c.dt;
  double Vc = E.car(C_VC, s);
  double acc = pymin(pymax(action, E.c.b00), E.c.b10);
  double sg;
  if (Vc == 0.) sg = pymax(0., acc / fabs(acc));
  else if (acc > 0) sg = 1;
  else sg = pymax(pymin(-Vc / (dt * acc), 1.), 0.);
  if (V == V_STOP && sg > 0.) acc = pymax(acc, -Vc / (dt * sg));  // stop :603-605
  // fa = 0 + 1*acc + 0*h0 + 0*h1 (:643-645): 0.0 + acc is never -0, so a finite h adds an
  // exact (signed) zero and changes nothing; a non-finite one makes fa NaN
  const uint32_t bit = 1u << s;
  const uint32_t h0nf = (uint32_t)E.hist_nf(0), h1nf = (uint32_t)E.hist_nf(1);
  double fa = 0.0;
  fa = fa + 1.0 * acc;
  if ((h0nf | h1nf) & bit) fa = __builtin_nan("");
  E.hist_nf(1) = (int32_t)((h1nf & ~bit) | (h0nf & bit));              // h1 <- h0
  E.hist_nf(0) = (int32_t)((h0nf & ~bit) | (isfinite(acc) ? 0u : bit));  // h0 <- acc
  fa = fa * sg;
  double speed = Vc + dt * fa;
  double pos = (fa * E.c.dt2 / 2.0) + (Vc * dt) + (E.car(C_SC, s));
  E.car(C_AC, s) = fa;
  E.car(C_VC, s) = speed;
  E.car(C_SC, s) = pos;
  E.car(C_LIGHT, s) = light;
}

MHPPO_HD inline double car_reward(double Vc) { return -10. * pow_2(Vc - 10.0) / 100.0; }


#ifdef __HIP__  // HIP translation units (host and device passes), not the host-only simulator
// Wave-cooperative regeneration of stale MT blocks (see RngT): for every lane of this
// wave with a stale block, the 64 lanes load its active block (coalesced) and, in ring order,
// twist each stale block from its predecessor in three dependency phases through LDS (the
// stale blocks are always a suffix of the ring order after the active one: a block goes
// stale only when the cursor leaves it), storing each.  Call at kernel start from every lane
// of the wave (valid = this lane owns an env).
template <int WAVES>
__device__ __forceinline__ void mt_refill_wave(const Bufs &b, int N, int e, bool valid) {
  __shared__ uint32_t sh_a[WAVES][MT_N], sh_b[WAVES][MT_N];
  constexpr int NQ = (MT_N + 63) / 64;  // words of one block per lane
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int mtb = valid ? b.envi[sidx(EI_NI, EI_MTB, e)] : 0;
  uint64_t stale = __ballot(valid && (mtb >> 2) != 0);
  if (!stale) return;
  // The stale envs of the wave one after another, the next one's source block loaded (into
  // registers) while the current one twists: its load latency overlaps the twist and the stores
  // instead of opening every env's refill.
  int ln = 0, el = 0, bl = 0, k = MT_BLOCKS;  // the current env's lane, id, ring state, first stale block
  uint32_t nxt[NQ];
  auto take = [&](int &l, int &el_, int &bl_, int &k_) {  // pop the next stale lane; load its source block
    l = __ffsll((unsigned long long)stale) - 1;
    stale &= stale - 1;
    el_ = __shfl(e, l);
    bl_ = __shfl(mtb, l);
    const int a = mt_active(bl_);
    k_ = 1;
    while (k_ < MT_BLOCKS && !mt_stale(bl_, (a + k_) & 3)) k_++;  // first stale block in ring order
    if (k_ == MT_BLOCKS) return;
    const uint32_t *g_src = b.mt + (size_t)el_ * (MT_BLOCKS * MT_N) + ((a + k_ - 1) & 3) * MT_N;
#pragma unroll
    for (int i = 0; i < NQ; i++)
      if (lane + 64 * i < MT_N) nxt[i] = g_src[lane + 64 * i];
  };
  take(ln, el, bl, k);
  for (;;) {
    uint32_t *src = sh_a[w], *dst = sh_b[w];
    if (k < MT_BLOCKS) {
#pragma unroll
      for (int i = 0; i < NQ; i++)
        if (lane + 64 * i < MT_N) src[lane + 64 * i] = nxt[i];
    }
    const int l_c = ln, el_c = el, bl_c = bl, k_c = k;
    const bool more = stale != 0;
    if (more) take(ln, el, bl, k);  // the next env's block in flight during this one's twists
    if (k_c < MT_BLOCKS) {
      uint32_t *blk = b.mt + (size_t)el_c * (MT_BLOCKS * MT_N);
      const int a = mt_active(bl_c);
      for (int kk = k_c; kk < MT_BLOCKS; kk++) {
        uint32_t *g_dst = blk + ((a + kk) & 3) * MT_N;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q = lane; q < 227; q += 64) dst[q] = src[q + 397] ^ mt_mix(src[q], src[q + 1]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q = 227 + lane; q < 454; q += 64) dst[q] = dst[q - 227] ^ mt_mix(src[q], src[q + 1]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q = 454 + lane; q < 623; q += 64) dst[q] = dst[q - 227] ^ mt_mix(src[q], src[q + 1]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) dst[623] = dst[396] ^ mt_mix(src[623], dst[0]);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int q = lane; q < MT_N; q += 64) g_dst[q] = dst[q];
        uint32_t *t = src;  // the new block is the next twist's source
        src = dst;
        dst = t;
      }
      if (lane == l_c) b.envi[sidx(EI_NI, EI_MTB, el_c)] = a;  // active block kept, none stale
    }
    // every lane has read this env's last LDS image before the next env's block overwrites sh_a
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (!more) break;
  }
  // the owning lanes read their new blocks later in this launch: stores complete first
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
#endif

}  // namespace mhppo
