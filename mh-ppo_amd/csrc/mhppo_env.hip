// mhppo_env.hip — crosswalk env kernels (create/reset/step/state) + their C-ABI.
//
// One env per lane, 256-thread workgroups (4 waves), grid = ceil(N/256).
// The launch is variant-templated so each reference env class compiles to
// its own straight-line kernel with no variant branches.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mhppo.h"
#include "common.h"
#include "env_body.h"

using namespace mhppo;

namespace {
constexpr int TPB = 256;

// ------------------------------------------------------------- kernels
template <int V>
__global__ void __launch_bounds__(TPB) k_env_reset(Cfg c, Bufs b, float *obs) {
  int e = blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(b, c.N, e, e < c.N);
  if (e < c.N) env_reset_one<V>(c, b, e, obs);
}

__global__ void __launch_bounds__(TPB) k_env_choix(Cfg c, Bufs b, float *obs) {
  int e = blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(b, c.N, e, e < c.N);
  if (e < c.N) env_choix_test_one<V_SCALABLE>(c, b, e, obs);
}

template <int V>
__global__ void __launch_bounds__(TPB)
    k_env_step(Cfg c, Bufs b, const double *actions, float *obs, double *rew, double *rlight, uint8_t *done) {
  int e = blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(b, c.N, e, e < c.N);
  if (e < c.N)
    env_step_one<V>(c, b, e, actions + (size_t)e * 2 * c.nS, obs, rew ? rew + (size_t)e * c.nAV : nullptr,
                    rlight ? rlight + (size_t)e * c.nAV : nullptr, done);
}

template <int V, int NC, int NAV, int NP>
__global__ void __launch_bounds__(TPB)
    k_env_step_r(Cfg c, Bufs b, const double *actions, float *obs, double *rew, double *rlight, uint8_t *done) {
  int e = blockIdx.x * TPB + threadIdx.x;
  mt_refill_wave<TPB / 64>(b, c.N, e, e < c.N);
  if (e < c.N) {
    constexpr int NS = V == V_4CARS2 ? 2 * NAV : NAV;
    const double *ap = actions + (size_t)e * 2 * NS;
    PlainArr<double, 2 * NS> act;
#pragma unroll
    for (int k = 0; k < 2 * NS; k++) act.v[k] = ap[k];
    EnvR<V, NC, NAV, NP> E(c, b, e);
    env_step_body(E, act, obs, done);
#pragma unroll
    for (int i = 0; i < NAV; i++) {
      if (rew) rew[(size_t)e * NAV + i] = E.rw.v[i];
      if (rlight) rlight[(size_t)e * NAV + i] = E.rl.v[i];
    }
  }
}

__global__ void __launch_bounds__(TPB) k_env_seed(Cfg c, Bufs b) {
  int e = blockIdx.x * TPB + threadIdx.x;
  if (e < c.N) env_seed_one(c, b, e);
}

template <int V>
__global__ void __launch_bounds__(TPB) k_env_state(Cfg c, Bufs b, double *out, int dim) {
  int e = blockIdx.x * TPB + threadIdx.x;
  if (e < c.N) env_state_one<V>(c, b, e, out, dim);
}

__global__ void __launch_bounds__(TPB) k_env_events(Cfg c, Bufs b, uint32_t *out) {
  const int e = blockIdx.x * TPB + threadIdx.x;
  if (e < c.N)
#pragma unroll
    for (int k = 0; k < EV_N; k++) out[(size_t)e * EV_N + k] = b.ev[sidx(EV_N, k, e)];
}

__global__ void k_env_rng(Cfg c, Bufs b, uint32_t *mt, int32_t *mti) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  // the active block of each env (the CPython state) and its cursor
  if (i < (size_t)c.N * MT_N) {
    const size_t e = i / MT_N, k = i % MT_N;
    mt[i] = b.mt[e * (MT_BLOCKS * MT_N) + mt_active(b.envi[sidx(EI_NI, EI_MTB, e)]) * MT_N + k];
  }
  if (i < (size_t)c.N) mti[i] = b.envi[sidx(EI_NI, EI_MTI, i)];
}

}  // namespace

struct mhppo_env {
  Cfg c;
  Bufs b;
  int device;
  void *blob;
  size_t blob_bytes;
};

#define VARIANT_LAUNCH(kern, variant, grid, stream, ...)                                    \
  do {                                                                                      \
    switch (variant) {                                                                      \
      case V_COOP: hipLaunchKernelGGL(kern<V_COOP>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break;   \
      case V_4CARS: hipLaunchKernelGGL(kern<V_4CARS>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break; \
      case V_SCALABLE: hipLaunchKernelGGL(kern<V_SCALABLE>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break; \
      case V_NAIF: hipLaunchKernelGGL(kern<V_NAIF>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break;      \
      case V_4CARS2: hipLaunchKernelGGL(kern<V_4CARS2>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break;  \
      default: hipLaunchKernelGGL(kern<V_STOP>, grid, dim3(TPB), 0, stream, __VA_ARGS__); break;       \
    }                                                                                       \
  } while (0)

extern "C" {

int mhppo_env_create(const mhppo_env_cfg *cfg, int device, mhppo_env **out) {
  if (!cfg || !out) return set_error(MHPPO_EINVAL, "null argument");
  *out = nullptr;
  if (cfg->variant < 0 || cfg->variant > 5) return set_error(MHPPO_EINVAL, "unknown variant %d", cfg->variant);
  if (cfg->n_envs <= 0) return set_error(MHPPO_EINVAL, "n_envs must be > 0");
  if (cfg->nb_car < 1 || cfg->nb_ped < 1 || cfg->nb_lines < 1 || cfg->nb_ped > 8)
    return set_error(MHPPO_EINVAL, "bad nb_car/nb_ped/nb_lines");
  int nS = cfg->variant == V_SCALABLE ? 2 * cfg->nb_lines : (cfg->variant == V_4CARS2 ? 2 : 1) * cfg->nb_car;
  if (nS > MAXS) return set_error(MHPPO_EINVAL, "too many car slots (%d > %d)", nS, MAXS);
  static_assert(2 * MAXS <= MAX_CAR_SLOTS, "history bit words");
  if (cfg->variant == V_SCALABLE && cfg->nb_car > nS)
    return set_error(MHPPO_EINVAL, "scalable: nb_car must be <= 2*nb_lines (random.sample)");
  if (cfg->variant == V_NAIF && nS > 16) return set_error(MHPPO_EINVAL, "naif: at most 16 cars");
  if (!(cfg->car_b[0] < 0.0)) return set_error(MHPPO_EINVAL, "car_b[0][0] must be negative");
  GUARD_DEVICE(device);
  mhppo_env *h = new mhppo_env();
  build_cfg(*cfg, h->c);
  const Cfg &c = h->c;
  h->device = device;
  size_t N = npad(c.N);  // env-blocked arrays: whole blocks of EB envs
  size_t bytes_car = sizeof(double) * C_NF * c.nC * N, bytes_ped = sizeof(double) * P_NF * c.P * N;
  size_t bytes_pfl = sizeof(uint32_t) * c.P * N, bytes_envd = sizeof(double) * E_ND * N;
  size_t bytes_envi = sizeof(int32_t) * EI_NI * N, bytes_mt = sizeof(uint32_t) * (MT_BLOCKS * MT_N * (size_t)c.N + MT_PAD);
  size_t bytes_ev = sizeof(uint32_t) * EV_N * N, bytes_carb = (size_t)2 * c.nC * N;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t total = al(bytes_car) + al(bytes_ped) + al(bytes_pfl) + al(bytes_envd) + al(bytes_envi) + al(bytes_ev) +
                 al(bytes_carb) + al(bytes_mt);
  if (hipMalloc(&h->blob, total) != hipSuccess) {
    delete h;
    return set_error(MHPPO_ENOMEM, "hipMalloc(%zu) failed", total);
  }
  h->blob_bytes = total;
  char *p = (char *)h->blob;
  h->b.car = (double *)p; p += al(bytes_car);
  h->b.ped = (double *)p; p += al(bytes_ped);
  h->b.pfl = (uint32_t *)p; p += al(bytes_pfl);
  h->b.envd = (double *)p; p += al(bytes_envd);
  h->b.envi = (int32_t *)p; p += al(bytes_envi);
  h->b.ev = (uint32_t *)p; p += al(bytes_ev);
  h->b.carb = (uint8_t *)p; p += al(bytes_carb);
  h->b.mt = (uint32_t *)p;
  // any failure past the allocation releases the blob and the handle before reporting
  hipError_t e = hipMemset(h->blob, 0, total);
  if (e == hipSuccess) {
    dim3 grid((c.N + TPB - 1) / TPB);
    hipLaunchKernelGGL(k_env_seed, grid, dim3(TPB), 0, (hipStream_t)0, c, h->b);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    (void)hipFree(h->blob);
    delete h;
    return set_error(MHPPO_EHIP, "env seeding failed: %s", hipGetErrorString(e));
  }
  *out = h;
  return MHPPO_OK;
}

void mhppo_env_destroy(mhppo_env *env) {
  if (!env) return;
  // destroy has no error channel: a failing device switch or free is not reportable here;
  // the caller's current device is restored either way (it may run from a GC finalizer)
  mhppo::DeviceGuard g(env->device);
  (void)hipFree(env->blob);
  delete env;
}

int mhppo_env_obs_dim(const mhppo_env *env) { return env ? env->c.obs_dim : MHPPO_EINVAL; }
int mhppo_env_slots(const mhppo_env *env) { return env ? env->c.nS : MHPPO_EINVAL; }
int mhppo_env_reward_slots(const mhppo_env *env) { return env ? env->c.nAV : MHPPO_EINVAL; }
int mhppo_env_state_dim(const mhppo_env *env) { return env ? 21 * env->c.P + 8 * env->c.nC + 4 : MHPPO_EINVAL; }

int64_t mhppo_env_state_bytes(const mhppo_env *env) { return env ? (int64_t)env->blob_bytes : MHPPO_EINVAL; }

int mhppo_env_export(const mhppo_env *env, void *dst, void *stream) {
  if (!env || !dst) return set_error(MHPPO_EINVAL, "null argument");
  GUARD_DEVICE(env->device);
  CHECK_HIP(hipMemcpyAsync(dst, env->blob, env->blob_bytes, hipMemcpyDefault, (hipStream_t)stream));
  return MHPPO_OK;
}

int mhppo_env_import(mhppo_env *env, const void *src, void *stream) {
  if (!env || !src) return set_error(MHPPO_EINVAL, "null argument");
  GUARD_DEVICE(env->device);
  CHECK_HIP(hipMemcpyAsync(env->blob, src, env->blob_bytes, hipMemcpyDefault, (hipStream_t)stream));
  return MHPPO_OK;
}

int mhppo_env_reset(mhppo_env *env, float *obs, void *stream) {
  if (!env) return set_error(MHPPO_EINVAL, "null env");
  GUARD_DEVICE(env->device);
  dim3 grid((env->c.N + TPB - 1) / TPB);
  VARIANT_LAUNCH(k_env_reset, env->c.variant, grid, (hipStream_t)stream, env->c, env->b, obs);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_env_choix_test(mhppo_env *env, float *obs, void *stream) {
  if (!env) return set_error(MHPPO_EINVAL, "null env");
  if (env->c.variant != V_SCALABLE || env->c.nS < 2)
    return set_error(MHPPO_EINVAL, "choix_test is the scalable driver's scenario (Coop-MH-PPO-scalable.py:629-633); "
                                   "the coop/naif drivers' version calls reset_pedestrian with 8 of its 10 "
                                   "arguments and raises TypeError");
  GUARD_DEVICE(env->device);
  dim3 grid((env->c.N + TPB - 1) / TPB);
  hipLaunchKernelGGL(k_env_choix, grid, dim3(TPB), 0, (hipStream_t)stream, env->c, env->b, obs);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_env_step(mhppo_env *env, const double *actions, float *obs, double *rewards, double *reward_light,
                   uint8_t *done, void *stream) {
  if (!env || !actions) return set_error(MHPPO_EINVAL, "null env/actions");
  GUARD_DEVICE(env->device);
  dim3 grid((env->c.N + TPB - 1) / TPB);
  const Cfg &c = env->c;
#define STEP_REG(V_, NC_, NAV_, NP_)                                                                    \
  if (use_reg_view(c, V_, NC_, NAV_, NP_)) {                                                            \
    hipLaunchKernelGGL((k_env_step_r<V_, NC_, NAV_, NP_>), grid, dim3(TPB), 0, (hipStream_t)stream, c, env->b, \
                       actions, obs, rewards, reward_light, done);                                     \
    CHECK_HIP(hipGetLastError());                                                                       \
    return MHPPO_OK;                                                                                    \
  }
  MHPPO_REG_SHAPES(STEP_REG)
#undef STEP_REG
  VARIANT_LAUNCH(k_env_step, env->c.variant, grid, (hipStream_t)stream, env->c, env->b, actions, obs, rewards,
                 reward_light, done);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_env_get_state(mhppo_env *env, double *out, void *stream) {
  if (!env || !out) return set_error(MHPPO_EINVAL, "null env/out");
  GUARD_DEVICE(env->device);
  dim3 grid((env->c.N + TPB - 1) / TPB);
  int dim = mhppo_env_state_dim(env);
  VARIANT_LAUNCH(k_env_state, env->c.variant, grid, (hipStream_t)stream, env->c, env->b, out, dim);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_env_events(mhppo_env *env, uint32_t *out, void *stream) {
  if (!env || !out) return set_error(MHPPO_EINVAL, "null env/out");
  GUARD_DEVICE(env->device);
  dim3 grid((env->c.N + TPB - 1) / TPB);
  hipLaunchKernelGGL(k_env_events, grid, dim3(TPB), 0, (hipStream_t)stream, env->c, env->b, out);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

int mhppo_env_get_rng(mhppo_env *env, uint32_t *mt, int32_t *mti, void *stream) {
  if (!env || !mt || !mti) return set_error(MHPPO_EINVAL, "null argument");
  GUARD_DEVICE(env->device);
  size_t n = (size_t)env->c.N * 624;
  dim3 grid((unsigned)((n + TPB - 1) / TPB));
  hipLaunchKernelGGL(k_env_rng, grid, dim3(TPB), 0, (hipStream_t)stream, env->c, env->b, mt, mti);
  CHECK_HIP(hipGetLastError());
  return MHPPO_OK;
}

}  // extern "C"

// internal accessors for the rollout kernels (same library)
namespace mhppo {
const Cfg &env_cfg(const mhppo_env *env) { return env->c; }
const Bufs &env_bufs(const mhppo_env *env) { return env->b; }
int env_device(const mhppo_env *env) { return env->device; }
}  // namespace mhppo
