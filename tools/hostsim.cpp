// hostsim.cpp — runs the device env source (env_body.h) on the CPU, one env at a
// time, for debugging the HIP path against the oracle without a GPU.  Host libm
// (glibc) is used for transcendentals, so any mismatch vs the oracle is logic.
// Build: make -C tools hostsim   ->  tools/libhostsim.so (ctypes)
#include <stdlib.h>
#include <string.h>

#include "../mh-ppo_amd/csrc/env_body.h"

using namespace mhppo;

struct HostEnv {
  Cfg c;
  Bufs b;
  void *blob;
};

extern "C" {
HostEnv *hs_create(const mhppo_env_cfg *cfg) {
  HostEnv *h = new HostEnv();
  build_cfg(*cfg, h->c);
  const Cfg &c = h->c;
  size_t N = npad(c.N);
  h->b.car = (double *)calloc((size_t)C_NF * c.nC * N, 8);
  h->b.ped = (double *)calloc((size_t)P_NF * c.P * N, 8);
  h->b.pfl = (uint32_t *)calloc((size_t)c.P * N, 4);
  h->b.envd = (double *)calloc((size_t)E_ND * N, 8);
  h->b.envi = (int32_t *)calloc((size_t)EI_NI * N, 4);
  h->b.ev = (uint32_t *)calloc((size_t)EV_N * N, 4);
  h->b.carb = (uint8_t *)calloc((size_t)2 * c.nC * N, 1);
  h->b.mt = (uint32_t *)calloc((size_t)MT_BLOCKS * MT_N * c.N + MT_PAD, 4);
  for (int e = 0; e < c.N; e++) env_seed_one(c, h->b, e);
  return h;
}
void hs_destroy(HostEnv *h) {
  if (!h) return;
  free(h->b.car);
  free(h->b.ped);
  free(h->b.pfl);
  free(h->b.envd);
  free(h->b.envi);
  free(h->b.ev);
  free(h->b.carb);
  free(h->b.mt);
  delete h;
}
int hs_obs_dim(HostEnv *h) { return h->c.obs_dim; }
int hs_state_dim(HostEnv *h) { return 21 * h->c.P + 8 * h->c.nC + 4; }
#define HS_DISPATCH(call)                                     \
  switch (h->c.variant) {                                     \
    case V_COOP: { constexpr int V = V_COOP; call; } break;     \
    case V_4CARS: { constexpr int V = V_4CARS; call; } break;   \
    case V_SCALABLE: { constexpr int V = V_SCALABLE; call; } break; \
    case V_NAIF: { constexpr int V = V_NAIF; call; } break;     \
    case V_4CARS2: { constexpr int V = V_4CARS2; call; } break; \
    default: { constexpr int V = V_STOP; call; } break;         \
  }
int hs_reward_slots(HostEnv *h) { return h->c.nAV; }
void hs_reset(HostEnv *h, float *obs) {
  for (int e = 0; e < h->c.N; e++) HS_DISPATCH(env_reset_one<V>(h->c, h->b, e, obs));
}
int hs_choix(HostEnv *h, float *obs) {
  if (h->c.variant != V_SCALABLE) return -1;
  for (int e = 0; e < h->c.N; e++) env_choix_test_one<V_SCALABLE>(h->c, h->b, e, obs);
  return 0;
}
void hs_step(HostEnv *h, const double *a0, float *obs, double *rew0, double *rl0, uint8_t *done) {
  const int S = h->c.nS, R = h->c.nAV;
  for (int e = 0; e < h->c.N; e++) {
    const double *a = a0 + (size_t)e * 2 * S;
    double *rew = rew0 + (size_t)e * R, *rl = rl0 + (size_t)e * R;
    bool reg = false;
    // the register env view for the shapes the device compiles it for (as mhppo_env_step)
#define HS_REG(V_, NC_, NAV_, NP_)                                       \
    if (!reg && use_reg_view(h->c, V_, NC_, NAV_, NP_)) {                \
      EnvR<V_, NC_, NAV_, NP_> E(h->c, h->b, e);                         \
      env_step_body(E, a, obs, done);                                    \
      for (int i = 0; i < R; i++) { rew[i] = E.rw[i]; rl[i] = E.rl[i]; } \
      reg = true;                                                        \
    }
    MHPPO_REG_SHAPES(HS_REG)
#undef HS_REG
    if (!reg) HS_DISPATCH(env_step_one<V>(h->c, h->b, e, a, obs, rew, rl, done));
  }
}
void hs_events(HostEnv *h, uint32_t *out) {
  for (int e = 0; e < h->c.N; e++)
    for (int k = 0; k < EV_N; k++) out[(size_t)e * EV_N + k] = h->b.ev[sidx(EV_N, k, e)];
}
void hs_state(HostEnv *h, double *out) {
  int dim = hs_state_dim(h);
  for (int e = 0; e < h->c.N; e++) HS_DISPATCH(env_state_one<V>(h->c, h->b, e, out, dim));
}
}
