// env_body.h — per-env reset/step/state bodies (host+device).  The HIP
// kernels in mhppo_env.hip launch one lane per env over these; tools/hostsim.cpp
// runs the same source on the CPU.
#pragma once
#include <string.h>

#include "../../include/mhppo.h"
#include "env_dev.h"

namespace mhppo {
constexpr int MAXS = 16;  // AV slots per env (scalable 2*nb_lines, coop nb_car)

// Shapes (variant, nC, nAV, P) with a register-view step kernel: the benchmark configs
// (coop 2/1/2, 4cars 4/1/2, scalable 8/1/4) and the other single-pedestrian fixture
// shapes (stop 2/1/2, 4cars2 4/1/2).  Every other shape runs on the generic view.
// (Multi-pedestrian shapes are left generic: fully unrolling ped_step per pedestrian
// exceeds the unroller's budget and a runtime-indexed array would live in scratch.)
#define MHPPO_REG_SHAPES(X) \
  X(V_COOP, 2, 2, 1) X(V_4CARS, 8, 4, 1) X(V_SCALABLE, 8, 8, 1) X(V_STOP, 2, 2, 1) X(V_4CARS2, 8, 4, 1)

inline bool use_reg_view(const Cfg &c, int V_, int NC, int NAV, int NP) {
  return !(c.flags & MHPPO_GENERIC_STEP) && c.variant == V_ && c.nC == NC && c.nAV == NAV && c.P == NP;
}

// ----------------------------------------------------------------- reset
template <class EV>
MHPPO_HD void ped_init(EV &E, Ped &q, int is_crossing, int exist) {
  constexpr int V = EV::VAR;
  auto &r = E.rng;
  const Cfg &c = E.c;
  q = Ped{};
  q.wdl = 0.0;
  q.fl = 0;
  q.set(F_ISCROSS, is_crossing);
  (void)r.randint(0, 20);  // time_to_remove (never read)
  q.set(F_FOLLOW, r.randint(0, 9) < (V == V_NAIF ? 10 : 3));
  q.set(F_EXIST, exist);
  q.dir = 2 * r.randint(0, 1) - 1;
  q.lpos = (double)(c.nb_lines * (q.dir < 0) - 1 * (q.dir > 0));
  q.ivx = r.uniform(c.pb[0][0], c.pb[1][0]);
  q.ivy = r.uniform(c.pb[0][1], c.pb[1][1]) * (double)q.dir;
  double px = r.uniform(c.pb[0][2], c.pb[1][2]);
  double py = (r.uniform(c.pb[0][3], c.pb[1][3]) - E.cl / 2.) * (double)q.dir;
  q.ratio = 0.0;
  if (!exist) {
    q.ivx = 0.;
    q.ivy = 0.;
    if (V == V_4CARS || V == V_NAIF || V == V_4CARS2 || V == V_STOP) px = c.pb[0][2];
    py = c.pb[0][3] * (double)q.dir;
  } else if (!is_crossing) {
    q.ivx = 0.;
    q.ivy = 0.;
    q.dir = 0;
  } else {
    q.ratio = q.ivx / q.ivy;
  }
  q.Vx = q.ivx;
  q.Vy = q.ivy;
  q.Sx = px;
  q.Sy = py;
  q.tstop = 0;
  q.t0 = 0.0;
  q.set(F_GENDER, r.randint(0, 1) == 1);
  int age = r.randint(0, 2);
  q.fl = (q.fl & ~F_AGE_MASK) | ((uint32_t)age << F_AGE_SHIFT);
  (void)CG_score(E, q, E.cross);  // self.CG: draws, never read
  q.delta = 0.0;
  q.cstop = 0.0;
  if (V == V_COOP) {
    q.set(F_NEEDSTOP, true);
    q.cstop = r.uniform(-E.cl / 2 + 0.2, E.cl / 2 - 0.2);
  } else if (V == V_SCALABLE || V == V_4CARS2 || V == V_STOP) {
    q.set(F_NEEDSTOP, r.uniform(0, 1) < 0.5);
    q.cstop = r.uniform(-E.cl / 2 + 0.2, E.cl / 2 - 0.2);
  }
  q.A = q.B = q.W = 0.0;
  if (c.sin_model && is_crossing) {
    q.set(F_SIN, true);
    double abs_speed = fabs(q.ivy);
    double T = E.cl / (abs_speed + 10e-3);
    int check = ((abs_speed * PI) / 2.0 <= 2.5);
    q.A = (double)check * PI * abs_speed / 2.0 + (double)(!check) * (2.5 - abs_speed) / (1.0 - (2.0 / PI));
    q.B = (double)(!check) * (2.5 - q.A);
    q.W = PI / T;
  }
}

template <class EV>
MHPPO_HD void car_init(EV &E, int s, double line, double offset, int exist) {
  constexpr int V = EV::VAR;
  const Cfg &c = E.c;
  double finish = (E.cl * 10.0) / (c.mean_speed_ped);
  double Sc = E.rng.uniform(c.car_low - finish, c.car_high);
  if (V == V_SCALABLE) Sc = Sc - 20.0 * offset;
  E.car(C_AC, s) = 0.;
  E.car(C_VC, s) = 10.0;
  E.car(C_SC, s) = Sc;
  E.car(C_LIGHT, s) = 0.;
  E.car(C_PA, s) = 0.0;
  E.car(C_ES, s) = 0.0;
  E.car(C_TS, s) = (V == V_SCALABLE) ? 0. : -10.;
  E.hist_nf(0) &= ~(int32_t)(1u << s);  // history = [0, 0]
  E.hist_nf(1) &= ~(int32_t)(1u << s);
  E.set_line(s, line);
  E.set_exist(s, exist ? 1.0 : 0.0);
}

// car.get_data for the flat obs (coop :609-612, scalable :652-655)
template <class EV>
MHPPO_HD int write_car_obs(const EV &E, int s, float *o) {
  constexpr int V = EV::VAR;
  if (V == V_SCALABLE) {
    if (E.exists(s) == 0.0) {
      o[0] = 0.f; o[1] = 0.f; o[2] = 10.f; o[3] = -1000.f; o[4] = 0.f; o[5] = (float)E.line(s); o[6] = 0.f;
    } else {
      double Vc = E.car(C_VC, s);
      o[0] = (float)E.car(C_AC, s); o[1] = (float)Vc; o[2] = (float)(10.0 - Vc); o[3] = (float)E.car(C_SC, s);
      o[4] = (float)E.car(C_LIGHT, s); o[5] = (float)E.line(s); o[6] = 1.f;
    }
    return 7;
  }
  double Vc = E.car(C_VC, s);
  o[0] = (float)E.car(C_AC, s); o[1] = (float)Vc; o[2] = (float)(10.0 - Vc); o[3] = (float)E.car(C_SC, s);
  o[4] = (float)E.car(C_LIGHT, s); o[5] = (float)E.line(s);
  return 6;
}

// flat obs (gym-sorted car|car_follow|env|ped); ped.get_data runs even without
// an obs buffer because it advances the running-min `delta` (:441).
// The register view (EV::OBS_DIM > 0) builds the row in its staging buffer (the wave's LDS
// image on the device) and writes the wave's 64 rows as one coalesced block
// (EnvR::store_obs_row); the generic view writes the row in place.
template <class EV>
MHPPO_HD void env_observe(EV &E, int mode, float *obs) {
  constexpr int V = EV::VAR;
  constexpr int OD = EV::OBS_DIM;
  const Cfg &c = E.c;
  float *o;
  if constexpr (OD > 0) o = E.obs_stage();
  else o = obs ? obs + (size_t)E.e * c.obs_dim : nullptr;
  float tmp[8];
  int k = 0;
  if (o) {
    MHPPO_UNROLL
    for (int s = 0; s < E.nC(); s++) {
      const int w = write_car_obs(E, s, tmp);
      MHPPO_UNROLL
      for (int j = 0; j < 8; j++)  // w <= 7, known after inlining: constant offsets
        if (j < w) o[k + j] = tmp[j];
      k += w;
    }
    o[k++] = (float)(E.cross * (double)c.nb_lines / 2.);
    o[k++] = (float)E.ped_traffic();
    if (V == V_SCALABLE) o[k++] = (float)E.car_traffic();
    o[k++] = (float)c.nb_lines;
  }
  MHPPO_MARK(11);
  MHPPO_UNROLL
  for (int p = 0; p < E.nP(); p++) {
    Ped q = load_ped(E, p);
    double d[9];
    ped_get_data(E, q, mode, d);
    E.pedf(P_DELTA, p) = q.delta;
    if (o) {
      MHPPO_UNROLL
      for (int j = 0; j < 9; j++) o[k + j] = (float)d[j];
      k += 9;
    }
  }
  MHPPO_MARK(12);
  if constexpr (OD > 0) {
    if (obs) E.store_obs_row(obs);
  }
}

template <int V>
MHPPO_HD void env_reset_one(const Cfg &c, const Bufs &b, int e, float *obs) {
  // cross first: it sizes everything else (:844)
  Env<V> E(c, b, e);
  E.hist_nf(0) = 0;  // every car's history = [0, 0] (car_init clears its own bits as well)
  E.hist_nf(1) = 0;
  E.cross = E.rng.uniform(c.xb0, c.xb1);
  E.cl = (double)c.nb_lines * E.cross;
  b.envd[sidx(E_ND, E_CROSS, e)] = E.cross;
  for (int k = 0; k < EV_N; k++) b.ev[sidx(EV_N, k, e)] = 0u;  // counters are per episode
  for (int p = 0; p < c.P; p++) {
    Ped q;
    ped_init(E, q, 0, 0);
    store_ped(E, p, q, false);
  }
  int car_traffic = c.nb_car;
  if (V == V_SCALABLE) {
    // car(..., i//2) then line = (i//2)//2, offset (i//2)%2 (:900-906, :537, :576); the
    // MHPPO_FIX_SCALABLE_LANES bug-fix passes the slot itself
    const bool fix = (c.flags & MHPPO_FIX_SCALABLE_LANES) != 0;
    auto ci = [&](int i) { return fix ? i : i / 2; };
    for (int i = 0; i < c.nS; i++) car_init(E, i, (double)(ci(i) / 2), (double)(ci(i) % 2), 0);
    car_traffic = E.rng.randint(1, c.nb_car);
    // random.sample(range(S), k) (pool algorithm) draws every index first; the
    // chosen cars are then re-built in sample order (:903-906)
    uint64_t pool = 0, order = 0;
    for (int i = 0; i < c.nS; i++) pool |= (uint64_t)i << (4 * i);
    for (int k = 0; k < car_traffic; k++) {
      int j = (int)E.rng.randbelow((uint32_t)(c.nS - k));
      uint64_t pick = (pool >> (4 * j)) & 15u;
      uint64_t last = (pool >> (4 * (c.nS - k - 1))) & 15u;
      pool = (pool & ~(15ull << (4 * j))) | (last << (4 * j));
      order |= pick << (4 * k);
    }
    for (int k = 0; k < car_traffic; k++) {
      int pick = (int)((order >> (4 * k)) & 15u);
      car_init(E, pick, (double)(ci(pick) / 2), (double)(ci(pick) % 2), 1);
    }
  } else {
    for (int i = 0; i < c.nb_car; i++) car_init(E, i, (double)(i % c.nb_lines), 0, 1);
    if (has_followers(V))
      for (int i = 0; i < c.nb_car; i++) car_init(E, c.nAV + i, E.line(i), 0, 1);
  }
  b.envi[sidx(EI_NI, EI_CARTRAF, e)] = car_traffic;
  int ped_traffic = E.rng.randint(1, c.nb_ped);
  b.envi[sidx(EI_NI, EI_PEDTRAF, e)] = ped_traffic;
  for (int p = 0; p < ped_traffic; p++) {
    Ped q;
    ped_init(E, q, 1, 1);
    store_ped(E, p, q, false);
  }
  if (has_followers(V)) {
    for (int i = 0; i < c.nb_car; i++) {  // reset_car(speed_limit, Sc - 15., 0, line) (:878-879; 4cars2 Sc - U(10,30) :895)
      const double gap = V == V_4CARS2 ? E.rng.uniform(10, 30) : 15.;
      E.car(C_SC, c.nAV + i) = E.car(C_SC, i) - gap;
      E.car(C_VC, c.nAV + i) = 10.0;
      E.car(C_LIGHT, c.nAV + i) = 0.;
      E.set_line(c.nAV + i, E.line(i));
    }
  }
  env_observe(E, 0, obs);
  b.envd[sidx(E_ND, E_TIME, e)] = 0.0;
  E.save_rng();
}

// ------------------------------------------------------------ choix_test
// Env_rollout.choix_test (Coop-MH-PPO-scalable.py:629-633) right after a reset, then the
// driver's env.get_state() (:171-172); scalable env (oracle_env_choix_test restates it):
// cross = 3; every pedestrian rebuilt non-crossing / non-existent (reset_pedestrian
// :948-955, their draws), pedestrian 0 reset_ped (:106-134) to speed (0, 1.25) at (0, -1),
// direction +1, ped_left = -1 and ped_in_cross = cross as VALUES (the observation shows
// them; the flags hold their truthiness, which is all the dynamics read before the next
// step's boolean_ped_position), a CG_score draw, the sin profile; cars 0/1 reset_car
// (:583-587) to (state["car"][1], -45 / -22, light 0, lane 0 / 1), state["car"][1] being
// car 0's float32 observed speed.  (NumPy >= 2 would then step cars 0/1 in float32 — NEP 50
// on that np.float32 speed; the reference's pinned NumPy 1.26 promotes to float64, as here.)
template <int V>
MHPPO_HD void env_choix_test_one(const Cfg &c, const Bufs &b, int e, float *obs) {
  Env<V> E(c, b, e);
  const double v0 = (double)(float)(E.exists(0) != 0.0 ? E.car(C_VC, 0) : 0.0);
  E.cross = 3.0;
  E.cl = (double)c.nb_lines * E.cross;
  b.envd[sidx(E_ND, E_CROSS, e)] = E.cross;
  for (int p = 0; p < c.P; p++) {
    Ped q;
    ped_init(E, q, 0, 0);
    store_ped(E, p, q, false);
  }
  Ped q = load_ped(E, 0);
  q.ivx = 0.0;
  q.ivy = 1.25;
  q.Vx = q.ivx;
  q.Vy = q.ivy;
  q.Sx = 0.0;
  q.Sy = -1.0;
  q.ratio = q.ivx / (q.ivy + 1e-3);
  q.dir = 1;
  q.lpos = (double)(c.nb_lines * (q.dir < 0) - 1 * (q.dir > 0));
  q.delta = 0.0;
  q.set(F_EXIST, true);
  q.set(F_LEFT, true);     // leave = -1 (truthy)
  q.set(F_INCROSS, true);  // CZ = cross = 3. (truthy)
  q.set(F_ISCROSS, true);
  (void)CG_score(E, q, E.cl);  // self.CG = CG_score(cross_lines): its normalvariate draw
  q.set(F_SIN, c.sin_model != 0);
  q.A = q.B = q.W = 0.0;
  if (c.sin_model) {
    const double abs_speed = fabs(q.ivy);
    const double T = E.cl / (abs_speed + 10e-3);
    const int check = ((abs_speed * PI) / 2.0 <= 2.5);
    q.A = (double)check * PI * abs_speed / 2.0 + (double)(!check) * (2.5 - abs_speed) / (1.0 - (2.0 / PI));
    q.B = (double)(!check) * (2.5 - q.A);
    q.W = PI / T;
  }
  store_ped(E, 0, q, false);
  E.car(C_SC, 0) = -45.0; E.car(C_VC, 0) = v0; E.car(C_LIGHT, 0) = 0.0; E.set_line(0, 0.0);
  E.car(C_SC, 1) = -22.0; E.car(C_VC, 1) = v0; E.car(C_LIGHT, 1) = 0.0; E.set_line(1, 1.0);
  env_observe(E, 0, obs);
  if (obs) {  // get_data shows ped_left / ped_in_cross as stored: -1 and 3.0
    float *o = obs + (size_t)e * c.obs_dim + (c.obs_dim - 9 * c.P);
    o[5] = -1.0f;
    o[6] = (float)E.cross;
  }
  E.save_rng();
}

// ------------------------------------------------------------------ step
// act: this env's [2 nS] actions [acc..., light...]; rw/rl: this env's [nAV] outputs (nullable)
// act: [2 nS] (pointer or array type); per-AV rewards land in E.rw / E.rl
template <class EV, class ACT>
MHPPO_HD void env_step_body(EV &E, const ACT &act, float *obs, uint8_t *done) {
  constexpr int V = EV::VAR;
  const Cfg &c = E.c;
  const Bufs &b = E.b;
  const int e = E.e;
  const int nS = E.nAV();  // AV slots (4cars2: followers handled below)
  double time = b.envd[sidx(E_ND, E_TIME, e)];
  E.rng.prefetch();  // register view: the draws' window, in flight during the car steps
  typename EV::AvArr prev, acc;
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) prev[i] = E.car(C_SC, i);
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) {
    double a = act[i];
    if (V == V_SCALABLE) {
      double idm = 2.;
      if (i % 2 == 1 && E.exists(i - 1) != 0.0 && E.exists(i) != 0.0)
        idm = car_follow_action(E, i, E.car(C_VC, i - 1), E.car(C_SC, i - 1));
      a = pymin(idm, a);
    }
    car_step(E, i, a, act[i + E.nS()]);
  }
  if (has_followers(V)) {
    MHPPO_UNROLL
    for (int i = 0; i < nS; i++) {  // one follower per AV (nb_car == nAV)
      double a = car_follow_action(E, nS + i, E.car(C_VC, i), E.car(C_SC, i));
      double light = E.car(C_LIGHT, i);
      if (V == V_4CARS2) {  // follower step(action_ppo, action_light, leader) (:75-79, :811)
        a = pymin(a, act[nS + i]);
        light = act[E.nS() + nS + i];
      }
      car_step(E, nS + i, a, light);
    }
  }
  E.commit_cars();
  MHPPO_MARK(4);
  MHPPO_UNROLL
  for (int p = 0; p < E.nP(); p++) {
    Ped q = load_ped(E, p);
    ped_step(E, q, time);
    store_ped(E, p, q, true);
  }
  E.commit_peds();
  MHPPO_MARK(5);
  // The observation (:825-832, get_state after detection and rewards) reads only fields that
  // detection and the rewards never write (cars' kinematics/light/line/existence, the
  // pedestrians' kinematics/flags other than accident/worst-scenario, and the running-min
  // delta that only get_data itself updates), so it is taken here, right after the
  // pedestrian step: its wave-coalesced block store then drains while detection and the
  // rewards compute instead of at the very end of the step.
  env_observe(E, 1, obs);
  MHPPO_MARK(8);
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) acc[i] = 0.;
  MHPPO_UNROLL
  for (int p = 0; p < E.nP(); p++) {
    Ped q = load_ped(E, p);
    bool add = q.has(F_ISCROSS) && (V != V_SCALABLE || q.has(F_EXIST));
    ped_detection(E, q, prev, acc, add);
    E.pflag(p) = (E.pflag(p) & ~(F_ACCIDENT | F_WSA | F_PNW)) | (q.fl & (F_ACCIDENT | F_WSA | F_PNW));
  }
  E.commit_det();
  MHPPO_MARK(6);
  MHPPO_UNROLL
  for (int i = 0; i < nS; i++) {
    E.rl[i] = acc[i];
    double Vc = E.car(C_VC, i);
    double r = car_reward(Vc);
    if (E.car(C_LIGHT, i) > 0.0) {
      bool have = false;
      double mn = 0.;
      MHPPO_UNROLL
      for (int p = 0; p < E.nP(); p++) {
        uint32_t fl = E.pflag(p);
        if (!(fl & F_EXIST)) continue;
        Ped q = load_ped(E, p);
        double w = new_reward_wait_safety(E, q, Vc, E.car(C_SC, i), E.line(i));
        E.pedf(P_WDL, p) = q.wdl;
        if (!have) { mn = w; have = true; }
        else if (w < mn) mn = w;
      }
      if (have) r += mn;
    }
    E.rw[i] = r;
  }
  MHPPO_MARK(7);
  int d = (time >= c.ep_len) || (E.ped_traffic() <= 0);
  if (done) done[e] = (uint8_t)d;
  b.envd[sidx(E_ND, E_TIME, e)] = time + c.dt;
  E.commit();
  MHPPO_MARK(9);
}

template <int V>
MHPPO_HD void env_step_one(const Cfg &c, const Bufs &b, int e, const double *act, float *obs, double *rw,
                           double *rl, uint8_t *done) {
  Env<V> E(c, b, e);
  env_step_body(E, act, obs, done);
  for (int i = 0; i < c.nAV; i++) {
    if (rw) rw[i] = E.rw[i];
    if (rl) rl[i] = E.rl[i];
  }
}


// ------------------------------------------------------------- seeding
MHPPO_HD inline void env_seed_one(const Cfg &c, const Bufs &b, int e) {
  uint32_t *blk = b.mt + (size_t)e * (MT_BLOCKS * MT_N);
  rng_seed(blk, c.seed_base + c.env_off + (uint64_t)e);
  for (int k = 1; k < MT_BLOCKS; k++) mt_twist_into(blk + (k - 1) * MT_N, blk + k * MT_N);  // ring ready
  b.envi[sidx(EI_NI, EI_MTI, e)] = MT_N;
  b.envi[sidx(EI_NI, EI_MTB, e)] = 0;
  b.envd[sidx(E_ND, E_CROSS, e)] = 0.0;
  b.envd[sidx(E_ND, E_TIME, e)] = 0.0;
}

// ------------------------------------------------------------- state dump
// [peds 20P][AV cars 8 nS][followers 8 (nC-nS)][cross, time, ped_traffic, car_traffic][ped exist P]
template <int V>
MHPPO_HD void env_state_one(const Cfg &c, const Bufs &b, int e, double *out, int dim) {
  Env<V> E(c, b, e);
  double *o = out + (size_t)e * dim;
  int k = 0;
  for (int p = 0; p < c.P; p++) {
    Ped q = load_ped(E, p);
    double f[20] = {q.Sx, q.Sy, q.Vx, q.Vy, (double)q.has(F_DECISION), (double)q.has(F_ATCROSS),
                    (double)q.has(F_LEFT), (double)q.has(F_INCROSS), (double)q.has(F_ACCIDENT), (double)q.tstop,
                    (double)q.has(F_STOP), q.lpos, q.wt, q.ct, q.wdl, q.delta, q.t0,
                    (double)q.has(F_NEEDSTOP), (double)q.dir, (double)q.has(F_FOLLOW)};
    for (int j = 0; j < 20; j++) o[k++] = f[j];
  }
  for (int s = 0; s < c.nC; s++) {
    double f[8] = {E.car(C_AC, s), E.car(C_VC, s), E.car(C_SC, s), E.car(C_LIGHT, s),
                   E.car(C_PA, s), E.car(C_ES, s), E.car(C_TS, s), E.exists(s)};
    for (int j = 0; j < 8; j++) o[k++] = f[j];
  }
  o[k++] = E.cross;
  o[k++] = b.envd[sidx(E_ND, E_TIME, e)];
  o[k++] = (double)b.envi[sidx(EI_NI, EI_PEDTRAF, e)];
  o[k++] = (double)b.envi[sidx(EI_NI, EI_CARTRAF, e)];
  for (int p = 0; p < c.P; p++) o[k++] = (E.pflag(p) & F_EXIST) ? 1.0 : 0.0;
}


// host: mhppo_env_cfg -> Cfg (constants that are transcendental functions of the
// config are evaluated here, with glibc, exactly as the reference does)
inline void build_cfg(const mhppo_env_cfg &cfg_, Cfg &c) {
  const mhppo_env_cfg *cfg = &cfg_;
  int nS = cfg->variant == V_SCALABLE ? 2 * cfg->nb_lines : (cfg->variant == V_4CARS2 ? 2 : 1) * cfg->nb_car;
  memset(&c, 0, sizeof(c));
  c.variant = cfg->variant;
  c.N = cfg->n_envs;
  c.nb_car = cfg->nb_car;
  c.nb_ped = cfg->nb_ped;
  c.nb_lines = cfg->nb_lines;
  c.nS = nS;
  c.nAV = cfg->variant == V_4CARS2 ? cfg->nb_car : nS;
  c.nC = has_followers(cfg->variant) ? 2 * cfg->nb_car : nS;
  c.P = cfg->nb_ped;
  c.max_episode = cfg->max_episode;
  c.sin_model = cfg->sin_model;
  c.obs_dim = has_followers(cfg->variant) ? 12 * cfg->nb_car + 3 + 9 * c.P
                                      : (cfg->variant == V_SCALABLE ? 7 * nS + 4 + 9 * c.P : 6 * nS + 3 + 9 * c.P);
  c.dt = cfg->dt;
  c.dt2 = pow(cfg->dt, 2.0);  // math.pow(self.dt, 2.0) (:604), glibc on the host
  c.b00 = cfg->car_b[0];
  c.b10 = cfg->car_b[2];
  for (int i = 0; i < 8; i++) c.pb[i / 4][i % 4] = cfg->ped_b[i];
  c.xb0 = cfg->cross_b[0];
  c.xb1 = cfg->cross_b[1];
  c.idm_den = 2 * sqrt(-c.b00 * c.b10);                 // (:619)
  c.ep_len = (double)(cfg->max_episode - 1) * cfg->dt;  // episode_length (:892)
  c.mean_speed_ped = c.pb[0][1] + c.pb[1][1] / 2;       // (:549)
  c.car_low = (c.pb[0][3] * 10.0) / c.pb[0][1];         // low_car_range (:557)
  c.car_high = (c.pb[1][3] * 10.0) / c.pb[1][1];        // high_car_range (:558)
  c.seed_base = cfg->seed_base;
  c.env_off = cfg->env_id_offset;
  c.flags = cfg->flags;
  c.tb = -(10.0 / (2.0 * c.b00)) + 1.;  // (:564) as the device computed it per call
  {
    const double d = -2.0 * c.b00;
    int e = 0;
    c.brake_p2 = d > 0.0 && frexp(d, &e) == 0.5;  // d = 2^(e-1): 1 / d is exact
    c.brake_inv = c.brake_p2 ? 1.0 / d : 0.0;
  }
}
}  // namespace mhppo
