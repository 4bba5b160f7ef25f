/* mhppo.h — C-ABI of libmhppo.so, the MI355X-native hot path of MH-PPO.
 *
 * The reference is pure Python (no FFI); each entry point below replaces a
 * Python call site on the hot path.  Callers bind it
 * with ctypes (mh-ppo_amd/mhppo/_lib.py; INTEGRATION.md shows the binding a
 * maintainer of the reference would add).
 *
 * Conventions
 *  - Every function returns 0 on success or a negative MHPPO_E* code;
 *    mhppo_last_error() returns a thread-local message for the last failure.
 *  - All data pointers are DEVICE pointers owned by the caller (e.g. torch
 *    tensor data_ptr()s on the handle's device); nothing is freed across the ABI.
 *  - Calls are asynchronous on `stream` (a hipStream_t, NULL = default stream).
 *  - A handle is bound to one device and is not re-entrant.
 */
#ifndef MHPPO_H
#define MHPPO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHPPO_OK 0
#define MHPPO_EINVAL -1   /* invalid configuration / argument */
#define MHPPO_EHIP -2     /* HIP runtime error */
#define MHPPO_ENOMEM -3   /* device allocation failed */

/* Env variants = the reference gym ids (Environments/__init__.py:3-42). */
#define MHPPO_COOP 0      /* Crosswalk_hybrid_multi_coop-v0          Env_hybrid_multi_coop.py:625 */
#define MHPPO_4CARS 1     /* Crosswalk_hybrid_multi_coop_4cars-v0    Env_hybrid_multi_coop_4cars.py:667 */
#define MHPPO_SCALABLE 2  /* Crosswalk_hybrid_multi_coop_scalable-v0 Env_hybrid_multi_coop_scalable.py:668 */
#define MHPPO_NAIF 3      /* Crosswalk_hybrid_multi_naif-v0          Env_hybrid_multi_naif.py:616 */

typedef struct mhppo_env_cfg {
    int32_t variant;      /* MHPPO_* */
    int32_t n_envs;       /* N: envs on this handle (this rank's shard) */
    int32_t nb_car, nb_ped, nb_lines;
    int32_t max_episode;  /* 80 in every reference driver */
    int32_t sin_model;    /* simulation == "sin" */
    int32_t reserved;
    double dt;            /* 0.3 */
    double car_b[4];      /* row-major [[acc_min, v],[acc_max, v]] */
    double ped_b[8];      /* row-major [2][4] */
    double cross_b[2];
    uint64_t seed_base;   /* env e draws from random.seed(seed_base + env_id_offset + e) */
    uint64_t env_id_offset;
} mhppo_env_cfg;

typedef struct mhppo_env mhppo_env;

/* Replaces gym.make(id, car_b=..., ...) -> Crosswalk_*.__init__ (Env_hybrid_multi_coop.py:637-692)
 * plus the module-import `random.seed(10)` (:10), per env: seeds N CPython
 * MT19937 streams on the device. */
int mhppo_env_create(const mhppo_env_cfg *cfg, int device, mhppo_env **out);
void mhppo_env_destroy(mhppo_env *env);

/* Geometry of the flat observation (gym-sorted keys car|car_follow|env|ped) and slots. */
int mhppo_env_obs_dim(const mhppo_env *env);
int mhppo_env_slots(const mhppo_env *env);   /* S: AV action slots per env */

/* Replaces Crosswalk_*.reset() (Env_hybrid_multi_coop.py:838-893; 4cars :850-911;
 * scalable :884-946).  obs: float32 [N, obs_dim] or NULL. */
int mhppo_env_reset(mhppo_env *env, float *obs, void *stream);

/* Replaces Crosswalk_*.step(actions) (Env_hybrid_multi_coop.py:745-832; 4cars :783-844;
 * scalable :789-878).  actions: float64 [N, 2S] = [acc_0..acc_{S-1}, light_0..light_{S-1}];
 * obs float32 [N, obs_dim] (nullable); rewards, reward_light float64 [N, S];
 * done uint8 [N]. */
int mhppo_env_step(mhppo_env *env, const double *actions, float *obs, double *rewards,
                   double *reward_light, uint8_t *done, void *stream);

/* Read back the per-env scalar/attribute view the reference drivers touch
 * (env.cross, ped_traffic, car_traffic, cars[i].exist, pedestrian[j].waiting_time,
 * internal flags): out float64 [N, mhppo_env_state_dim()]. */
int mhppo_env_state_dim(const mhppo_env *env);
int mhppo_env_get_state(mhppo_env *env, double *out, void *stream);
/* RNG cursor: mt uint32 [N, 624], mti int32 [N] (device). */
int mhppo_env_get_rng(mhppo_env *env, uint32_t *mt, int32_t *mti, void *stream);

/* ---- rollout collector (Env_rollout.iterations_rand, Coop-MH-PPO-scalable.py:357-517) ---- */

/* Model_PPO weights of one MLP (Coop-MH-PPO-scalable.py:42-93) in torch layout:
 * W1 [32,in] b1 [32] W2 [64,32] b2 [64] W3 [32,64] b3 [32] W4 [out,32] b4 [out]. */
typedef struct mhppo_mlp {
    const float *w1, *b1, *w2, *b2, *w3, *b3, *w4, *b4;
    int32_t n_in, n_out;
} mhppo_mlp;

/* t=0 choice features, obs_car_ped_d (Coop-MH-PPO-scalable.py:574-611): feat_d float32
 * [N, S, P, dc]; closest ped per slot (closest_ped_d :614-627): int32 [N, S]. */
int mhppo_featurize_choice(mhppo_env *env, float *feat_d, int32_t *closest, void *stream);
int mhppo_choice_dim(const mhppo_env *env);

/* Choice head forward + Categorical sample for every (env, slot, ped)
 * (:403-428).  u: float32 [N,S,P] uniforms (parity replay or Philox draws);
 * outputs a_d int32 [N,S,P], logp_d float32 [N,S,P], probs float32 [N,S,P,2]. */
int mhppo_choice_sample(mhppo_env *env, const mhppo_mlp *actor_choice, const float *feat_d,
                        const float *u, int32_t *a_d, float *logp_d, float *probs, void *stream);

/* One fused rollout step (:430-461): obs_car_ped features for every (slot, ped),
 * cross/wait head forward selected by action_d, min over existing peds, MVN(loc, 0.5)
 * sample from eps float32 [N,S], env step, episodic min of reward_light.
 * Writes step t of the rollout buffers: obs_c float32 [N,S,T,13], act float32 [N,S,T],
 * logp float32 [N,S,T], rew float64 [N,S,T]; updates ep_min float64 [N,S]. */
int mhppo_rollout_step(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                       const int32_t *action_d, const int32_t *light_d, const float *eps, int t,
                       int T, float *obs_c, float *act, float *logp, double *rew, double *ep_min,
                       void *stream);

/* Philox-4x32-10 noise for the rollout (perf mode): normal eps [n] and uniforms [n],
 * counter = (seed, offset + i). */
int mhppo_philox_normal(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream);
int mhppo_philox_uniform(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream);

/* ---- returns / advantage / PPO losses (futur_rewards :658-684, train_model_c/_d :778-851) ---- */

/* Segmented reverse discounted scan: G_t = r_t + gamma*G_{t+1} in float64, one segment
 * of T per row; rew float64 [B, T] -> ret float32 [B, T]. */
int mhppo_returns_scan(const double *rew, float *ret, int64_t B, int32_t T, double gamma, void *stream);

/* Advantage A = G - V, then (A - mean) / (std_unbiased + 1e-10) over M rows.
 * stats float64 [3] receives (sum A, sum A^2, M) — partial sums when `local_only`
 * (multi-GPU: all-reduce then call mhppo_adv_normalize). */
int mhppo_adv_stats(const float *ret, const float *value, int64_t M, double *stats, void *stream);
int mhppo_adv_normalize(const float *ret, const float *value, int64_t M, const double *stats,
                        float *adv, void *stream);

/* Continuous PPO clip surrogate (:795-806): logp = MVN(mu, 0.5).log_prob(act),
 * ratio = exp(logp - logp_old) in float64, L = mean(-min(r A, clip(r, .8, 1.2) A)).
 * Writes dL/dmu float32 [M] (already scaled by 1/M_global) and loss_sum float64 [1]. */
int mhppo_ppo_cont_fwd_bwd(const float *mu, const float *act, const double *logp_old,
                           const float *adv, int64_t M, double inv_m, float *dmu,
                           double *loss_sum, void *stream);

/* Choice PPO surrogate over the reference's M x M broadcast (:834-842) in its exact
 * O(M) form: L = (1/M^2) sum_j [n0 f(r_j0, A_j) + n1 f(r_j1, A_j)].  probs float32
 * [M,2] (softmax outputs), counts int64 [2] = (n0, n1).  Writes dL/dprobs [M,2]. */
int mhppo_ppo_choice_fwd_bwd(const float *probs, const double *logp_old, const float *adv,
                             int64_t M, const double *counts, double inv_m2, float *dprobs,
                             double *loss_sum, void *stream);

/* Critic MSE (:808-809): loss_sum = sum (V-G)^2, dV = 2 (V-G) * inv_m. */
int mhppo_mse_fwd_bwd(const float *value, const float *ret, int64_t M, double inv_m, float *dv,
                      double *loss_sum, void *stream);

const char *mhppo_last_error(void);
const char *mhppo_version(void);

#ifdef __cplusplus
}
#endif
#endif
