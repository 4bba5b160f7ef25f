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
#define MHPPO_ENAN -4     /* NaN policy output: the reference raises ValueError from torch.distributions'
                             argument validation (Categorical probs / MultivariateNormal loc) */

/* Env variants = the reference gym ids (Environments/__init__.py:3-42). */
#define MHPPO_COOP 0      /* Crosswalk_hybrid_multi_coop-v0          Env_hybrid_multi_coop.py:625 */
#define MHPPO_4CARS 1     /* Crosswalk_hybrid_multi_coop_4cars-v0    Env_hybrid_multi_coop_4cars.py:667 */
#define MHPPO_SCALABLE 2  /* Crosswalk_hybrid_multi_coop_scalable-v0 Env_hybrid_multi_coop_scalable.py:668 */
#define MHPPO_NAIF 3      /* Crosswalk_hybrid_multi_naif-v0          Env_hybrid_multi_naif.py:616 */
#define MHPPO_4CARS2 4    /* Crosswalk_hybrid_multi_coop_4cars2-v0   Env_hybrid_multi_coop_4cars2.py:683
                             (env only: actions [AV acc, follower acc, AV light, follower light]) */
#define MHPPO_STOP 5      /* Crosswalk_hybrid_multi_stop-v0          Env_hybrid_multi_stop.py:634 */
/* mhppo_env_cfg.flags */
#define MHPPO_FIX_SCALABLE_LANES 1 /* scalable: build slot i's car with i (lane i//2, follower 20 m behind
                                      when i is odd) instead of i//2 (lane (i//2)//2, :900-906, :537, :576) */
#define MHPPO_GENERIC_STEP 2       /* not a semantic flag: always run the step on the generic in-HBM env view
                                      (the register view serves the shapes it is compiled for; tests compare both) */

typedef struct mhppo_env_cfg {
    int32_t variant;      /* MHPPO_* */
    int32_t n_envs;       /* N: envs on this handle (this rank's shard) */
    int32_t nb_car, nb_ped, nb_lines;
    int32_t max_episode;  /* 80 in every reference driver */
    int32_t sin_model;    /* simulation == "sin" */
    int32_t flags;        /* opt-in bug fixes, 0 = the reference's behaviour */
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
int mhppo_env_slots(const mhppo_env *env);   /* S: action slots per env (actions are [N, 2S]) */
int mhppo_env_reward_slots(const mhppo_env *env); /* reward/reward_light width: S, except 4cars2 = nb_car
                                                     (its PPO-driven followers earn none, :836-847) */

/* Checkpoint/resume (the reference saves only weights, :985-1001):
 * the env's whole device state — every field of every env plus its CPython MT19937
 * stream (624 words + cursor) — as one opaque blob of mhppo_env_state_bytes bytes.
 * export copies it to `dst`, import restores it from `src` (host or device memory,
 * stream-ordered); a blob is valid only for a handle created with the same config. */
int64_t mhppo_env_state_bytes(const mhppo_env *env);
int mhppo_env_export(const mhppo_env *env, void *dst, void *stream);
int mhppo_env_import(mhppo_env *env, const void *src, void *stream);

/* Replaces Crosswalk_*.reset() (Env_hybrid_multi_coop.py:838-893; 4cars :850-911;
 * scalable :884-946).  obs: float32 [N, obs_dim] or NULL. */
int mhppo_env_reset(mhppo_env *env, float *obs, void *stream);

/* Replaces Env_rollout.choix_test (Coop-MH-PPO-scalable.py:629-633) + env.get_state(), the
 * scripted scenario evaluate(n, choix=True) plays after every reset (:170-172): cross 3,
 * pedestrians rebuilt with pedestrian 0 crossing from (0, -1) at 1.25 m/s, cars 0/1 at -45 /
 * -22 m on lanes 0 / 1.  Scalable env only (MHPPO_EINVAL otherwise).  obs: float32
 * [N, obs_dim] or NULL. */
int mhppo_env_choix_test(mhppo_env *env, float *obs, void *stream);

/* Replaces Crosswalk_*.step(actions) (Env_hybrid_multi_coop.py:745-832; 4cars :783-844;
 * scalable :789-878).  actions: float64 [N, 2S] = [acc_0..acc_{S-1}, light_0..light_{S-1}];
 * obs float32 [N, obs_dim] (nullable); rewards, reward_light float64 [N, S];
 * done uint8 [N]. */
int mhppo_env_step(mhppo_env *env, const double *actions, float *obs, double *rewards,
                   double *reward_light, uint8_t *done, void *stream);

/* Read back the per-env scalar/attribute view the reference drivers touch
 * (env.cross, ped_traffic, car_traffic, cars[i].exist, pedestrian[j].waiting_time,
 * internal flags): out float64 [N, mhppo_env_state_dim() = 21P + 8 car slots + 4], laid out
 * [per ped 20][per car slot 8][cross, time, ped_traffic, car_traffic][per ped exist]. */
int mhppo_env_state_dim(const mhppo_env *env);
int mhppo_env_get_state(mhppo_env *env, double *out, void *stream);
/* Per-env event counters since the env's last reset (SURVEY §5 Metrics): the reference's only
 * run-time diagnostics are five prints inside pedestrian.detection; each one the reference would
 * print increments the env's counter instead (no device printf).  out uint32 [N, MHPPO_EV_N]. */
#define MHPPO_EV_ACCIDENT 0  /* "Accident! : "                scalable :186, 4cars :293, coop :185 */
#define MHPPO_EV_POSSIBLE 1  /* "Possible accident! "         scalable :200, 4cars :307, coop :199 */
#define MHPPO_EV_SMALL 2     /* "Small mistake - priority ? " scalable :222, 4cars :320, coop :221 */
#define MHPPO_EV_NOTWAIT 3   /* "Pedestrian is not waiting "  scalable :227, 4cars :325, coop :226
                                (once per pedestrian; naif :224 every time) */
#define MHPPO_EV_GREEN 4     /* "Mauvais signal vert "        scalable :236, 4cars :334, coop :235 */
#define MHPPO_EV_N 5
int mhppo_env_events(mhppo_env *env, uint32_t *out, void *stream);
/* RNG cursor: mt uint32 [N, 624], mti int32 [N] (device). */
int mhppo_env_get_rng(mhppo_env *env, uint32_t *mt, int32_t *mti, void *stream);

/* ---- rollout collector (Env_rollout.iterations_rand, Coop-MH-PPO-scalable.py:357-517) ---- */

/* One Model_PPO MLP (Coop-MH-PPO-scalable.py:42-93), in -> 32 -> 64 -> 32 -> out, ReLU,
 * packed contiguously in torch layout: W1[32][in] b1[32] W2[64][32] b2[64] W3[32][64]
 * b3[32] W4[out][32] b4[out] (float32, device).  kind: 0 linear (critic), 1 tanh*std+mean
 * (continuous actor), 2 pairwise softmax (choice actor). */
typedef struct mhppo_mlp {
    const float *packed;
    int32_t n_in, n_out, kind, reserved;
    float mean, std;
} mhppo_mlp;

/* Per-iteration rollout buffers for N envs, S slots, P peds, T steps (device, caller-owned).
 * Shapes: feat_d [N,S,P,dc] f32, probs_d [N,S,P,2] f32, a_d [N,S,P] i32, logp_d [N,S,P] f32,
 * closest [N,S] i32, feat_c [N,S,P,13] f32, out_c [N,S,P] f32, obs [N,obs_dim] f32 (current
 * observation), ep_min [N,S] f64, exist [N,S] u8, and the per-step records TIME-MAJOR (step t
 * of every env is one contiguous block): obs_c [T,N,S,13] f32, act [T,N,S] f32, logp [T,N,S]
 * f32, rew [T,N,S] f64.  The reference's episode-major batch order (:489-507) is a gather
 * of (env, slot) segments over t, see mhppo/rollout.py bucket_segments.
 * With P == 1, feat_c may point at obs_c + t*N*S*13 for step t (the selected feature row is
 * the only row, so the policy writes the record in place and sample_env copies nothing).
 * rows (int32 [N*S*P + 2]; required by the policy step, which returns MHPPO_EINVAL without it):
 * scratch for the head-sorted policy step — begin lists the (env, slot, ped) rows of the cross
 * head, then those of the wait head, counts last. */
typedef struct mhppo_rollout_bufs {
    float *feat_d, *probs_d, *logp_d;
    int32_t *a_d, *closest;
    float *feat_c, *out_c, *obs;
    float *obs_c, *act, *logp;
    double *rew, *ep_min;
    uint8_t *exist;
    int32_t *rows;
    int32_t T, flags;   /* flags: MHPPO_ROLLOUT_* */
    uint32_t *status;   /* optional device word, zeroed by mhppo_rollout_begin (flags of the current
                           episode only): bit 0 = a NaN choice probability, bit 1 = a NaN continuous
                           action mean was sampled; see mhppo_rollout_check */
    int32_t parts;      /* 0/1, or P > 1: the envs split in P contiguous parts (boundaries at multiples
                           of 64 envs) whose steps run as independent chains, e.g. on P streams
                           (mhppo_rollout_policy_part / _sample_env_part); rows then needs
                           N*S*P + 2 + 2 (parts + 1) entries */
    int32_t reserved;
    int32_t *rec_of;    /* optional [N*S + N + 1] (NULL: record index = segment index): the compact
                           record layout.  mhppo_rollout_begin fills it from exist: segment s = env*S
                           + slot gets record rec_of[s] = its rank among the existing segments, or -1,
                           and rec_of[N*S + e] = the existing segments before env e (e = 0 .. N);
                           every per-step record of segment s (obs_c row, act, logp, rew) is then
                           stored at record rec_of[s] of step t (obs_c[t][rec_of[s]], ...), and none
                           for rec_of[s] = -1, so the present segments' records are contiguous and
                           absent ones cost no stores (and share no cache line with present ones
                           for mhppo_bucket_scatter, whose pos / bucket are then per record).  With
                           one pedestrian (P == 1) feat_c must be obs_c[t] (the in-place record).
                           The scalable env only (the variant whose car slots can be absent):
                           mhppo_rollout_begin returns MHPPO_EINVAL for another. */
} mhppo_rollout_bufs;
/* mhppo_rollout_bufs.flags: run the policy step on the VALU reference kernels instead of the MFMA
 * kernel (bit-identical).  Those kernels are compiled into the test build only
 * (tests/lib/libmhppo_test.so, -DMHPPO_TEST_KERNELS); the shipped library returns MHPPO_EINVAL. */
#define MHPPO_ROLLOUT_VALU_POLICY 1

int mhppo_choice_dim(const mhppo_env *env);

/* Deterministic evaluation (Env_rollout.iterations :152-252, run by Algo_PPO.evaluate
 * :738-747).  Device buffers; per-step outputs are time-major [T][N][..]. */
typedef struct mhppo_eval_bufs {
    float *obs;       /* [N, obs_dim] current observation (in/out; mhppo_env_reset fills it) */
    int32_t *a_d;     /* [N, S, P] current choice (argmax of the choice actor) */
    uint8_t *trig;    /* [N] re-decision due at the next step */
    double *ep_min;   /* [N, S] episodic min of reward_light since the last decision */
    float *obs_hist;  /* [T, N, obs_dim] pre-step observations (batch_obs) */
    float *acts;      /* [T, N, S] continuous actions (batch_acts) */
    float *rews_c;    /* [T, N, S] step rewards (batch_rews_c) */
    float *rews_d;    /* [T, N, S] episodic reward at a save (batch_rews_d), rows with saved = 1 */
    float *waiting;   /* [T, N, P] pedestrians' waiting_time at a save, rows with saved = 1 */
    uint8_t *saved;   /* [T, N] a save happened after step t (re-decision or done) */
    int32_t T, reserved;
} mhppo_eval_bufs;

/* Step t of an evaluation episode in every env (t = 0 right after mhppo_env_reset):
 * choice argmax when a decision is due (t = 0 or the re-decision test fired), per car
 * a = min over pedestrians of the head's mean action (left-lane pedestrians: clamped
 * speed-limit tracking), capped by (10 - V)/dt; lights = 2 a_d[flat i] - 1; env step. */
int mhppo_eval_step(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                    const mhppo_mlp *actor_choice, int t, mhppo_eval_bufs *bufs, void *stream);

/* Episode start (:377-428): reset every env, write obs, choice features obs_car_ped_d
 * (:574-611) and closest pedestrian (:614-627), run the choice actor and draw
 * Categorical samples.  When `forced_a` (int32 [N,S,P]) is non-NULL the draws are
 * replayed from it (parity mode); otherwise u (float32 [N,S,P] uniforms) picks
 * a = (u >= p0/(p0+p1)). */
int mhppo_rollout_begin(mhppo_env *env, const mhppo_mlp *actor_choice, const float *u,
                        const int32_t *forced_a, mhppo_rollout_bufs *bufs, void *stream);

/* Step t (:430-461): obs_car_ped features for every (slot, ped) (:541-572), cross/wait
 * actor chosen by action_d (:440-445), min over pedestrians, MVN(loc, 0.5) sample from
 * eps (float32 [N,S] standard normals), env.step, episodic min of reward_light (:461). */
int mhppo_rollout_step(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                       const float *eps, int t, mhppo_rollout_bufs *bufs, void *stream);
/* The two launches of mhppo_rollout_step, separately (for per-kernel timing):
 * policy = features + actor forward per (env, slot, ped); sample_env = per-env
 * min/sample/buffers + env.step + episodic min. */
int mhppo_rollout_policy(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                         mhppo_rollout_bufs *bufs, void *stream);
int mhppo_rollout_sample_env(mhppo_env *env, const float *eps, int t, mhppo_rollout_bufs *bufs, void *stream);
/* The same two launches for part `part` of bufs->parts only (its envs' rows / its envs): the parts'
 * step chains are independent, so on separate streams one part's policy MFMA work fills the CUs
 * another part's latency-bound env step leaves idle.  Results are those of the whole-N calls. */
int mhppo_rollout_policy_part(mhppo_env *env, const mhppo_mlp *actor_cross, const mhppo_mlp *actor_wait,
                              mhppo_rollout_bufs *bufs, int part, void *stream);
int mhppo_rollout_sample_env_part(mhppo_env *env, const float *eps, int t, mhppo_rollout_bufs *bufs, int part,
                                  void *stream);

/* Measurement (bench.py): the next `n` env-step launches (mhppo_rollout_sample_env) of the
 * calling thread on the device current at this call carry HIP events attached to their dispatch
 * packets (hipExtLaunchKernelGGL start/stop events: the kernel's execution, not the queue's
 * event-packet gaps);
 * mhppo_kernel_timing_end synchronises them and returns the summed milliseconds and the
 * number of timed launches.  No reference counterpart. */
int mhppo_kernel_timing_begin(int n);
int mhppo_kernel_timing_end(double *ms_total, int *launches);
/* As mhppo_kernel_timing_end, but writes each timed launch's milliseconds, in launch order, to
 * ms_each[0 .. min(cap, launches)) (the per-step durations of a rollout: tools/env_steps.py). */
int mhppo_kernel_timing_end_each(float *ms_each, int cap, int *launches);

/* Status of the rollout launches queued on `stream` so far: synchronises the stream, reads
 * and clears bufs->status, and returns MHPPO_ENAN when a NaN policy output was drawn from
 * (Categorical(probs) at the episode start, :409; MultivariateNormal(loc) per step, :451:
 * where the reference's torch.distributions raise ValueError), else MHPPO_OK. */
int mhppo_rollout_check(mhppo_rollout_bufs *bufs, void *stream);

/* Philox-4x32-10 noise (perf mode): out[i] for counter (offset + i) under key `seed`. */
int mhppo_philox_normal(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream);
int mhppo_philox_uniform(uint64_t seed, uint64_t offset, float *out, int64_t n, void *stream);
/* rows x cols normals, out[r * cols + c] from counter (offset + r * stride + c): a rollout's
 * per-step noise in one launch (the same values as `rows` calls of mhppo_philox_normal). */
int mhppo_philox_normal_2d(uint64_t seed, uint64_t offset, uint64_t stride, float *out, int64_t rows,
                           int64_t cols, void *stream);

/* ---- returns / advantage / PPO losses (futur_rewards :658-684, train_model_c/_d :778-851) ---- */

/* The rollout policy heads' float transcendentals (csrc/libm_glibc.h: glibc 2.35's tanhf, expm1f,
 * expf restated so the device returns glibc's bits — the functions the reference's batch-1 CPU
 * forward calls, Model_PPO :81-89) evaluated on the float bit patterns first .. first + n - 1
 * (mod 2^32): the device side of their exhaustive pin (tests/test_libm_gpu.py).
 * fn: 0 tanhf, 1 expm1f, 2 expf.  out float [n]. */
int mhppo_libm_eval(int fn, uint64_t first, int64_t n, float *out, void *stream);

/* Segmented reverse discounted scan, G_t = r_t + gamma*G_{t+1} in float64, one segment of
 * T per row: rew float64 [B,T] -> ret float32 [B,T]. */
int mhppo_returns_scan(const double *rew, float *ret, int64_t B, int32_t T, double gamma, void *stream);
/* The same scan over time-major records: rew float64 [T,B] -> ret float32 [T,B] (segment b
 * is column b; the rollout's rew buffer is [T, N*S]). */
int mhppo_returns_scan_tm(const double *rew, float *ret, int64_t B, int32_t T, double gamma, void *stream);

/* Segment-major buckets (bucket_segments; replaces the per-episode concatenation of
 * Coop-MH-PPO-scalable.py:489-507).  Segment s < NS (= N*S records per step) with pos[s] >= 0
 * belongs to bucket bucket[s] (0 or 1) at position pos[s]: its time-major records t < T
 * (obs [.., 13] float32, act / logp / ret float32, rew float64; record t*NS + s) go to rows
 * pos[s]*T + t of dst[bucket[s]] (caller-sized: count of segments x T rows). */
typedef struct {
  float *obs, *act, *logp, *ret;
  double *rew;
} mhppo_bucket_dst;
int mhppo_bucket_scatter(const int64_t *pos, const int8_t *bucket, int64_t NS, int32_t T, const float *obs_tm,
                         const float *act_tm, const float *logp_tm, const float *ret_tm, const double *rew_tm,
                         const mhppo_bucket_dst *dst, void *stream);

/* Advantage statistics of A = G - V over M rows: stats float64 [2] += (sum A, sum A^2)
 * (caller zeroes it; partial sums all-reduce across ranks).  Normalisation
 * A' = (A - mean) / (std_unbiased + 1e-10) with mean/std from (stats, M_global). */
int mhppo_adv_stats(const float *ret, const float *value, int64_t M, double *stats, void *stream);
int mhppo_adv_normalize(const float *ret, const float *value, int64_t M, const double *stats,
                        double m_global, float *adv, void *stream);

/* Continuous PPO clip surrogate (:795-806): logp = MVN(mu, 0.5).log_prob(act) (float32),
 * ratio = exp(logp - logp_old) in float64, L = mean(-min(r A, clamp(r, .8, 1.2) A)).
 * dmu float32 [M] = dL/dmu with the 1/M_global factor (inv_m); loss float64 [1] += sum. */
int mhppo_ppo_cont_fwd_bwd(const float *mu, const float *act, const float *logp_old,
                           const float *adv, int64_t M, double inv_m, float *dmu,
                           double *loss, void *stream);

/* Choice PPO surrogate over the reference's M x M broadcast (:834-842) in its exact O(M)
 * form L = (1/M^2) sum_j [n0 f(r_j0, A_j) + n1 f(r_j1, A_j)], f(r,A) = -min(rA, clip(r)A),
 * r_jk = exp(log clamp(p_jk/(p_j0+p_j1)) - logp_old_j).  probs float32 [M,2] (softmax
 * outputs); counts float64 [2] = (n0, n1) global.  dprobs float32 [M,2] = dL/dprobs. */
int mhppo_ppo_choice_fwd_bwd(const float *probs, const float *logp_old, const float *adv,
                             int64_t M, const double *counts, double inv_m2, float *dprobs,
                             double *loss, void *stream);

/* Fused training pass of one Model_PPO head (n_in -> 32 -> 64 -> 32 -> n_out) on f32 MFMA:
 * forward + loss gradient + backward + weight gradient over M rows, replacing the torch
 * GEMMs/autograd of one epoch of train_model_c (:778-815) / train_model_d (:818-851).
 * kind 0 = critic (n_in <= 64, n_out 1): writes value[M]; grad = dMSE/dW;
 *          sums[0..2] += (sum (V-G)^2, sum A, sum A^2) with A = G - V.
 * kind 1 = continuous actor (n_in 13, n_out 1, tanh*out_std + out_mean): reads value[M],
 *          act, logp_old and the GLOBAL (sum A, sum A^2) in stats[0..1];
 *          grad = d(clip surrogate)/dW, sums[0] += sum of surrogate terms.
 * kind 2 = choice actor (n_in <= 64, n_out 2, pairwise softmax): reads value, logp_old,
 *          stats and the GLOBAL action counts counts[0..1] (float64);
 *          grad = d(O(M) Categorical surrogate / M_global^2)/dW, sums[0] += its sum.
 *          counts == NULL selects the opt-in per-row loss: act[M] (0/1 as
 *          float) is read and each row contributes its own action's surrogate / M_global.
 * grad: packed torch layout W1 b1 W2 b2 W3 b3 W4 b4 (32 n_in + 4224 + 33 n_out floats).
 * m_global = the global row count (data parallel: all ranks' rows).
 * Heads with n_in <= 54 run on bf16 MFMA with every f32 operand split exactly into three
 * bf16 parts (products to f32 accuracy; X must then be 16-byte aligned); kind |
 * MHPPO_TRAIN_EXACT_F32 selects the f32-MFMA kernel, whose sums are k-ordered fmaf chains
 * (wider heads always run on it).
 * Per-device, per-stream workspace (up to 4 streams per device): calls on one stream are ordered by
 * it, calls on different streams may run concurrently (MHPPO_EINVAL for a fifth stream). */
#define MHPPO_TRAIN_EXACT_F32 0x100
int mhppo_mlp_train(int kind, int n_in, const float *packed, const float *X, int64_t M, const float *ret,
                    float *value, const float *act, const float *logp_old, const double *stats,
                    const double *counts, double m_global, float out_mean, float out_std, float *grad,
                    double *sums, void *stream);

/* One epoch step of a continuous head run as a pipeline (Algo_PPO.train_model_c :778-815, epochs
 * e and e + 1 overlapped): the ACTOR pass of epoch e (kind 1 of mhppo_mlp_train: advantage
 * A = ret - value normalised with `stats`, the critic pass e's (sum A, sum A^2) over m_global
 * rows) and the CRITIC pass of epoch e + 1 (kind 0, with the critic's weights after its Adam step
 * e) in ONE launch over the same rows: one input load per tile for both nets.  `value` holds V_e
 * on entry and V_{e+1} on return (each row is read before it is overwritten).  grad_* / sums_*
 * as mhppo_mlp_train's (sums_actor += (sum surrogate, 0, 0), sums_critic += (sum (V-G)^2,
 * sum A, sum A^2) of epoch e + 1).  bf16x3 split-precision kernel only (13 inputs, 1 output). */
int mhppo_mlp_train_pair(const float *packed_actor, const float *packed_critic, const float *X, int64_t M,
                         const float *ret, float *value, const float *act, const float *logp_old,
                         const double *stats, double m_global, float out_mean, float out_std,
                         float *grad_actor, double *sums_actor, float *grad_critic, double *sums_critic,
                         void *stream);

/* Critic MSE (:808-809): loss += sum (V-G)^2, dV = 2 (V-G) * inv_m. */
int mhppo_mse_fwd_bwd(const float *value, const float *ret, int64_t M, double inv_m, float *dv,
                      double *loss, void *stream);

const char *mhppo_last_error(void);
const char *mhppo_version(void);

#ifdef __cplusplus
}
#endif
#endif
