/* ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).
 *
 * Many-env driver of the C restatement: N independent envs (env e on its own
 * CPython stream seeded seed_base + e, as the reference runs one env on the
 * module-global stream, tests/golden/gen/make_env_golden.py), stepped with
 * OpenMP over envs.  Nothing here adds semantics: every call is the per-env
 * oracle_env_* / oracle_rollout_episode restatement (env_oracle.c,
 * rollout_oracle.c), run for each env on whichever host thread picks it up.
 * Used for the full-scale GPU-vs-oracle parity test and the all-core CPU
 * baseline ("the C restatement with OpenMP over envs").
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct OEnv OEnv;
OEnv *oracle_env_create(int variant, int nb_car, int nb_ped, int nb_lines, double dt, int max_episode,
                        int sin_model, const double *car_b, const double *ped_b, const double *cross_b);
void oracle_env_destroy(OEnv *e);
void oracle_env_set_flags(OEnv *e, int flags);
void oracle_env_seed(OEnv *e, uint64_t seed);
void oracle_env_get_rng(const OEnv *e, uint32_t *mt, int32_t *mti);
int oracle_env_obs_dim(const OEnv *e);
void oracle_env_reset(OEnv *e, float *obs);
int oracle_env_step(OEnv *e, const double *actions, float *obs, double *rewards, double *reward_light);
int oracle_env_dump(const OEnv *e, double *out);
void oracle_env_events(const OEnv *e, uint32_t *out);
int oracle_choice_dim(int variant, int S);
int oracle_rollout_episode(OEnv *e, int variant, int S, int P, int T, const float *w_cross, const float *w_wait,
                           const float *w_choice, float act_mean, float act_std, const int32_t *forced_a,
                           const float *u, const float *eps, float *o_feat_d, float *o_probs, int32_t *o_a_d,
                           float *o_logp_d, int32_t *o_closest, uint8_t *o_exist, float *o_obs_c, float *o_act,
                           float *o_logp, double *o_rew, double *o_ep_min);

typedef struct OBatch {
    int n, variant, S, P, rs, od, dk;
    OEnv **e;
} OBatch;

int oracle_set_threads(int n) {
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
}

/* rs = reward width of one env (S; 4cars2: nb_car); dk = oracle_env_dump width. */
OBatch *oracle_batch_create(int variant, int n, int nb_car, int nb_ped, int nb_lines, double dt, int max_episode,
                            int sin_model, const double *car_b, const double *ped_b, const double *cross_b,
                            uint64_t seed_base, int flags) {
    OBatch *b = (OBatch *)calloc(1, sizeof(OBatch));
    b->n = n;
    b->variant = variant;
    b->P = nb_ped;
    b->e = (OEnv **)calloc((size_t)n, sizeof(OEnv *));
    int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
    for (int i = 0; i < n; i++) {
        b->e[i] = oracle_env_create(variant, nb_car, nb_ped, nb_lines, dt, max_episode, sin_model, car_b, ped_b,
                                    cross_b);
        if (!b->e[i]) {
            bad = 1;
            continue;
        }
        if (flags) oracle_env_set_flags(b->e[i], flags);
        oracle_env_seed(b->e[i], seed_base + (uint64_t)i);
    }
    if (bad || n < 1) {
        for (int i = 0; i < n; i++)
            if (b->e[i]) oracle_env_destroy(b->e[i]);
        free(b->e);
        free(b);
        return NULL;
    }
    b->S = variant == 2 ? 2 * nb_lines : nb_car;
    b->rs = b->S;
    b->od = oracle_env_obs_dim(b->e[0]);
    double tmp[4096];
    b->dk = oracle_env_dump(b->e[0], tmp);
    return b;
}

void oracle_batch_destroy(OBatch *b) {
    if (!b) return;
    for (int i = 0; i < b->n; i++) oracle_env_destroy(b->e[i]);
    free(b->e);
    free(b);
}

int oracle_batch_obs_dim(const OBatch *b) { return b->od; }
int oracle_batch_dump_dim(const OBatch *b) { return b->dk; }

void oracle_batch_reset(OBatch *b, float *obs) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < b->n; i++) oracle_env_reset(b->e[i], obs + (size_t)i * b->od);
}

/* actions float64 [n, 2S]; obs f32 [n, od]; rew / rl f64 [n, rs]; done u8 [n];
 * dump f64 [n, dk] and mti i32 [n] nullable (state after the step). */
void oracle_batch_step(OBatch *b, const double *actions, float *obs, double *rew, double *rl, uint8_t *done,
                       double *dump, int32_t *mti) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < b->n; i++) {
        done[i] = (uint8_t)oracle_env_step(b->e[i], actions + (size_t)i * 2 * b->S, obs + (size_t)i * b->od,
                                           rew + (size_t)i * b->rs, rl + (size_t)i * b->rs);
        if (dump) oracle_env_dump(b->e[i], dump + (size_t)i * b->dk);
        if (mti) {
            uint32_t mt[624];
            oracle_env_get_rng(b->e[i], mt, mti + i);
        }
    }
}

/* dump f64 [n, dk]: every env's oracle_env_dump (state as it stands, e.g. after a rollout) */
void oracle_batch_dump(const OBatch *b, double *dump) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < b->n; i++) oracle_env_dump(b->e[i], dump + (size_t)i * b->dk);
}

/* events u32 [n, 5]: every env's detection print counts since its last reset */
void oracle_batch_events(const OBatch *b, uint32_t *events) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < b->n; i++) oracle_env_events(b->e[i], events + (size_t)i * 5);
}

/* mt u32 [n, 624], mti i32 [n] */
void oracle_batch_get_rng(const OBatch *b, uint32_t *mt, int32_t *mti) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < b->n; i++) oracle_env_get_rng(b->e[i], mt + (size_t)i * 624, mti + i);
}

/* One Env_rollout.iterations_rand episode in every env (oracle_rollout_episode per env).
 * Per-env inputs: forced_a i32 [n,S,P] (nullable) or u f32 [n,S,P]; eps f32 [n,T,S].
 * Per-env outputs laid out like oracle/__init__.py rollout(): feat_d [n,S,P,dc],
 * probs [n,S,P,2], a_d/logp_d [n,S,P], closest [n,S], exist [n,S], obs_c [n,S,T,13],
 * act/logp [n,S,T] f32, rew [n,S,T] f64, ep_min [n,S] f64. */
void oracle_batch_rollout(OBatch *b, int T, const float *w_cross, const float *w_wait, const float *w_choice,
                          float act_mean, float act_std, const int32_t *forced_a, const float *u, const float *eps,
                          float *feat_d, float *probs, int32_t *a_d, float *logp_d, int32_t *closest,
                          uint8_t *exist, float *obs_c, float *act, float *logp, double *rew, double *ep_min) {
    const int S = b->S, P = b->P, dc = oracle_choice_dim(b->variant, S);
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < b->n; i++) {
        const size_t sp = (size_t)i * S * P, st = (size_t)i * S * T;
        oracle_rollout_episode(b->e[i], b->variant, S, P, T, w_cross, w_wait, w_choice, act_mean, act_std,
                               forced_a ? forced_a + sp : NULL, u + sp, eps + st, feat_d + sp * dc,
                               probs + 2 * sp, a_d + sp, logp_d + sp, closest + (size_t)i * S,
                               exist + (size_t)i * S, obs_c + st * 13, act + st, logp + st, rew + st,
                               ep_min + (size_t)i * S);
    }
}

/* glibc's own tanhf / expm1f / expf (fn 0 / 1 / 2) on the float bit patterns first .. first + n - 1
 * (mod 2^32): the reference values the device restatements (mh-ppo_amd/csrc/libm_glibc.h) are
 * compared with bit for bit (tests/test_libm_gpu.py). */
void oracle_libm_eval(int fn, uint64_t first, int64_t n, float *out) {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; i++) {
        const uint32_t u = (uint32_t)(first + (uint64_t)i);
        float x;
        memcpy(&x, &u, 4);
        out[i] = fn == 0 ? tanhf(x) : (fn == 1 ? expm1f(x) : expf(x));
    }
}
