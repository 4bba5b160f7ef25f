/* ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).
 *
 * CPU restatement of one episode of Env_rollout.iterations_rand
 * (Coop-MH-PPO-scalable.py:357-517, scalable driver; Coop-MH-PPO.ipynb cell 0,
 * coop driver — also used by MH-PPO.ipynb for naif and as the build-defined
 * 4cars featurization), driving the C env oracle (env_oracle.c):
 *   featurizers  obs_car_ped :541-572, obs_car_ped_d :574-611, closest_ped_d :614-627,
 *                is_in_cross :526-530, leave_cross :532-539 — float32 arithmetic on
 *                the float32 observation, as numpy float32 scalars compute it
 *   choice       Categorical(actor_choice(obs_d)) at t = 0 (:403-428)
 *   continuous   head by action_d[i*P+p] (:440-445), torch.min over pedestrians,
 *                `==` keeps the last minimiser's features (:448-450),
 *                MVN(loc, 0.5) sample/log_prob (:451-453)
 *   env          env.step([acc..., light...]) (:460), episodic min (:461)
 * Draws: the Categorical draw is either replayed (forced) or a = (u >= p0/(p0+p1));
 * the MVN standard normals come in as eps (recorded or Philox).
 * Model_PPO forward (:70-93): each output is a float32 fmaf chain over inputs in
 * ascending order from 0, plus bias, ReLU; tanh*std+mean; pairwise softmax.
 *
 * oracle_eval_episode restates one episode of the deterministic evaluation
 * Env_rollout.iterations (Coop-MH-PPO-scalable.py:152-252; Coop-MH-PPO.ipynb /
 * MH-PPO.ipynb same body), the routine Algo_PPO.evaluate (:738-747) runs.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct OEnv OEnv;
int oracle_env_obs_dim(const OEnv *e);
void oracle_env_reset(OEnv *e, float *obs);
int oracle_env_step(OEnv *e, const double *actions, float *obs, double *rewards, double *reward_light);
int oracle_env_dump(const OEnv *e, double *out);
int oracle_env_choix_test(OEnv *e, float *obs);

#define NF 13

typedef struct {
    int S, P, cw, env_off, ped_off, lines_idx, scalable;
} Lay;

static Lay layout(int variant, int S, int P) {
    Lay L;
    L.S = S; L.P = P;
    L.scalable = variant == 2;
    L.cw = L.scalable ? 7 : 6;
    L.env_off = L.cw * S + (variant == 1 ? 6 * S : 0);
    L.ped_off = L.env_off + (L.scalable ? 4 : 3);
    L.lines_idx = L.scalable ? 3 : 2;
    return L;
}

int oracle_choice_dim(int variant, int S) { return variant == 2 ? 2 + 6 * (S - 1) + 10 : 2 + 5 * (S - 1) + 10; }

static void is_in_cross(float car_line, float pos, float dir, float cl, float lines, float *crossing, float *dstart) {
    float cross = (cl * 2.0f) / lines;
    float ls = (-cl) + cross * car_line;
    float le = (-cl) + cross * (car_line + 1.0f);
    *dstart = (pos - ls) * (float)(dir > 0) + (le - pos) * (float)(dir < 0);
    *crossing = (pos > ls && pos < le) ? 1.0f : 0.0f;
}

static void leave_cross(float car_line, float pos, float dir, float cl, float lines, float *endc, float *dend) {
    float cross = (cl * 2.0f) / lines;
    float ls = (-cl) + cross * car_line;
    float le = (-cl) + cross * (car_line + 1.0f);
    if (dir == -1.0f) { *endc = (pos < ls) ? 1.0f : 0.0f; *dend = ls - pos; }
    else { *endc = (pos > le) ? 1.0f : 0.0f; *dend = pos - le; }
}

static float feat_c(const float *o, const Lay *L, int i, int p, float *f) {
    const float *car = o + i * L->cw, *ped = o + L->ped_off + p * 9, *env = o + L->env_off;
    float cl = env[0], lines = env[L->lines_idx];
    float crossing, ds, endc, de;
    is_in_cross(car[5], ped[3], ped[8], cl, lines, &crossing, &ds);
    leave_cross(car[5], ped[3], ped[8], cl, lines, &endc, &de);
    float d = ped[2] - car[3];
    float den = car[1] - ped[0];
    if (0.01f > den) den = 0.01f;
    float q = d / den;
    float t = (q < 10.0f) ? q : 10.0f;
    float ttc = (ped[2] > car[3]) ? t : 10.0f;
    float v[NF] = {car[1], car[2], ped[1], (ped[2] > car[3]) ? 1.0f : 0.0f, d, ped[4], crossing, endc, ds, de, ttc,
                   cl, lines};
    memcpy(f, v, sizeof(v));
    return ped[7];
}

static void feat_d(const float *o, const Lay *L, int i, int p, float *f) {
    const float *car = o + i * L->cw, *ped = o + L->ped_off + p * 9, *env = o + L->env_off;
    int k = 0;
    f[k++] = car[1];
    f[k++] = car[2];
    for (int j = 0; j < L->S; j++) {
        if (j == i) continue;
        const float *c2 = o + j * L->cw;
        f[k++] = c2[1];
        f[k++] = (ped[2] > c2[3]) ? 1.0f : 0.0f;
        f[k++] = ped[2] - c2[3];
        f[k++] = c2[4];
        f[k++] = c2[5] - car[5];
        if (L->scalable) f[k++] = car[6];
    }
    float cl = env[0], lines = env[L->lines_idx];
    float crossing, ds, endc, de;
    is_in_cross(car[5], ped[3], ped[8], cl, lines, &crossing, &ds);
    leave_cross(car[5], ped[3], ped[8], cl, lines, &endc, &de);
    f[k++] = ped[1];
    f[k++] = (ped[2] > car[3]) ? 1.0f : 0.0f;
    f[k++] = ped[2] - car[3];
    f[k++] = ped[4];
    f[k++] = crossing;
    f[k++] = endc;
    f[k++] = ds;
    f[k++] = de;
    f[k++] = cl;
    f[k++] = lines;
}

static int closest(const float *o, const Lay *L, int i) {
    const float *car = o + i * L->cw;
    int mp = 0;
    if (L->scalable) {
        float md = 1000000.f;
        for (int p = 0; p < L->P; p++) {
            const float *ped = o + L->ped_off + p * 9;
            float d = ped[2] - car[3];
            if (d < md && ped[7] != 0.0f) { md = d; mp = p; }
        }
    } else {
        float md = o[L->ped_off + 2] - car[3];
        for (int p = 0; p < L->P; p++) {
            const float *ped = o + L->ped_off + p * 9;
            float d = ped[2] - car[3];
            if (d < md) { md = d; mp = p; }
        }
    }
    return mp;
}

static float relu(float x) { return (x < 0.0f) ? 0.0f : x; }

/* Model_PPO forward, packed torch layout W1 b1 W2 b2 W3 b3 W4 b4 */
void oracle_mlp_forward(const float *W, int n_in, int n_out, const float *x, float *out) {
    const float *w1 = W, *b1 = w1 + 32 * n_in, *w2 = b1 + 32, *b2 = w2 + 64 * 32, *w3 = b2 + 64, *b3 = w3 + 32 * 64,
                *w4 = b3 + 32, *b4 = w4 + n_out * 32;
    float h1[32], h2[64], h3[32];
    for (int o = 0; o < 32; o++) {
        float acc = 0.0f;
        for (int k = 0; k < n_in; k++) acc = fmaf(w1[o * n_in + k], x[k], acc);
        h1[o] = relu(acc + b1[o]);
    }
    for (int o = 0; o < 64; o++) {
        float acc = 0.0f;
        for (int k = 0; k < 32; k++) acc = fmaf(w2[o * 32 + k], h1[k], acc);
        h2[o] = relu(acc + b2[o]);
    }
    for (int o = 0; o < 32; o++) {
        float acc = 0.0f;
        for (int k = 0; k < 64; k++) acc = fmaf(w3[o * 64 + k], h2[k], acc);
        h3[o] = relu(acc + b3[o]);
    }
    for (int j = 0; j < n_out; j++) {
        float acc = 0.0f;
        for (int k = 0; k < 32; k++) acc = fmaf(w4[j * 32 + k], h3[k], acc);
        out[j] = acc + b4[j];
    }
}

static const float MVN_L = 0x1.6a09e6p-1f, MVN_INV_L = 0x1.6a09e6p+0f, MVN_LOG2PI = 0x1.d67f1cp+0f,
                   MVN_HLD = -0x1.62e432p-2f;

static float tmin(float a, float b) {
    if (a != a) return a;
    if (b != b) return b;
    return (b < a) ? b : a;
}

/* One episode of one env.  Returns the number of steps played. */
int oracle_rollout_episode(OEnv *e, int variant, int S, int P, int T, const float *w_cross, const float *w_wait,
                           const float *w_choice, float act_mean, float act_std, const int32_t *forced_a,
                           const float *u, const float *eps, float *o_feat_d, float *o_probs, int32_t *o_a_d,
                           float *o_logp_d, int32_t *o_closest, uint8_t *o_exist, float *o_obs_c, float *o_act,
                           float *o_logp, double *o_rew, double *o_ep_min) {
    Lay L = layout(variant, S, P);
    int dc = oracle_choice_dim(variant, S);
    float obs[1024];
    double actions[64], rew[32], rl[32];
    oracle_env_reset(e, obs);
    for (int i = 0; i < S; i++) {
        for (int p = 0; p < P; p++) {
            int r = i * P + p;
            float *f = o_feat_d + (size_t)r * dc;
            feat_d(obs, &L, i, p, f);
            float lg[2];
            oracle_mlp_forward(w_choice, dc, 2, f, lg);
            float mx = lg[0] > lg[1] ? lg[0] : lg[1];
            float e0 = expf(lg[0] - mx), e1 = expf(lg[1] - mx);
            float s = e0 + e1;
            float p0 = e0 / s, p1 = e1 / s;
            o_probs[2 * r] = p0;
            o_probs[2 * r + 1] = p1;
            float sum = p0 + p1, n0 = p0 / sum, n1 = p1 / sum;
            int a = forced_a ? forced_a[r] : (u[r] >= n0 ? 1 : 0);
            const float ep = 1.1920928955078125e-07f, hi = 1.0f - 1.1920928955078125e-07f;
            float pn = a ? n1 : n0;
            pn = pn < ep ? ep : (pn > hi ? hi : pn);
            o_a_d[r] = a;
            o_logp_d[r] = logf(pn);
        }
        o_closest[i] = closest(obs, &L, i);
        o_exist[i] = L.scalable ? (uint8_t)(obs[i * L.cw + 6] != 0.0f) : 1;
        o_ep_min[i] = 0.0;
    }
    int t;
    for (t = 0; t < T; t++) {
        for (int i = 0; i < S; i++) {
            float loc = 2.0f;
            float fsel[NF], f[NF];
            feat_c(obs, &L, i, 0, fsel);
            for (int p = 0; p < P; p++) {
                float ex = feat_c(obs, &L, i, p, f);
                if (L.scalable && ex == 0.0f) continue;
                int wait = (2 * o_a_d[i * P + p] - 1) > 0;
                float out;
                oracle_mlp_forward(wait ? w_wait : w_cross, NF, 1, f, &out);
                float tt = tanhf(out) * act_std;
                out = tt + act_mean;
                loc = tmin(loc, out);
                if (out == loc) memcpy(fsel, f, sizeof(f));
            }
            float a = loc + MVN_L * eps[t * S + i];
            float x = (a - loc) * MVN_INV_L;
            size_t bt = (size_t)i * T + t;
            o_act[bt] = a;
            o_logp[bt] = (-0.5f * (MVN_LOG2PI + x * x)) - MVN_HLD;
            memcpy(o_obs_c + bt * NF, fsel, sizeof(fsel));
            actions[i] = (double)a;
            actions[S + i] = (double)(2 * o_a_d[i * P + o_closest[i]] - 1);
        }
        int done = oracle_env_step(e, actions, obs, rew, rl);
        for (int i = 0; i < S; i++) {
            o_rew[(size_t)i * T + t] = rew[i];
            double m = o_ep_min[i], xx = rl[i];
            o_ep_min[i] = (m != m) ? m : ((xx != xx) ? xx : (xx < m ? xx : m));
        }
        if (done) { t++; break; }
    }
    return t;
}

/* One episode of Env_rollout.iterations (:152-252), deterministic:
 *  - at need_new_d (episode start; then whenever the re-decision test fires):
 *    episodic_reward = 0, choice a_d[i*P+p] = argmax(actor_choice(obs_d)) (torch.argmax:
 *    first maximum, :180-186)
 *  - per car i: a = car_b[1,0]; per ped p (every ped, no exist gate): if obs_car_ped[7]
 *    (the pedestrian has left the car's lane): cand = max(min((10 - V)/dt, car_b[1,0]),
 *    car_b[0,0]) else the cross (action_d <= 0) / wait actor's mean output; a =
 *    min(a, cand); a = min(a, (10 - V)/dt) — Python min keeps the first on ties (:193-207)
 *  - lights: action_d_light = 2*action_all_d - 1, i.e. entry i of the FLAT (car, ped)
 *    choice array, not the closest pedestrian's (:188, :210; the env reads entries S..2S-1)
 *  - env.step; rews_c = reward; episodic_reward = np.minimum(.., reward_light) (:212-216)
 *  - re-decision test (:218-220): scalable driver state["env"][1] != nb_ped; coop and
 *    naif drivers state["env"][1] != its previous value; a save (rews_d = episodic_reward,
 *    every pedestrian's waiting_time) happens when it fires or at done (:224-229).
 * Outputs per step t: obs (the pre-step observation), acts [S] and rews_c [S] as
 * float32 (torch.tensor(..., dtype=float)), saved flag, rews_d [S] and waiting [P]
 * when saved.  Returns the number of steps played. */
int oracle_eval_episode(OEnv *e, int variant, int S, int P, int T, const float *w_cross, const float *w_wait,
                        const float *w_choice, float act_mean, float act_std, double acc_lo, double acc_hi,
                        double dt, float *o_obs, float *o_acts, float *o_rews_c, uint8_t *o_saved, float *o_rews_d,
                        float *o_waiting, int choix) {
    Lay L = layout(variant, S, P);
    const int dc = oracle_choice_dim(variant, S), od = oracle_env_obs_dim(e);
    float obs[1024];
    double actions[64], rew[32], rl[32], epr[32], dump[4096];
    int a_d[256];
    oracle_env_reset(e, obs);
    if (choix && oracle_env_choix_test(e, obs) != 0) return -1;  /* iterations(choix=True) :170-172 */
    int need = 1, t;
    for (t = 0; t < T; t++) {
        if (need) {
            for (int i = 0; i < S; i++) epr[i] = 0.0;
            for (int i = 0; i < S; i++)
                for (int p = 0; p < P; p++) {
                    float f[256], lg[2];
                    feat_d(obs, &L, i, p, f);
                    oracle_mlp_forward(w_choice, dc, 2, f, lg);
                    float mx = lg[0] > lg[1] ? lg[0] : lg[1];
                    float e0 = expf(lg[0] - mx), e1 = expf(lg[1] - mx);
                    float sm = e0 + e1;
                    a_d[i * P + p] = (e1 / sm > e0 / sm) ? 1 : 0;
                }
        }
        need = 0;
        memcpy(o_obs + (size_t)t * od, obs, sizeof(float) * od);
        for (int i = 0; i < S; i++) {
            double a = acc_hi;
            for (int p = 0; p < P; p++) {
                float f[NF];
                feat_c(obs, &L, i, p, f);
                double cand;
                if (f[7] != 0.0f) {
                    double x = (10.0 - (double)f[0]) / dt;
                    double m = (acc_hi < x) ? acc_hi : x;
                    cand = (acc_lo > m) ? acc_lo : m;
                } else {
                    int wait = (2 * a_d[i * P + p] - 1) > 0;
                    float out;
                    oracle_mlp_forward(wait ? w_wait : w_cross, NF, 1, f, &out);
                    float tt = tanhf(out) * act_std;
                    cand = (double)(tt + act_mean);
                }
                if (cand < a) a = cand;
                double lim = (10.0 - (double)f[0]) / dt;
                if (lim < a) a = lim;
            }
            actions[i] = a;
            o_acts[(size_t)t * S + i] = (float)a;
        }
        for (int i = 0; i < S; i++) actions[S + i] = (double)(2 * a_d[i] - 1);
        const float prev1 = obs[L.env_off + 1];
        int done = oracle_env_step(e, actions, obs, rew, rl);
        for (int i = 0; i < S; i++) {
            o_rews_c[(size_t)t * S + i] = (float)rew[i];
            double m = epr[i], x = rl[i];
            epr[i] = (m != m) ? m : ((x != x) ? x : (x < m ? x : m));
        }
        const float cur1 = obs[L.env_off + 1];
        int trig = L.scalable ? (cur1 != (float)P) : (cur1 != prev1);
        o_saved[t] = (uint8_t)(trig || done);
        if (o_saved[t]) {
            oracle_env_dump(e, dump);
            for (int i = 0; i < S; i++) o_rews_d[(size_t)t * S + i] = (float)epr[i];
            for (int p = 0; p < P; p++) o_waiting[(size_t)t * P + p] = (float)dump[20 * p + 12];
        }
        if (trig) need = 1;
        if (done) { t++; break; }
    }
    return t;
}
