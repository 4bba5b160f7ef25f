// hostsim_asan.cpp — the device env source (env_body.h via hostsim.cpp) as a standalone CPU
// program built under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers on
// host builds of the kernel source; GPU ASan is not available on the pool).  A standalone
// binary, not a shared object loaded into Python, so no sanitizer runtime has to be preloaded.
// Build: make -C tools asan.  Used by tests/test_env_asan.py.
//
// stdin-free file protocol: argv[1] = input: mhppo_env_cfg (raw struct), int32 T, then float64
// actions [T][N][2S]; argv[2] = output: reset obs f32 [N][od], then per step obs f32 [N][od],
// rewards f64 [N][R], reward_light f64 [N][R], done u8 [N], state f64 [N][sd].
#include <stdio.h>

#include "hostsim.cpp"

int main(int argc, char **argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s <in> <out>\n", argv[0]);
    return 2;
  }
  FILE *fi = fopen(argv[1], "rb");
  if (!fi) return 2;
  mhppo_env_cfg cfg;
  int32_t T = 0;
  if (fread(&cfg, sizeof(cfg), 1, fi) != 1 || fread(&T, 4, 1, fi) != 1 || T < 0) return 2;
  HostEnv *h = hs_create(&cfg);
  const int N = h->c.N, S = h->c.nS, R = hs_reward_slots(h), od = hs_obs_dim(h), sd = hs_state_dim(h);
  double *act = (double *)malloc(sizeof(double) * (size_t)T * N * 2 * S);
  if (fread(act, sizeof(double), (size_t)T * N * 2 * S, fi) != (size_t)T * N * 2 * S) return 2;
  fclose(fi);
  float *obs = (float *)malloc(sizeof(float) * (size_t)N * od);
  double *rew = (double *)malloc(sizeof(double) * (size_t)N * R), *rl = (double *)malloc(sizeof(double) * (size_t)N * R);
  double *st = (double *)malloc(sizeof(double) * (size_t)N * sd);
  uint8_t *done = (uint8_t *)malloc((size_t)N);
  FILE *fo = fopen(argv[2], "wb");
  if (!fo) return 2;
  hs_reset(h, obs);
  fwrite(obs, sizeof(float), (size_t)N * od, fo);
  for (int t = 0; t < T; t++) {
    hs_step(h, act + (size_t)t * N * 2 * S, obs, rew, rl, done);
    hs_state(h, st);
    fwrite(obs, sizeof(float), (size_t)N * od, fo);
    fwrite(rew, sizeof(double), (size_t)N * R, fo);
    fwrite(rl, sizeof(double), (size_t)N * R, fo);
    fwrite(done, 1, (size_t)N, fo);
    fwrite(st, sizeof(double), (size_t)N * sd, fo);
  }
  fclose(fo);
  free(act);
  free(obs);
  free(rew);
  free(rl);
  free(st);
  free(done);
  hs_destroy(h);
  return 0;
}
