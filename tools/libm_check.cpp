// libm_check.cpp — pins mh-ppo_amd/csrc/libm_glibc.h against this host's glibc: every one of
// the 2^32 float bit patterns through mhppo_tanhf / mhppo_expm1f / mhppo_expf and through
// glibc's tanhf / expm1f / expf (the functions the C oracle and the reference's batch-1 torch
// calls use); a result counts as equal when the bits match (any NaN equals any NaN).
// Test infrastructure (tests/test_libm_glibc.py); build: make -C tools libm_check.
// Usage: libm_check [stride]  — stride > 1 checks every stride-th bit pattern (quick runs).
#include <math.h>
#include <omp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../mh-ppo_amd/csrc/libm_glibc.h"

static unsigned bits(float x) {
  unsigned u;
  memcpy(&u, &x, 4);
  return u;
}
static float flt(unsigned u) {
  float x;
  memcpy(&x, &u, 4);
  return x;
}
static bool same(float a, float b) { return (a != a && b != b) || bits(a) == bits(b); }

int main(int argc, char **argv) {
  const unsigned long long stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  const char *names[3] = {"tanhf", "expm1f", "expf"};
  unsigned long long bad[3] = {0, 0, 0}, checked = 0;
  unsigned first[3] = {0, 0, 0};
  bool have[3] = {false, false, false};
#pragma omp parallel
  {
    unsigned long long b[3] = {0, 0, 0}, n = 0;
    unsigned f[3] = {0, 0, 0};
    bool h[3] = {false, false, false};
#pragma omp for schedule(static)
    for (long long i = 0; i < (long long)(0x100000000ull / stride); i++) {
      const unsigned u = (unsigned)((unsigned long long)i * stride);
      const float x = flt(u);
      const float got[3] = {mhppo::mhppo_tanhf(x), mhppo::mhppo_expm1f(x), mhppo::mhppo_expf(x)};
      const float ref[3] = {tanhf(x), expm1f(x), expf(x)};
      for (int k = 0; k < 3; k++)
        if (!same(got[k], ref[k])) {
          if (!h[k]) f[k] = u, h[k] = true;
          b[k]++;
        }
      n++;
    }
#pragma omp critical
    {
      checked += n;
      for (int k = 0; k < 3; k++) {
        bad[k] += b[k];
        if (h[k] && (!have[k] || f[k] < first[k])) first[k] = f[k], have[k] = true;
      }
    }
  }
  printf("{\"checked\": %llu", checked);
  for (int k = 0; k < 3; k++) {
    printf(", \"%s\": {\"mismatches\": %llu", names[k], bad[k]);
    if (have[k]) {
      const float x = flt(first[k]);
      const float g = k == 0 ? mhppo::mhppo_tanhf(x) : (k == 1 ? mhppo::mhppo_expm1f(x) : mhppo::mhppo_expf(x));
      const float r = k == 0 ? tanhf(x) : (k == 1 ? expm1f(x) : expf(x));
      printf(", \"first_input\": \"0x%08x\", \"got\": \"0x%08x\", \"glibc\": \"0x%08x\"", first[k], bits(g), bits(r));
    }
    printf("}");
  }
  printf("}\n");
  return (bad[0] || bad[1] || bad[2]) ? 1 : 0;
}
