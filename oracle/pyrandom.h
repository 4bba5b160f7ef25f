/* ORACLE — test infrastructure only.  Never linked into the product path.
 *
 * CPU restatement of CPython 3.10's `random` module (the stream every
 * reference env draws from: `random.seed(10)` at
 * Environments/Env_hybrid_multi_coop.py:10).  Algorithms restated from the
 * CPython sources shipped with this interpreter:
 *   Modules/_randommodule.c  init_genrand / init_by_array / genrand_uint32 /
 *                            random_random / getrandbits (k <= 32) / seed(int)
 *   /usr/lib/python3.10/random.py:239-250  _randbelow_with_getrandbits
 *   /usr/lib/python3.10/random.py:291-330  randrange -> randint
 *   /usr/lib/python3.10/random.py:380-394  shuffle
 *   /usr/lib/python3.10/random.py:480-497  sample (pool branch, n <= setsize)
 *   /usr/lib/python3.10/random.py:546-548  uniform
 *   /usr/lib/python3.10/random.py:570-589  normalvariate (Kinderman-Monahan)
 * Pinned bit-exact against the interpreter itself by tests/test_oracle_random.py.
 */
#ifndef MHPPO_ORACLE_PYRANDOM_H
#define MHPPO_ORACLE_PYRANDOM_H
#include <math.h>
#include <stdint.h>

#define PYR_N 624
#define PYR_M 397

typedef struct {
    uint32_t mt[PYR_N];
    int mti;
    uint64_t words; /* 32-bit outputs consumed since seeding (test counter) */
} PyRandom;

static void pyr_init_genrand(PyRandom *r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < PYR_N; i++)
        r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->mti = PYR_N;
}

static void pyr_init_by_array(PyRandom *r, const uint32_t *key, int klen) {
    pyr_init_genrand(r, 19650218u);
    int i = 1, j = 0;
    for (int k = (PYR_N > klen ? PYR_N : klen); k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= PYR_N) { r->mt[0] = r->mt[PYR_N - 1]; i = 1; }
        if (j >= klen) j = 0;
    }
    for (int k = PYR_N - 1; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= PYR_N) { r->mt[0] = r->mt[PYR_N - 1]; i = 1; }
    }
    r->mt[0] = 0x80000000u;
}

/* random.seed(n) for a non-negative int n < 2**64 */
static void pyr_seed(PyRandom *r, uint64_t n) {
    uint32_t key[2];
    int klen = 1;
    key[0] = (uint32_t)n;
    key[1] = (uint32_t)(n >> 32);
    if (key[1]) klen = 2;
    pyr_init_by_array(r, key, klen);
    r->words = 0;
}

static uint32_t pyr_genrand(PyRandom *r) {
    static const uint32_t mag01[2] = {0x0u, 0x9908b0dfu};
    uint32_t y;
    if (r->mti >= PYR_N) {
        int kk;
        for (kk = 0; kk < PYR_N - PYR_M; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + PYR_M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < PYR_N - 1; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + (PYR_M - PYR_N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (r->mt[PYR_N - 1] & 0x80000000u) | (r->mt[0] & 0x7fffffffu);
        r->mt[PYR_N - 1] = r->mt[PYR_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        r->mti = 0;
    }
    y = r->mt[r->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    r->words++;
    return y;
}

/* random.random(): 53-bit double from two words */
static double pyr_random(PyRandom *r) {
    uint32_t a = pyr_genrand(r) >> 5, b = pyr_genrand(r) >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
}

static int pyr_bit_length(uint32_t n) {
    int k = 0;
    while (n) { k++; n >>= 1; }
    return k;
}

/* _randbelow_with_getrandbits(n), n < 2**32 */
static uint32_t pyr_randbelow(PyRandom *r, uint32_t n) {
    if (!n) return 0;
    int k = pyr_bit_length(n);
    uint32_t v = pyr_genrand(r) >> (32 - k);
    while (v >= n) v = pyr_genrand(r) >> (32 - k);
    return v;
}

static long pyr_randint(PyRandom *r, long a, long b) {
    return a + (long)pyr_randbelow(r, (uint32_t)(b - a + 1));
}

static double pyr_uniform(PyRandom *r, double a, double b) {
    return a + (b - a) * pyr_random(r);
}

/* NV_MAGICCONST = 4 * exp(-0.5) / sqrt(2.0), value of this interpreter */
#define PYR_NV_MAGICCONST 0x1.b72cd3f331398p+0

static double pyr_normalvariate(PyRandom *r, double mu, double sigma) {
    double z;
    for (;;) {
        double u1 = pyr_random(r);
        double u2 = 1.0 - pyr_random(r);
        z = PYR_NV_MAGICCONST * (u1 - 0.5) / u2;
        double zz = z * z / 4.0;
        if (zz <= -log(u2)) break;
    }
    return mu + z * sigma;
}

/* shuffle(x) for a list of n ints in place */
static void pyr_shuffle(PyRandom *r, int *x, int n) {
    for (int i = n - 1; i >= 1; i--) {
        int j = (int)pyr_randbelow(r, (uint32_t)(i + 1));
        int t = x[i]; x[i] = x[j]; x[j] = t;
    }
}

/* sample(range(n), k), pool branch (n <= 21 + ... always true for n <= 21) */
static void pyr_sample_range(PyRandom *r, int n, int k, int *out) {
    int pool[64];
    for (int i = 0; i < n; i++) pool[i] = i;
    for (int i = 0; i < k; i++) {
        int j = (int)pyr_randbelow(r, (uint32_t)(n - i));
        out[i] = pool[j];
        pool[j] = pool[n - i - 1];
    }
}

#endif
