"""Pin the oracle's CPython-`random` restatement against this interpreter's own `random`.

The reference envs draw every random number from `random` (seeded at
Environments/Env_hybrid_multi_coop.py:10); the oracle and the HIP kernels
restate its MT19937 + helpers.  Bit-exact equality is required.
"""
import random

import numpy as np
import pytest

import oracle

SEEDS = [0, 1, 10, 12345, 2**32 - 1, 2**32 + 7, 2**40 + 3]


@pytest.mark.parametrize("seed", SEEDS)
def test_random_floats(seed):
    r = random.Random(seed)
    ref = np.array([r.random() for _ in range(5000)])
    assert np.array_equal(oracle.rng_stream(seed, 0, 5000), ref)


@pytest.mark.parametrize("seed", SEEDS[:4])
@pytest.mark.parametrize("ab", [(0, 20), (0, 9), (0, 1), (0, 2), (1, 1), (1, 8), (2, 5), (5, 35)])
def test_randint(seed, ab):
    r = random.Random(seed)
    ref = np.array([r.randint(*ab) for _ in range(3000)], dtype=np.float64)
    assert np.array_equal(oracle.rng_stream(seed, 1, 3000, *ab), ref)


@pytest.mark.parametrize("seed", SEEDS[:4])
def test_uniform_and_normal(seed):
    r = random.Random(seed)
    ref = np.array([r.uniform(-0.05, 0.75) for _ in range(3000)])
    assert np.array_equal(oracle.rng_stream(seed, 2, 3000, -0.05, 0.75), ref)
    r = random.Random(seed)
    ref = np.array([r.normalvariate(0.0, 0.09) for _ in range(3000)])
    assert np.array_equal(oracle.rng_stream(seed, 3, 3000, 0.0, 0.09), ref)


@pytest.mark.parametrize("seed", SEEDS[:4])
@pytest.mark.parametrize("n", [1, 2, 5, 8, 16])
def test_shuffle_and_sample(seed, n):
    r = random.Random(seed)
    ref = []
    for _ in range(200):
        x = list(range(n))
        r.shuffle(x)
        ref += x
    assert np.array_equal(oracle.rng_stream(seed, 5, 200, n, per=n), np.array(ref, dtype=np.float64))
    for k in range(1, n + 1):
        r = random.Random(seed)
        ref = sum((r.sample(list(range(n)), k) for _ in range(50)), [])
        assert np.array_equal(oracle.rng_stream(seed, 6, 50, n, k, per=k), np.array(ref, dtype=np.float64))
