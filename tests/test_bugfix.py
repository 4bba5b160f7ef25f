"""Opt-in bug-fix mode, oracle side: with MHPPO_FIX_SCALABLE_LANES the
scalable env builds slot i's car with i (lanes 0,0,1,1,..., followers 20 m behind on odd
slots) instead of the reference's i//2 (lanes 0,0,0,0,1,1,1,1); without it nothing
changes (the reference fixtures stay bit-exact: test_oracle_golden.py)."""
import numpy as np

import oracle


def test_scalable_lane_fix_mapping():
    ref = oracle.OracleEnv("scalable", 8, 1, 4, seed=5).reset()
    fix = oracle.OracleEnv("scalable", 8, 1, 4, seed=5, flags=1).reset()
    np.testing.assert_array_equal(ref[5:56:7], [0, 0, 0, 0, 1, 1, 1, 1])
    np.testing.assert_array_equal(fix[5:56:7], [0, 0, 1, 1, 2, 2, 3, 3])
    # same draws: existing cars' positions differ exactly by the follower offset change
    sc_r, sc_f, ex = ref[3:56:7], fix[3:56:7], ref[6:56:7]
    for i in range(8):
        if ex[i]:
            off_r, off_f = 20.0 * ((i // 2) % 2), 20.0 * (i % 2)
            assert abs((sc_r[i] + off_r) - (sc_f[i] + off_f)) < 1e-4
