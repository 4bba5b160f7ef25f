"""Full-scale discrete parity of the HIP env against the C oracle (OpenMP over envs).

The bench's env shapes at the bench's env count (65 536 envs x 80 steps): config 3
(4cars 4/1/2, Env_hybrid_multi_coop_4cars.py:783-911) and config 4 (scalable 8/1/4,
Env_hybrid_multi_coop_scalable.py:789-946), plus config 2's coop 2/1/2 env.  Forced
actions (uniform accelerations in [-4.5, 2.5] rounded through float32, one fixed light
per env and slot), the same per-env CPython streams on both sides.

Checked EVERY step for EVERY env, exactly: done, the RNG cursor (number of MT19937
words drawn so far, mod 624 — the data-dependent draw count of the gap-acceptance
decisions, normalvariate rejections and stop draws), every discrete
pedestrian field (decision, at_crossing, left, in_cross, accident, time_stop, stop,
line, need_to_stop, direction, follow_rule), each car's light and existence, and the five
per-env event counters (detection's prints, tests/test_events.py).  At the
end: every env's whole MT19937 state.  Float64 state/rewards: device libm vs glibc may
differ in the last bits; asserted to rel 1e-9 (float32 observations 1e-6), and the
fraction of bit-different outputs is reported.
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DISCRETE_PED = [4, 5, 6, 7, 8, 9, 10, 11, 17, 18, 19]
DISCRETE_CAR = [3, 7]  # light, exist


def _report(name, rec):
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"parity_fullscale_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)
    print(name, json.dumps(rec))


# cfg5_shard7: config 5 (524 288 scalable envs over 8 GPUs) is env-id sharded; its last rank runs
# global ids 458 752 .. 524 287 (env_id_offset = 7 x 65 536) and must draw exactly the streams the
# reference's env would at those ids (random.seed(seed_base + global id)) — the one config-5
# property a single GPU can pin.
@pytest.mark.parametrize("case", [("4cars", 4, 1, 2, 0), ("scalable", 8, 1, 4, 0), ("coop", 2, 1, 2, 0),
                                  ("scalable", 8, 1, 4, 7 * 65536)],
                         ids=["cfg3_4cars", "cfg4_scalable", "cfg2_coop", "cfg5_shard7_scalable"])
def test_fullscale_discrete_parity(case):
    from mhppo.env import VecCrosswalk
    from oracle import OracleBatch, set_threads
    set_threads(min(16, os.cpu_count() or 1))
    v, nc, npd, nl, off = case
    N, T, seed = 65536, 80, 31000
    env = VecCrosswalk(v, N, nc, npd, nl, seed_base=seed, env_id_offset=off)
    orc = OracleBatch(v, N, nc, npd, nl, seed_base=seed + off)  # the oracle's env e = global id off + e
    assert np.array_equal(env.reset().cpu().numpy(), orc.reset())
    k = orc.dump_dim
    S = env.n_slots
    rng = np.random.default_rng(7)
    light = rng.choice([-1.0, 1.0], size=(N, S))
    div = np.zeros(N, bool)          # any discrete mismatch so far
    first_div = np.full(N, -1)
    n_bits = n_tot = 0
    r_bits = r_tot = 0  # rewards + reward_light only
    max_rel = max_rel_obs = 0.0
    for t in range(T):
        acc = rng.uniform(-4.5, 2.5, size=(N, S)).astype(np.float32).astype(np.float64)
        a = np.concatenate([acc, light], 1)
        o, r, rl, d = env.step(torch.from_numpy(a).cuda())
        st = env.get_state()[:, :k].cpu().numpy()
        _, mti_g = env.get_rng()
        o, r, rl, d, mti_g = o.cpu().numpy(), r.cpu().numpy(), rl.cpu().numpy(), d.cpu().numpy(), mti_g.cpu().numpy()
        oo, ro, rlo, do, dm, mti_o = orc.step(a, want_dump=True)
        ped_g = st[:, :20 * npd].reshape(N, npd, 20)[:, :, DISCRETE_PED].reshape(N, -1)
        ped_o = dm[:, :20 * npd].reshape(N, npd, 20)[:, :, DISCRETE_PED].reshape(N, -1)
        car_g = st[:, 20 * npd:].reshape(N, -1, 8)[:, :, DISCRETE_CAR].reshape(N, -1)
        car_o = dm[:, 20 * npd:].reshape(N, -1, 8)[:, :, DISCRETE_CAR].reshape(N, -1)
        ev_g, ev_o = env.events().cpu().numpy().astype(np.uint32), orc.events()
        bad = (d != do) | (mti_g != mti_o) | (ped_g != ped_o).any(1) | (car_g != car_o).any(1) | (ev_g != ev_o).any(1)
        first_div[bad & ~div] = t
        div |= bad
        ok = ~div
        for g, ref in ((r, ro), (rl, rlo), (st, dm), (o, oo)):
            is_obs = g is o
            is_rew = g is r or g is rl
            g, ref = g[ok].astype(np.float64), ref[ok].astype(np.float64)
            n_bits += int((g != ref).sum())
            n_tot += g.size
            if is_rew:
                r_bits += int((g != ref).sum())
                r_tot += g.size
            if g.size:
                rel = float(np.nanmax(np.abs(g - ref) / np.maximum(np.abs(ref), 1e-3)))
                if is_obs:
                    max_rel_obs = max(max_rel_obs, rel)
                else:
                    max_rel = max(max_rel, rel)
    mt_g, _ = env.get_rng()
    mt_o, _ = orc.rng_state()
    mt_bad = (mt_g.cpu().numpy().view(np.uint32) != mt_o).any(1)
    rec = dict(config=f"{v} {nc}/{npd}/{nl}", envs=N, env_id_offset=off, steps=T, diverged_envs=int(div.sum()),
               mt_state_mismatch_envs=int(mt_bad.sum()), first_divergence_steps=sorted(set(first_div[div].tolist()))[:20],
               diverged_env_ids=np.nonzero(div)[0][:20].tolist(), float_outputs_bit_different=n_bits,
               float_outputs=n_tot, bit_different_fraction=n_bits / max(n_tot, 1),
               reward_bit_different_fraction=r_bits / max(r_tot, 1),
               event_counts_gpu=dict(zip(("accident", "possible_accident", "small_mistake", "not_waiting",
                                          "bad_green"), ev_g.sum(0).tolist())),
               max_rel_err_f64_undiverged=max_rel, max_rel_err_obs_f32_undiverged=max_rel_obs)
    _report(v + (f"_offset{off}" if off else ""), rec)
    assert rec["diverged_envs"] == 0 and rec["mt_state_mismatch_envs"] == 0, rec
    assert max_rel <= 1e-9 and max_rel_obs <= 1e-6, rec
