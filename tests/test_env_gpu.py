"""HIP env kernels vs the reference fixtures and vs the C oracle.

Bit-exact: RNG streams (final MT19937 state), done flags, every discrete field of
the internal state, observations.  Float64 rewards / reward_light / continuous
state: device libm (ocml exp/pow/log/sin/cos) may differ from glibc by an ulp,
so those are checked to 1e-9 relative, and at most 12 % of the rewards may differ in their
last bits (the measured fractions are reported by test_env_fullscale_gpu.py).
"""
import glob
import os

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "env_*.npz")))
pytestmark = pytest.mark.gpu
DISCRETE = [4, 5, 6, 7, 8, 9, 10, 11, 17, 18, 19]  # per-ped dump fields that are flags / ints


# view "default": the register env view where compiled (single-pedestrian fixture shapes),
# "generic": every step forced onto the in-HBM view
@pytest.mark.parametrize("view", ["default", "generic"])
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[4:-4] for f in FILES])
def test_gpu_env_matches_reference(path, view):
    from mhppo.env import VecCrosswalk
    g = np.load(path)
    E, T = g["obs"].shape[:2]
    npd = int(g["nb_ped"])
    env = VecCrosswalk(str(g["variant"]), E, int(g["nb_car"]), npd, int(g["nb_lines"]), seed_base=int(g["seed_base"]),
                       generic_step=view == "generic")
    assert np.array_equal(env.reset().cpu().numpy(), g["obs0"])
    assert not env.events().any()
    # detection's prints per env and step, as the reference printed them (tests/test_events.py)
    ev = np.cumsum(np.load(path.replace("env_", "events_"))["events"], axis=1)
    k = g["dump"].shape[2]
    for t in range(T):
        o, r, rl, d = env.step(torch.from_numpy(g["actions"][:, t]).cuda())
        assert np.array_equal(env.events().cpu().numpy(), ev[:, t]), t
        st = env.get_state().cpu().numpy()[:, :k]
        ref = g["dump"][:, t]
        assert np.array_equal(d.cpu().numpy(), g["done"][:, t])
        np.testing.assert_allclose(o.cpu().numpy(), g["obs"][:, t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(r.cpu().numpy(), g["rewards"][:, t], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(rl.cpu().numpy(), g["reward_light"][:, t], rtol=1e-9, atol=1e-12)
        ped = st[:, :20 * npd].reshape(E, npd, 20)[:, :, DISCRETE]
        assert np.array_equal(ped, ref[:, :20 * npd].reshape(E, npd, 20)[:, :, DISCRETE]), t
        np.testing.assert_allclose(st, ref, rtol=1e-9, atol=1e-12)
    mt, _ = env.get_rng()
    assert np.array_equal(mt.cpu().numpy().view(np.uint32), g["final_mt"])


@pytest.mark.parametrize("case", [("coop", 2, 1, 2), ("4cars", 4, 1, 2), ("scalable", 8, 1, 4), ("naif", 1, 1, 1),
                                  ("coop", 4, 3, 2), ("scalable", 4, 2, 2)])
def test_gpu_env_matches_oracle_many_envs(case):
    from mhppo.env import VecCrosswalk
    from oracle import OracleEnv
    v, nc, npd, nl = case
    N = 512
    env = VecCrosswalk(v, N, nc, npd, nl, seed_base=9000)
    orc = [OracleEnv(v, nc, npd, nl, seed=9000 + e) for e in range(N)]
    assert np.array_equal(env.reset().cpu().numpy(), np.stack([o.reset() for o in orc]))
    rng = np.random.default_rng(1)
    S = env.n_slots
    light = rng.choice([-1.0, 1.0], size=(N, S))
    n_diff = n_tot = 0
    for t in range(80):
        a = np.concatenate([rng.uniform(-4.5, 2.5, size=(N, S)).astype(np.float32).astype(np.float64), light], 1)
        o, r, rl, d = env.step(torch.from_numpy(a).cuda())
        o, r, rl, d = o.cpu().numpy(), r.cpu().numpy(), rl.cpu().numpy(), d.cpu().numpy()
        ref = [orc[e].step(a[e]) for e in range(N)]
        ro = np.stack([x[0] for x in ref]); rr = np.stack([x[1] for x in ref]); rrl = np.stack([x[2] for x in ref])
        assert np.array_equal(d, np.array([x[3] for x in ref]))
        np.testing.assert_allclose(o, ro, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(r, rr, rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(rl, rrl, rtol=1e-9, atol=1e-12)
        n_diff += int((r != rr).sum() + (rl != rrl).sum())
        n_tot += r.size + rl.size
    # rewards / reward_light whose last bits differ (device libm vs glibc exp/pow): 6.2 % measured for
    # coop 2/1/2 here; tests/test_env_fullscale_gpu.py measures every config at 65 536 envs (none
    # diverges discretely there)
    print(f"{case}: {n_diff}/{n_tot} float64 rewards differ in their last bits")
    assert n_diff <= 0.12 * n_tot, f"{n_diff}/{n_tot} float64 outputs differ in their last bits"


@pytest.mark.parametrize("case", [("coop", 2, 1, 2), ("4cars", 4, 1, 2), ("scalable", 8, 1, 4), ("stop", 2, 1, 2),
                                  ("4cars2", 4, 1, 2)])
def test_register_view_is_bit_identical_to_generic(case):
    """The register env view and the in-HBM view run the same arithmetic on the same
    device libm: every output and the whole env state must agree bit for bit."""
    from mhppo.env import VecCrosswalk
    v, nc, npd, nl = case
    N = 4096
    envs = [VecCrosswalk(v, N, nc, npd, nl, seed_base=777, generic_step=g) for g in (False, True)]
    o0 = [e.reset() for e in envs]
    assert torch.equal(o0[0], o0[1])
    S = envs[0].n_slots
    gen = torch.Generator().manual_seed(4)
    for t in range(160):  # two episodes: the second starts without a reset (time keeps running)
        acc = torch.rand((N, S), generator=gen, dtype=torch.float64) * 7 - 4.5
        light = torch.where(torch.rand((N, S), generator=gen) < 0.5, -1.0, 1.0).double()
        a = torch.cat([acc.float().double(), light], 1).cuda()
        outs = [e.step(a) for e in envs]
        for x, y in zip(outs[0], outs[1]):
            assert torch.equal(x, y), t
    assert torch.equal(envs[0].get_state(), envs[1].get_state())
    (m0, i0), (m1, i1) = envs[0].get_rng(), envs[1].get_rng()
    assert torch.equal(m0, m1) and torch.equal(i0, i1)
