"""GPU rollout collector (mhppo_rollout_begin/step kernels) vs the reference rollout
fixtures (recorded noise replayed) and vs the C rollout oracle at larger N with
Philox noise.  Discrete outputs (Categorical draws, closest pedestrian, car
existence, bucket membership) must be identical; continuous ones agree to
float32 tolerance (device vs glibc libm: tanh/exp/log/pow ulps)."""
import glob
import os

import numpy as np
import pytest
import torch

import oracle
from rollout_util import bucket, returns

pytestmark = pytest.mark.gpu
FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rollout_*.npz")))


def _actors(wc, ww, wd, dc):
    from mhppo.models import Model_PPO
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).load_packed(wc).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).load_packed(ww).cuda()
    ad = Model_PPO(dc, 2, 2).load_packed(wd).cuda()
    return ac, aw, ad


def _gpu_out(batch):
    return {k: getattr(batch, k).cpu().numpy() for k in ("feat_d", "a_d", "logp_d", "closest", "exist", "obs_c", "act",
                                                         "logp", "rew", "ep_min")}


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[8:-4] for f in FILES])
def test_gpu_rollout_matches_reference(path):
    from mhppo.env import VecCrosswalk
    from mhppo.rollout import RolloutGPU
    g = np.load(path)
    v = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    E = g["a_d"].shape[0]
    venv = VecCrosswalk(v, E, nc, npd, nl, seed_base=int(g["seed_base"]))
    ro = RolloutGPU(venv)
    ac, aw, ad = _actors(g["w_cross"], g["w_wait"], g["w_choice"], ro.dc)
    batch = ro.collect(ac, aw, ad, forced_choice=torch.from_numpy(g["a_d"]), eps_tape=torch.from_numpy(g["eps"]))
    b = bucket(_gpu_out(batch), v == "scalable")
    np.testing.assert_array_equal(b["act_choice"], g["act_choice"])
    for k in ("obs_cross", "obs_wait", "obs_choice"):
        assert b[k].shape == g[k].shape, k
    for k, tol in (("obs_cross", 2e-5), ("obs_wait", 2e-5), ("obs_choice", 2e-5), ("act_cross", 2e-5),
                   ("act_wait", 2e-5), ("logp_cross", 2e-5), ("logp_wait", 2e-5), ("logp_choice", 2e-5),
                   ("rew_cross", 1e-5), ("rew_wait", 1e-5), ("rew_choice", 1e-5)):
        np.testing.assert_allclose(b[k], g[k], rtol=tol, atol=tol, err_msg=k)
    for h in ("cross", "wait"):
        np.testing.assert_allclose(returns(b["rew_" + h]), g["ret_" + h], rtol=1e-4, atol=1e-4, err_msg=h)


@pytest.mark.parametrize("case", [("4cars", 4, 1, 2), ("coop", 2, 1, 2), ("scalable", 8, 1, 4), ("coop", 4, 2, 2),
                                  ("stop", 2, 2, 2), ("stop", 2, 1, 2), ("4cars", 4, 1, 2, "generic")])
def test_gpu_rollout_matches_oracle_philox(case):
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    v, nc, npd, nl = case[:4]
    N = 256
    venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=31000, generic_step=len(case) > 4)
    ro = RolloutGPU(venv)
    torch.manual_seed(5)
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    ad = Model_PPO(ro.dc, 2, 2).cuda()
    batch = ro.collect(ac, aw, ad, seed=3, iteration=0)
    go = _gpu_out(batch)
    o = oracle.rollout(v, nc, npd, nl, [31000 + e for e in range(N)], ac.packed().cpu().numpy(),
                       aw.packed().cpu().numpy(), ad.packed().cpu().numpy(), u=ro.u.cpu().numpy(),
                       eps=ro.eps.cpu().numpy())
    for k in ("a_d", "closest", "exist"):
        np.testing.assert_array_equal(go[k], o[k], err_msg=k)
    np.testing.assert_allclose(go["feat_d"], o["feat_d"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(go["logp_d"], o["logp_d"], rtol=1e-5, atol=1e-5)
    # the per-(env, slot, t) records of present car slots (the scalable env's compact record layout
    # stores none for absent slots: include/mhppo.h mhppo_rollout_bufs.rec_of)
    m = go["exist"].astype(bool)
    assert batch.rec_of is not None or m.all()
    np.testing.assert_allclose(go["obs_c"][m], o["obs_c"][m], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(go["act"][m], o["act"][m], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(go["logp"][m], o["logp"][m], rtol=1e-5, atol=1e-5)
    # float64 env outputs downstream of float32 actions: ulp-level action differences
    # (device vs glibc tanhf) drift positions over 80 steps; 1e-5 keeps returns well
    # inside the 1e-4 bound
    np.testing.assert_allclose(go["rew"][m], o["rew"][m], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(go["ep_min"], o["ep_min"], rtol=1e-5, atol=1e-5)


def test_rollout_is_shard_invariant():
    """Envs split over two handles (as over two ranks: env_id_offset) replay exactly the
    single-handle trajectories: per-env CPython streams + global-id Philox counters."""
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    torch.manual_seed(9)
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    full = RolloutGPU(VecCrosswalk("4cars", 128, 4, 1, 2, seed_base=5))
    ad = Model_PPO(full.dc, 2, 2).cuda()
    a = _gpu_out(full.collect(ac, aw, ad, seed=1, iteration=2))
    parts = []
    for off in (0, 64):
        ro = RolloutGPU(VecCrosswalk("4cars", 64, 4, 1, 2, seed_base=5, env_id_offset=off))
        parts.append(_gpu_out(ro.collect(ac, aw, ad, seed=1, iteration=2)))
    for k in a:
        assert np.array_equal(a[k], np.concatenate([parts[0][k], parts[1][k]])), k


POLICY_CASES = [("4cars", 4, 1, 2), ("coop", 2, 1, 2), ("scalable", 8, 2, 4), ("stop", 2, 2, 2)]


@pytest.mark.parametrize("mode", ["sorted", "unsorted"])
def test_mfma_policy_bit_identical_to_valu(mode, tmp_path):
    """The shipped MFMA policy kernel (k_policy_mfma: permuted weight rows so every f32-MFMA fmaf
    chain runs in ascending input order) and the VALU reference kernels (k_policy_sorted, head-sorted
    SGPR weights; k_policy, one lane per row), which only the test build of the library carries
    (tests/lib/libmhppo_test.so, run in a child process), give the same episode bit for bit, ragged
    last tiles included (N*S*P not a multiple of 32)."""
    import subprocess
    import sys
    from rollout_policy_case import run_case
    here = os.path.dirname(os.path.abspath(__file__))
    test_lib = os.path.join(here, "lib", "libmhppo_test.so")
    assert os.path.exists(test_lib), "build the test library: make -C mh-ppo_amd/csrc test-lib"
    out = str(tmp_path / "valu.npz")
    env = dict(os.environ, MHPPO_LIB=test_lib)
    subprocess.run([sys.executable, os.path.join(here, "valu_policy_worker.py"), out, mode] +
                   [",".join(map(str, c)) for c in POLICY_CASES], env=env, check=True, timeout=300)
    valu = np.load(out)
    for case in POLICY_CASES:
        mfma = run_case(case, False)
        cs = ",".join(map(str, case))
        for k, x in mfma.items():
            assert np.array_equal(x, valu[f"{cs}/{k}"]), (case, k)


def test_valu_policy_refused_by_the_shipped_library():
    """The shipped library has no VALU policy kernels: asking for them is an error, not a fallback."""
    from mhppo import _lib
    from rollout_policy_case import run_case
    if os.environ.get("MHPPO_LIB"):
        pytest.skip("an alternative library build is loaded")
    with pytest.raises(_lib.MhppoError, match="test build only"):
        run_case(("coop", 2, 1, 2), True)


def test_kernel_timing_events_leave_results_unchanged():
    """mhppo_kernel_timing_begin/_end (bench.py's env-kernel clock): the timed launches
    (hipExtLaunchKernelGGL with dispatch-attached events) produce the same episode bit for bit
    as untimed ones, exactly the requested number of launches is timed, and the time is positive."""
    import ctypes
    from mhppo import _lib
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    L = _lib.lib()
    outs, times = [], []
    for timed in (False, True):
        ro = RolloutGPU(VecCrosswalk("4cars", 256, 4, 1, 2, seed_base=11))
        torch.manual_seed(4)
        ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        ad = Model_PPO(ro.dc, 2, 2).cuda()
        if timed:
            _lib.check(L.mhppo_kernel_timing_begin(50))  # fewer than the episode's 80 steps
        outs.append(_gpu_out(ro.collect(ac, aw, ad, seed=3, iteration=0, graph=False)))
        if timed:
            ms, n = ctypes.c_double(0.0), ctypes.c_int32(0)
            _lib.check(L.mhppo_kernel_timing_end(ctypes.byref(ms), ctypes.byref(n)))
            times.append((ms.value, n.value))
    for k in outs[0]:
        assert np.array_equal(outs[0][k], outs[1][k]), k
    ms, n = times[0]
    assert n == 50 and ms > 0.0


@pytest.mark.parametrize("case", [("4cars", 4, 1, 2, 4096), ("scalable", 8, 1, 4, 4000), ("coop", 4, 2, 2, 1000)])
def test_two_part_rollout_equals_one_chain(case):
    """RolloutGPU(parts=2): the two env parts' step chains on two streams (mhppo_rollout_policy_part /
    _sample_env_part, part bounds from k_part_bounds) give bit-identical records to the one-chain
    loop — including a ragged N (a part boundary at a multiple of 64 envs) and P = 2 pedestrians."""
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    v, nc, npd, nl, N = case
    outs = []
    for parts in (1, 2):
        venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=900)
        ro = RolloutGPU(venv, parts=parts)
        torch.manual_seed(3)
        ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        ad = Model_PPO(ro.dc, 2, 2).cuda()
        b = ro.collect(ac, aw, ad, seed=2, iteration=1)
        torch.cuda.synchronize()
        outs.append({k: getattr(b, k).clone() for k in ("a_d", "closest", "exist", "obs_c", "act", "logp", "rew",
                                                         "ep_min", "feat_d", "logp_d")})
        outs[-1]["state"] = venv.state_dict()["blob"]
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("parts,N", [(1, 1000), (2, 4000)])
def test_graph_replay_equals_eager(parts, N):
    """RolloutGPU.collect(graph=True): the one-chain step loop captured once as a HIP graph and
    replayed gives bit-identical records and env state to the eager launches — over two
    iterations with new noise and with the actors' weights changed in place in between (the graph
    reads the live weights); the two-stream parts loop (forked / joined inside the capture) too."""
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    outs = []
    for graph in (False, True):
        venv = VecCrosswalk("coop", N, 2, 1, 2, seed_base=77)
        ro = RolloutGPU(venv, parts=parts)
        torch.manual_seed(9)
        ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
        ad = Model_PPO(ro.dc, 2, 2).cuda()
        rec = []
        for it in range(3):
            if it == 2:
                with torch.no_grad():
                    ac.flat().mul_(0.9)
                    aw.flat().add_(0.01)
            b = ro.collect(ac, aw, ad, seed=5, iteration=it, graph=graph)
            torch.cuda.synchronize()
            rec.append({k: getattr(b, k).clone() for k in ("a_d", "obs_c", "act", "logp", "rew", "ep_min")})
            rec[-1]["state"] = venv.state_dict()["blob"]
            venv.reset(want_obs=False)
        assert len(ro._graphs) == (1 if graph else 0)
        outs.append(rec)
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k
