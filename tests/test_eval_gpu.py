"""GPU deterministic evaluation (mhppo_eval_step, RolloutGPU.evaluate — the body of
Env_rollout.iterations / Algo_PPO.evaluate) vs the reference's evaluation on its shipped
weights (tests/golden/eval_*.npz) — the same bar as the oracle (test_oracle_eval.py) —
and vs the C oracle at a larger env count with random-init heads."""
import os

import numpy as np
import pytest
import torch

from test_oracle_eval import CASES, CHOIX_CASES, TOL_CHOIX, check_eval

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
KEYS = ("obs", "acts", "rews_c", "rews_d", "waiting")


def _nets(wc, ww, wd, dc):
    from mhppo.models import Model_PPO
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).load_packed(wc).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).load_packed(ww).cuda()
    ad = Model_PPO(dc, 2, 2).load_packed(wd).cuda()
    return ac, aw, ad


def _evaluate(venv, nets, K, choix=False):
    from mhppo.rollout import RolloutGPU
    venv.reset(want_obs=False)  # Env_rollout.reset() before iterations (:744, :129)
    out = RolloutGPU(venv).evaluate(*nets, K, choix=choix)
    return dict(zip(KEYS, (t.cpu().numpy() for t in out)))


@pytest.mark.parametrize("name", CASES)
def test_gpu_eval_matches_reference(name):
    import oracle
    from mhppo.env import VecCrosswalk
    g = np.load(os.path.join(ROOT, "tests", "golden", f"eval_{name}.npz"))
    E, K, variant = len(g["n_obs"]), int(g["episodes"]), str(g["variant"])
    venv = VecCrosswalk(variant, E, int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]))
    nets = _nets(g["w_cross"], g["w_wait"], g["w_choice"], oracle.choice_dim(variant, venv.n_slots))
    check_eval(_evaluate(venv, nets, K), g)


def test_gpu_eval_matches_oracle_many_envs():
    """64 scalable envs (2 lanes, 2 peds, 4 slots) x 2 episodes: same saves, waiting times
    exact, continuous values within float32 noise."""
    import oracle
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    torch.manual_seed(7)
    venv = VecCrosswalk("scalable", 64, 4, 2, 2, seed_base=4242)
    dc = oracle.choice_dim("scalable", venv.n_slots)
    w = [Model_PPO(13, 1, 1).packed().numpy(), Model_PPO(13, 1, 1).packed().numpy(),
         Model_PPO(dc, 2, 2).packed().numpy()]
    out = _evaluate(venv, _nets(*w, dc), 2)
    res = oracle.evaluate("scalable", 4, 2, 2, [4242 + e for e in range(64)], 2, *w)
    check_eval(out, {k: np.concatenate([r[k] for r in res]) for k in res[0]})


def test_algo_evaluate_api():
    """Algo_PPO.evaluate(k) returns the reference's five tensors with N*k episodes."""
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    venv = VecCrosswalk("coop", 8, 2, 1, 2, seed_base=11)
    algo = Algo_PPO(Model_PPO, venv, verbose=False)
    obs, acts, rc, rd, wt = algo.evaluate(3)
    assert obs.shape == (8 * 3 * 80, venv.obs_dim) and acts.shape == (8 * 3 * 80, 2) and rc.shape == acts.shape
    assert rd.shape == (8 * 3, 2) and wt.shape == (8 * 3,)
    assert torch.isfinite(obs).all() and torch.isfinite(acts).all()


@pytest.mark.parametrize("name", CHOIX_CASES)
def test_gpu_eval_choix_matches_reference(name):
    """evaluate(n, choix=True): the scripted choix_test scenario after every reset."""
    import oracle
    from mhppo.env import VecCrosswalk
    g = np.load(os.path.join(ROOT, "tests", "golden", f"eval_{name}.npz"))
    E, K, variant = len(g["n_obs"]), int(g["episodes"]), str(g["variant"])
    venv = VecCrosswalk(variant, E, int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]))
    nets = _nets(g["w_cross"], g["w_wait"], g["w_choice"], oracle.choice_dim(variant, venv.n_slots))
    out = _evaluate(venv, nets, K, choix=True)
    assert np.array_equal(out["obs"][0], g["obs"][0])  # the scripted observation
    check_eval(out, g, tol=TOL_CHOIX)


def test_gpu_eval_choix_matches_oracle_many_envs():
    import oracle
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    torch.manual_seed(8)
    venv = VecCrosswalk("scalable", 64, 4, 2, 2, seed_base=5151)
    dc = oracle.choice_dim("scalable", venv.n_slots)
    w = [Model_PPO(13, 1, 1).packed().numpy(), Model_PPO(13, 1, 1).packed().numpy(),
         Model_PPO(dc, 2, 2).packed().numpy()]
    out = _evaluate(venv, _nets(*w, dc), 2, choix=True)
    res = oracle.evaluate("scalable", 4, 2, 2, [5151 + e for e in range(64)], 2, *w, choix=True)
    check_eval(out, {k: np.concatenate([r[k] for r in res]) for k in res[0]})


def test_choix_rejected_off_scalable():
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    algo = Algo_PPO(Model_PPO, VecCrosswalk("coop", 4, 2, 1, 2, seed_base=1), verbose=False)
    from mhppo._lib import MhppoError
    with pytest.raises(MhppoError):
        algo.evaluate(1, choix=True)


STATS = sorted(f[6:-4] for f in os.listdir(os.path.join(ROOT, "tests", "golden")) if f.startswith("stats_"))


@pytest.mark.parametrize("name", STATS)
def test_gpu_get_average_matches_reference(name):
    """get_average (:1550-1675) over the GPU's own evaluation (computed on the device) vs the
    reference function on the reference's trajectories (tests/golden/stats_*.npz): shares
    exact, statistics within float32 noise of the trajectories."""
    import oracle
    from mhppo.env import VecCrosswalk
    from mhppo.stats import get_average
    from test_stats import _check
    s = np.load(os.path.join(ROOT, "tests", "golden", f"stats_{name}.npz"))
    g = np.load(os.path.join(ROOT, "tests", "golden", str(s["eval_fixture"])))
    E, K, variant = len(g["n_obs"]), int(g["episodes"]), str(g["variant"])
    venv = VecCrosswalk(variant, E, int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]))
    nets = _nets(g["w_cross"], g["w_wait"], g["w_choice"], oracle.choice_dim(variant, venv.n_slots))
    from mhppo.rollout import RolloutGPU
    venv.reset(want_obs=False)
    states = RolloutGPU(venv).evaluate(*nets, K, choix="choix" in name)[0]
    assert states.is_cuda
    got = get_average(states, variant, venv.nb_car, venv.nb_ped, venv.nb_lines)
    for k in ("yield_share", "go_share", "could_stop_share", "episodes"):
        if k in s.files:
            assert got[k] == float(s[k]) or (np.isnan(got[k]) and np.isnan(float(s[k]))), k
    _check(got, s, 1e-4)
