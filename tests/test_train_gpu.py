"""One whole training iteration, end to end, against the reference's own Algo_PPO.train.

Fixtures tests/golden/train_<name>.npz (tests/golden/gen/make_train_golden.py): the
reference driver (coop 2/1/2: Coop-MH-PPO.ipynb cell 0; scalable 8/1/4 with its 54-wide
choice head: Coop-MH-PPO-scalable.py) collects one episode in each of 16 envs (per-env
CPython streams, recorded MVN / Categorical draws), buckets them (:489-507), and runs
Algo_PPO.train(1) unmodified: futur_rewards, 10 epochs of train_model_c (cross, wait),
10 epochs of train_model_d.

Here the product Algo_PPO does the same iteration on the GPU: rollout.reset ->
iterations_rand (replaying the recorded draws) -> bucket_segments -> update (10 joint
epochs of the fused kernels).  Checked:
  * the product's bucketed batches vs the reference's: row counts and choice actions
    exact, features within 1e-4 (float32 ulp at 300 m), actions / log-probs within 2e-5,
    returns within 1e-4;
  * update() on the reference's own batch: all six nets within 1e-5 of the reference's
    weights after 10 + 10 epochs (pins the update orchestration exactly);
  * the whole product iteration (its own batch): all six nets within 1e-4, reward curves
    within 1e-5 relative.
"""
import glob
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "train_*.npz")))
NETS = ("actor_net_cross", "actor_net_wait", "actor_net_choice", "critic_net_cross", "critic_net_wait",
        "critic_net_choice")


def _algo(g, exact_f32=False):
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    venv = VecCrosswalk(str(g["variant"]), int(g["E"]), int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"]),
                        seed_base=int(g["seed_base"]))
    algo = Algo_PPO(Model_PPO, venv, verbose=True, exact_f32=exact_f32)
    for n in NETS:
        pre = f"{n}_init_"
        getattr(algo, n).load_state_dict({k[len(pre):]: torch.tensor(g[k]) for k in g.files if k.startswith(pre)})
    return algo


def _replay(g):
    return torch.from_numpy(g["a_d"]), torch.from_numpy(g["eps"])


def _check_nets(algo, g, tol):
    for n in NETS:
        for k, v in getattr(algo, n).state_dict().items():
            np.testing.assert_allclose(v.cpu().numpy(), g[f"{n}_final_{k}"], rtol=0, atol=tol, err_msg=f"{n}.{k}")


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[6:-4] for f in FILES])
def test_bucketed_batch_matches_reference(path):
    g = np.load(path)
    algo = _algo(g)
    fc, et = _replay(g)
    algo.rollout.reset()
    algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice,
                                 forced_choice=fc, eps_tape=et)
    r = algo.rollout
    for h, b in (("cross", r.cross), ("wait", r.wait)):
        assert b["obs"].shape[0] == g["obs_" + h].shape[0], h
        # features are float32 differences of positions up to ~300 m (f32 ulp 3e-5 there): a last-bit
        # difference of a float64 position (device vs glibc libm) moves such a feature by one ulp
        np.testing.assert_allclose(b["obs"].cpu().numpy(), g["obs_" + h], rtol=2e-5, atol=1e-4, err_msg=h)
        np.testing.assert_allclose(b["act"].cpu().numpy(), g["act_" + h], rtol=2e-5, atol=2e-5, err_msg=h)
        np.testing.assert_allclose(b["logp"].cpu().numpy(), g["logp_" + h], rtol=2e-5, atol=2e-5, err_msg=h)
        np.testing.assert_allclose(b["ret"].cpu().numpy(), g["rtgs_" + h], rtol=1e-4, atol=1e-4, err_msg=h)
    d = r.choice
    assert d["obs"].shape == g["obs_choice"].shape
    np.testing.assert_array_equal(d["act"].cpu().numpy(), g["act_choice"].astype(np.int32))
    np.testing.assert_allclose(d["obs"].cpu().numpy(), g["obs_choice"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(d["logp"].cpu().numpy(), g["logp_choice"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(d["ret"].cpu().numpy(), g["rtgs_choice"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("exact", [False, True], ids=["bf16x3", "exact_f32"])
@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[6:-4] for f in FILES])
def test_update_on_reference_batch_matches_reference(path, exact):
    """Algo_PPO.update (10 joint epochs, fused kernels, bucketed collectives) on the
    reference's own batch -> the reference's final weights of all six nets; on the default
    split-precision train kernel and on the exact f32-MFMA one (Algo_PPO(exact_f32=True))."""
    g = np.load(path)
    algo = _algo(g, exact)
    dev = algo.venv.device
    t = lambda k, dt=torch.float32: torch.tensor(g[k], dtype=dt, device=dev)  # noqa: E731
    r = algo.rollout
    r.cross = dict(obs=t("obs_cross"), act=t("act_cross"), logp=t("logp_cross"), ret=t("rtgs_cross"))
    r.wait = dict(obs=t("obs_wait"), act=t("act_wait"), logp=t("logp_wait"), ret=t("rtgs_wait"))
    r.choice = dict(obs=t("obs_choice"), act=t("act_choice", torch.int32), logp=t("logp_choice"),
                    ret=t("rtgs_choice"))
    m_c, m_w, m_d = algo.update()
    assert (m_c, m_w) == tuple(float(x) for x in g["scenario_balance"][0])
    torch.cuda.synchronize()
    _check_nets(algo, g, 1e-5)


@pytest.mark.parametrize("path", FILES, ids=[os.path.basename(f)[6:-4] for f in FILES])
def test_train_iteration_matches_reference(path, tmp_path, monkeypatch):
    """Algo_PPO.train(1) with the recorded draws replayed: rollout, bucketing, returns,
    update, reward curves — the product iteration against the reference's."""
    g = np.load(path)
    algo = _algo(g)
    monkeypatch.chdir(tmp_path)
    algo.verbose = False
    algo.train(1, replay=[_replay(g)])
    torch.cuda.synchronize()
    assert algo.ep_scenario_balance == g["scenario_balance"].tolist()
    for k in ("ep_reward_cross", "ep_reward_wait", "ep_reward_choice"):
        np.testing.assert_allclose(np.array(getattr(algo, k)), g[k], rtol=1e-5, atol=1e-6, err_msg=k)
    _check_nets(algo, g, 1e-4)
    assert os.path.exists(tmp_path / "load_model" / "parameters")
