"""Checkpoint/resume: train, checkpoint, keep training; a fresh Algo_PPO
(different init) that loads the checkpoint and trains the same number of iterations ends
bit-identical — weights, Adam moments, every env's random stream, reward curves."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _algo(seed):
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    venv = VecCrosswalk("coop", 512, 2, 1, 2, seed_base=3)
    torch.manual_seed(seed)
    return Algo_PPO(Model_PPO, venv, verbose=False)


def _snap(a):
    params = [p.detach().clone() for n in a.nets() for p in n.parameters()]
    moments = [s["exp_avg"].clone() for o in a._optimizers().values() for s in o.state_dict()["state"].values()]
    mt, mti = a.venv.get_rng()
    return params, moments, mt.clone(), mti.clone(), list(a.ep_reward_cross), a.total_loop


def test_resume_is_bit_identical(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    a = _algo(0)
    a.train(1)
    a.save_checkpoint("ck.pt")
    a.train(2)
    ref = _snap(a)
    b = _algo(1234)
    b.load_checkpoint("ck.pt")
    b.train(2)
    got = _snap(b)
    for x, y in zip(ref[0] + ref[1], got[0] + got[1]):
        assert torch.equal(x, y)
    assert torch.equal(ref[2], got[2]) and torch.equal(ref[3], got[3])
    assert ref[4] == got[4] and ref[5] == got[5] == 3
    assert (tmp_path / "load_model" / "parameters").is_dir()  # train() wrote the reward curves (:908-916)


def test_keyless_env_checkpoint_is_refused():
    # r02 / r03 env checkpoints carry no "layout" key; their blobs (layouts 1 / 2) lack the cars'
    # line / existence bytes of layout 3 (r06), so this build refuses them instead of misreading them
    from mhppo.env import VecCrosswalk
    v = VecCrosswalk("coop", 128, 2, 1, 2, seed_base=5)
    v.reset()
    v.step(torch.zeros(128, 2 * v.n_slots, device=v.device))
    sd = v.state_dict()
    del sd["layout"]
    w = VecCrosswalk("coop", 128, 2, 1, 2, seed_base=5)
    with pytest.raises(ValueError, match="state layout"):
        w.load_state_dict(sd)
    sd["layout"] = VecCrosswalk.STATE_LAYOUT  # the same blob with its layout key resumes exactly
    w.load_state_dict(sd)
    assert torch.equal(v.get_rng()[0], w.get_rng()[0]) and torch.equal(v.get_rng()[1], w.get_rng()[1])
    assert torch.equal(v.get_state(), w.get_state())
