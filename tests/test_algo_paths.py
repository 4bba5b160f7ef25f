"""Checkpoint / reward-curve file names and keys follow the reference's formats
(Algo_PPO.loading/saving :935-1001, reward curves :908-916) and its shipped files."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mh-ppo_amd")]


class _V:
    variant = "scalable"


def _algo(num_algo, total_loop):
    from mhppo.algo import Algo_PPO
    a = Algo_PPO.__new__(Algo_PPO)
    a.venv, a.num_algo, a.total_loop = _V(), num_algo, total_loop
    return a


def test_weight_paths_match_reference_format():
    a = _algo(111, 1000)
    ref = "load_model/weights/pappo-scalable-coop-cross-{num_algo:02d}-actor-step-{epoch:03d}0.pth"
    assert a._path("cross", "actor", 111, 1000) == ref.format(num_algo=111, epoch=100)
    # the shipped checkpoint names (load_model/weights/*.pth) come out of the same format
    assert os.path.basename(a._path("choice", "critic", 111, 1000)) == "pappo-scalable-coop-choice-111-critic-step-1000.pth"


def test_reward_curve_paths_match_reference_format():
    a = _algo(111, 1000)
    ref = "load_model/parameters/pappo-scalable-coop-{num_algo:02d}-{name}-step-{epoch:03d}000.npy"
    for name in ("reward_cross", "reward_wait", "reward_choice", "scenario_balance"):
        assert a._curve_path(name) == ref.format(num_algo=111, epoch=1, name=name)


def test_env_checkpoint_layout_version_is_checked():
    import pytest
    from mhppo.env import VecCrosswalk

    class _E:
        STATE_LAYOUT = VecCrosswalk.STATE_LAYOUT

        def _cfg_key(self):
            return [0]
    for old in ({"cfg": [0], "layout": VecCrosswalk.STATE_LAYOUT - 1, "blob": None},):
        with pytest.raises(ValueError, match="state layout"):
            VecCrosswalk.load_state_dict(_E(), old)


def test_env_checkpoint_keyless_layout_inferred_from_size():
    # r02 / r03 checkpoints carry no "layout" key: an r03 blob has the layout-2 size, an r02 blob not
    import torch
    from mhppo.env import VecCrosswalk
    blob = torch.zeros(1000, dtype=torch.uint8)
    assert VecCrosswalk.blob_layout({"cfg": [0], "blob": blob}, 1000) == 2
    assert VecCrosswalk.blob_layout({"cfg": [0], "blob": blob}, 1200) == 1
    assert VecCrosswalk.blob_layout({"cfg": [0], "blob": None}, 1000) == 1
    assert VecCrosswalk.blob_layout({"cfg": [0], "layout": 7, "blob": blob}, 1000) == 7


def test_curves_flush_pending_entries():
    import torch
    a = _algo(1, 0)
    a.ep_reward_cross, a.ep_reward_wait, a.ep_reward_choice, a.ep_scenario_balance = [], [], [], []

    class _Ev:
        def synchronize(self):
            pass
    a._pending_curves = [(torch.tensor([2.0, 6.0, 3.0], dtype=torch.float64), _Ev(), 2.0, 3.0, 1.0)]
    c, w, d, b = a.curves()
    assert (c, w, d, b) == ([1.0], [2.0], [3.0], [[2, 3]]) and a._pending_curves == []
