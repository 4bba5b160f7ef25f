"""MHPPO_ENAN: a NaN policy output sampled in the rollout fails loudly, as the reference's
torch.distributions argument validation does (Categorical(probs) :409,
MultivariateNormal(loc) :451 raise ValueError on NaN)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _algo():
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    return Algo_PPO(Model_PPO, VecCrosswalk("coop", 64, 2, 1, 2, seed_base=3), verbose=False)


@pytest.mark.parametrize("head", ["actor_net_choice", "actor_net_cross"])
def test_nan_policy_output_raises(head):
    from mhppo._lib import MhppoNaNError
    algo = _algo()
    with torch.no_grad():
        getattr(algo, head).layer4.bias.fill_(float("nan"))
    if head == "actor_net_cross":  # every car on the cross head
        forced = torch.zeros((64, 2, 1), dtype=torch.int32)
    else:
        forced = None
    with pytest.raises(ValueError) as ei:
        algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice,
                                     forced_choice=forced, eps_tape=None if forced is None else torch.zeros(80, 64, 2))
    assert isinstance(ei.value, MhppoNaNError)
    # the flag was cleared: a clean rollout after fixing the weights passes
    with torch.no_grad():
        getattr(algo, head).layer4.bias.zero_()
    algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice)


def test_clean_rollout_has_no_nan_flag():
    algo = _algo()
    algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice)
    assert int(algo.rollout.gpu.status.item()) == 0


def test_compact_records_rejected_for_a_fixed_slot_env():
    """include/mhppo.h mhppo_rollout_bufs.rec_of: the scalable env's layout only (the kernels of the
    other variants are compiled without it), so mhppo_rollout_begin refuses it elsewhere."""
    import ctypes
    from mhppo._lib import MhppoError
    algo = _algo()
    g = algo.rollout.gpu
    N, S = g.a_d.shape[0], g.a_d.shape[1]
    buf = torch.zeros(N * S + N + 1, dtype=torch.int32, device=g.a_d.device)
    g._bufs.rec_of = ctypes.c_void_p(buf.data_ptr())
    try:
        with pytest.raises(MhppoError, match="scalable"):
            algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice)
    finally:
        g._bufs.rec_of = None
    algo.rollout.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice)
