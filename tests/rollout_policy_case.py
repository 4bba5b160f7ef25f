"""The policy bit-identity case of tests/test_rollout_gpu.py (shared with its worker process,
tests/valu_policy_worker.py): one 300-env episode with seeded random-init actors."""


def run_case(case, valu_policy):
    import torch

    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    v, nc, npd, nl = case
    ro = RolloutGPU(VecCrosswalk(v, 300, nc, npd, nl, seed_base=777), valu_policy=valu_policy, parts=1)
    torch.manual_seed(5)
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    ad = Model_PPO(ro.dc, 2, 2).cuda()
    b = ro.collect(ac, aw, ad, seed=2, iteration=1, graph=False)
    out = {k: getattr(b, k).cpu().numpy() for k in ("feat_d", "a_d", "logp_d", "closest", "exist", "obs_c", "act",
                                                      "logp", "rew", "ep_min")}
    return out
