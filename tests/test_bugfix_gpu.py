"""Opt-in bug-fix mode on the GPU: the fixed scalable lane mapping matches
the oracle's; the per-row choice loss in the fused kernel matches torch autograd of the
standard per-row PPO surrogate; the fixed bucketing follows each car's closest pedestrian."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fixed_lanes_env_matches_oracle():
    import oracle
    from mhppo.env import VecCrosswalk
    N = 64
    venv = VecCrosswalk("scalable", N, 8, 1, 4, seed_base=77, fix_scalable_lanes=True)
    envs = [oracle.OracleEnv("scalable", 8, 1, 4, seed=77 + e, flags=1) for e in range(N)]
    np.testing.assert_array_equal(venv.reset().cpu().numpy(), np.stack([o.reset() for o in envs]))
    rng = np.random.default_rng(0)
    for t in range(80):
        a = np.concatenate([rng.uniform(-4.5, 2.5, (N, 8)).astype(np.float32).astype(np.float64),
                            rng.choice([-1.0, 1.0], (N, 8))], 1)
        obs, rew, rl, done = venv.step(torch.from_numpy(a))
        ref = [o.step(a[e]) for e, o in enumerate(envs)]
        np.testing.assert_allclose(obs.cpu().numpy(), np.stack([r[0] for r in ref]), rtol=1e-6, atol=1e-4)
        np.testing.assert_allclose(rew.cpu().numpy(), np.stack([r[1] for r in ref]), rtol=1e-9, atol=1e-9)
    mt, mti = venv.get_rng()
    for e in (0, 17, 63):
        assert int(mti[e]) % 624 == envs[e].rng_state()[1] % 624


@pytest.mark.parametrize("M,dc", [(33, 17), (5000, 27)])
def test_per_row_choice_loss_matches_autograd(M, dc):
    from mhppo import ppo
    from mhppo.models import Model_PPO
    torch.manual_seed(M)
    actor, critic = Model_PPO(dc, 2, 2).cuda(), Model_PPO(dc, 1, 0).cuda()
    obs = (torch.randn(M, dc) * 2).cuda()
    ret = (torch.randn(M) * 3 - 5).cuda()
    act = (torch.rand(M) < 0.4).float().cuda()
    lp = torch.log(torch.rand(M) * 0.8 + 0.1).cuda()
    m = float(M)
    gc, sc, V = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m)
    st = sc[1:3].clone()
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CHOICE, actor, obs, ret, V, act, lp, st, None, m_global=m)
    # torch: standard per-row PPO surrogate on the same normalised advantage
    adv = ppo.k_adv_normalize(ret, V, st, m).double()
    probs = actor(obs).reshape(-1, 2)
    pn = probs / probs.sum(-1, keepdim=True)
    eps = torch.finfo(torch.float32).eps
    lpa = torch.log(pn.clamp(eps, 1 - eps)).gather(1, act.long().reshape(-1, 1)).reshape(-1)
    r = torch.exp(lpa.double() - lp.double())
    loss = (-torch.minimum(r * adv, r.clamp(0.8, 1.2) * adv)).mean()
    gat = torch.cat([g.reshape(-1) for g in torch.autograd.grad(loss, list(actor.parameters()))]).float()
    # the choice kernel reports the loss sum scaled by M^2 (as the M x M broadcast mode does)
    assert abs(float(sa[0].detach()) / (m * m) - float(loss.detach())) <= 1e-5 * abs(float(loss.detach())) + 1e-7
    torch.testing.assert_close(ga, gat, rtol=0, atol=1e-4 * float(gat.abs().max()) + 1e-9)


def test_fixed_bucket_follows_closest_pedestrian():
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU, bucket_segments
    torch.manual_seed(3)
    venv = VecCrosswalk("coop", 512, 2, 3, 2, seed_base=9)
    ro = RolloutGPU(venv)
    nets = (Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda(), Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda(),
            Model_PPO(ro.dc, 2, 2).cuda())
    b = ro.collect(*nets, seed=1, iteration=0)
    c_ref, w_ref, _ = bucket_segments(b)
    c_fix, w_fix, _ = bucket_segments(b, fix_bucket=True)
    a_car = b.a_d.gather(2, b.closest.long().unsqueeze(2)).squeeze(2)  # [N, S]
    n_cross = int(((a_car == 0) & b.exist.bool()).sum()) * b.T
    assert c_fix["obs"].shape[0] == n_cross and c_fix["obs"].shape[0] + w_fix["obs"].shape[0] == \
        c_ref["obs"].shape[0] + w_ref["obs"].shape[0]
    assert c_fix["obs"].shape[0] != c_ref["obs"].shape[0]  # P = 3: the flat index picks other decisions
