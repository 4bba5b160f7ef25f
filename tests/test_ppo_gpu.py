"""HIP PPO-update kernels (advantage stats/normalise, clip surrogates, MSE) vs the
reference's own update (tests/golden/ppo_update.npz) — losses within 1e-4 relative,
updated weights within 1e-5 absolute after each of 3 epochs; returns scan bit-exact
vs the float64 oracle scan."""
import os

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden", "ppo_update.npz")
pytestmark = pytest.mark.gpu


def _net(g, head, kind, dc=None):
    from mhppo.models import Model_PPO
    if head == "c":
        n = Model_PPO(13, 1, 1, mean=-1.0, std=3.0) if kind == "actor" else Model_PPO(13, 1, 0)
    else:
        n = Model_PPO(dc, 2, 2) if kind == "actor" else Model_PPO(dc, 1, 0)
    pre = f"{head}_init_{kind}_"
    n.load_state_dict({k[len(pre):]: torch.tensor(g[k]) for k in g.files if k.startswith(pre)})
    return n.cuda()


@pytest.mark.parametrize("head", ["c", "d"])
def test_update_matches_reference(head):
    from mhppo import ppo
    g = np.load(G)
    dc = g["d_obs"].shape[1]
    actor, critic = _net(g, head, "actor", dc), _net(g, head, "critic", dc)
    oa = torch.optim.Adam(actor.parameters(), 3e-4)
    oc = torch.optim.Adam(critic.parameters(), 1e-3)
    obs = torch.tensor(g[f"{head}_obs"]).cuda()
    act = torch.tensor(g[f"{head}_act"]).cuda()
    lp = torch.tensor(g[f"{head}_logp"]).cuda()
    rt = torch.tensor(g[f"{head}_rtgs"]).cuda()
    M = float(obs.shape[0])
    for ep in range(3):
        if head == "c":
            la, lc = ppo.train_model_c(actor, critic, oa, oc, obs, act, lp, rt, M)
            la = float(la.item()) / M
        else:
            counts = torch.tensor([(act == 0).sum().item(), (act == 1).sum().item()], dtype=torch.float64).cuda()
            la, lc = ppo.train_model_d(actor, critic, oa, oc, obs, act, lp, rt, M, counts)
            la = float(la.item()) / (M * M)
        lc = float(lc.item()) / M
        ref_a, ref_c = g[f"{head}_losses"][ep]
        assert abs(la - ref_a) <= 1e-4 * max(1.0, abs(ref_a)), (ep, la, ref_a)
        assert abs(lc - ref_c) <= 1e-4 * max(1.0, abs(ref_c)), (ep, lc, ref_c)
        for kind, net in (("actor", actor), ("critic", critic)):
            for k, v in net.state_dict().items():
                np.testing.assert_allclose(v.cpu().numpy(), g[f"{head}_ep{ep}_{kind}_{k}"], rtol=0, atol=1e-5,
                                           err_msg=f"{head} ep{ep} {kind} {k}")


def test_returns_scan_bit_exact():
    from mhppo.rollout import returns_scan
    from oracle import ppo_ref
    rng = np.random.default_rng(0)
    rew = torch.tensor(rng.normal(-10, 5, size=(1000, 80)))
    ref = ppo_ref.returns_scan(rew)
    out = returns_scan(rew.cuda()).cpu()
    assert torch.equal(out, ref)


def test_returns_scan_time_major_bit_exact():
    """The rollout's time-major records [T, N, S]: column scan == the oracle's row scan."""
    from mhppo.rollout import returns_scan_tm
    from oracle import ppo_ref
    rng = np.random.default_rng(1)
    rew = torch.tensor(rng.normal(-10, 5, size=(777, 80)))
    ref = ppo_ref.returns_scan(rew)
    out = returns_scan_tm(rew.t().contiguous().reshape(80, 7, 111).cuda()).cpu().reshape(80, 777).t()
    assert torch.equal(out, ref)


def test_philox_noise_moments():
    from mhppo import _lib
    n = 1 << 20
    x = torch.empty(n, device="cuda")
    _lib.check(_lib.lib().mhppo_philox_normal(7, 0, _lib.ptr(x), n, _lib.stream_ptr()))
    assert abs(float(x.mean())) < 5e-3 and abs(float(x.std()) - 1) < 5e-3
    u = torch.empty(n, device="cuda")
    _lib.check(_lib.lib().mhppo_philox_uniform(7, 0, _lib.ptr(u), n, _lib.stream_ptr()))
    assert 0 <= float(u.min()) and float(u.max()) < 1 and abs(float(u.mean()) - 0.5) < 2e-3
    # counter-based: a shifted window reproduces the same draws
    y = torch.empty(1000, device="cuda")
    _lib.check(_lib.lib().mhppo_philox_normal(7, 5000, _lib.ptr(y), 1000, _lib.stream_ptr()))
    assert torch.equal(y, x[5000:6000])


def _close_grad(g, gt):
    torch.testing.assert_close(g, gt, rtol=0, atol=1e-4 * float(gt.abs().max()) + 1e-9)


def _critic_pass(ppo, critic, obs, ret, m, exact=False):
    gc, sc, V = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m, exact=exact)
    Vt = torch.squeeze(critic(obs), -1)
    torch.testing.assert_close(V, Vt.detach(), rtol=1e-5, atol=1e-5)
    dv, lc = ppo.k_mse(Vt, ret, m)
    st = ppo.k_adv_stats(ret, Vt)
    gct = torch.cat([g.reshape(-1) for g in torch.autograd.grad(Vt, list(critic.parameters()), dv)])
    assert abs(float(sc[0]) - float(lc[0])) <= 1e-5 * abs(float(lc[0])) + 1e-6
    torch.testing.assert_close(sc[1:3], st, rtol=1e-5, atol=1e-3)
    _close_grad(gc, gct)
    return Vt, st


@pytest.mark.parametrize("M", [1, 31, 33, 1000, 70001])
def test_fused_cont_grads_vs_autograd(M):
    """mhppo_mlp_train kinds 0/1 (fused MFMA forward/backward, 13 inputs, DMA-prefetch
    path) vs torch autograd of the same losses on the same weights: V 1e-5, loss sums
    1e-5 rel, gradients within 1e-4 of the gradient's max-abs (fp32 summation order)."""
    from mhppo import ppo
    from mhppo.models import Model_PPO
    torch.manual_seed(M)
    actor = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    critic = Model_PPO(13, 1, 0).cuda()
    obs = (torch.randn(M, 13) * 3).cuda()
    ret = (torch.randn(M) * 8 - 20).cuda()
    act = (torch.randn(M) - 1).cuda()
    lp = (torch.randn(M) * 0.3 - 0.9).cuda()
    m = float(M) if M > 1 else 2.0  # unbiased std needs m > 1
    Vt, st = _critic_pass(ppo, critic, obs, ret, m)
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CONT, actor, obs, ret, Vt, act, lp, st, m_global=m)
    mu = torch.squeeze(actor(obs), -1)
    adv = ppo.k_adv_normalize(ret, Vt, st, m)
    dmu, la = ppo.k_ppo_cont(mu, act, lp, adv, m)
    gat = torch.cat([g.reshape(-1) for g in torch.autograd.grad(mu, list(actor.parameters()), dmu)])
    assert abs(float(sa[0]) - float(la[0])) <= 1e-5 * abs(float(la[0])) + 1e-6
    _close_grad(ga, gat)


@pytest.mark.parametrize("M,dc,exact", [(1, 12, False), (45, 17, False), (4096, 27, False), (20001, 30, False),
                                        (333, 32, False), (70, 54, False), (65536, 54, False), (1000, 40, False),
                                        (257, 64, False), (20001, 30, True), (4097, 16, True), (100003, 17, False),
                                        (64, 16, False), (65, 31, False), (524288, 54, False), (4099, 36, False)])
def test_fused_choice_grads_vs_autograd(M, dc, exact):
    """mhppo_mlp_train kinds 0/2 on choice-head shapes (dc = 12..64 inputs — 54 is the
    scalable 8-slot driver's choice head, 2-way softmax, O(M) count-weighted surrogate) vs
    torch autograd + the HIP choice-loss kernel.  dc <= 54 runs on the bf16x3 split kernel
    (K = 16 / 32 / 64 geometries), exact=True and dc > 54 on the f32-MFMA one."""
    from mhppo import ppo
    from mhppo.models import Model_PPO
    torch.manual_seed(M + dc)
    actor = Model_PPO(dc, 2, 2).cuda()
    critic = Model_PPO(dc, 1, 0).cuda()
    obs = (torch.randn(M, dc) * 2).cuda()
    ret = (torch.randn(M) * 3 - 5).cuda()
    act = (torch.rand(M) < 0.4).float().cuda()
    lp = torch.log(torch.rand(M) * 0.8 + 0.1).cuda()
    m = float(M) if M > 1 else 2.0
    counts = torch.tensor([float((act == 0).sum()), float((act == 1).sum())], dtype=torch.float64).cuda()
    Vt, st = _critic_pass(ppo, critic, obs, ret, m, exact)
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CHOICE, actor, obs, ret, Vt, None, lp, st, counts, m_global=m, exact=exact)
    probs = actor(obs).reshape(-1, 2)
    adv = ppo.k_adv_normalize(ret, Vt, st, m)
    dp, la = ppo.k_ppo_choice(probs, lp, adv, counts, m)
    gat = torch.cat([g.reshape(-1) for g in torch.autograd.grad(probs, list(actor.parameters()), dp)])
    assert abs(float(sa[0]) - float(la[0])) <= 1e-5 * abs(float(la[0])) + 1e-6
    _close_grad(ga, gat)


def test_philox_normal_2d_equals_rows():
    """The one-launch rollout noise (mhppo_philox_normal_2d) is bit-identical to one
    mhppo_philox_normal call per step (the counters of rollout.py's draw_noise)."""
    from mhppo import _lib
    L = _lib.lib()
    rows, cols, stride, off = 5, 1000, 1 << 40, (1 << 40) + 777
    a = torch.empty((rows, cols), device="cuda")
    _lib.check(L.mhppo_philox_normal_2d(12345, off, stride, _lib.ptr(a), rows, cols, _lib.stream_ptr()))
    b = torch.empty((rows, cols), device="cuda")
    for r in range(rows):
        _lib.check(L.mhppo_philox_normal(12345, off + r * stride, _lib.ptr(b[r]), cols, _lib.stream_ptr()))
    assert torch.equal(a, b)


def test_adam_steps_bit_identical_to_per_optimizer_steps():
    """ppo.adam_steps (all six nets' fused Adam steps batched by hyper-parameters) gives the same
    parameters and moments bit for bit as one o.step() per optimiser, over several steps."""
    from mhppo import ppo
    from mhppo.models import Model_PPO

    def make():
        torch.manual_seed(3)
        nets = [Model_PPO(13, 1, 1, mean=-1.0, std=3.0), Model_PPO(13, 1, 0), Model_PPO(13, 1, 1, mean=-1.0, std=3.0),
                Model_PPO(13, 1, 0), Model_PPO(30, 2, 2), Model_PPO(30, 1, 0)]
        nets = [n.cuda() for n in nets]
        lrs = [3e-4, 1e-3, 3e-4, 1e-3, 1e-4, 2e-3]
        opts = [torch.optim.Adam(n.parameters(), lr, fused=True) for n, lr in zip(nets, lrs)]
        return nets, opts

    runs = []
    for batched in (False, True):
        nets, opts = make()
        g = torch.Generator(device="cuda").manual_seed(7)
        for _ in range(4):
            for n in nets:
                for p in n.parameters():
                    p.grad = torch.randn(p.shape, device="cuda", generator=g)
            if batched:
                ppo.adam_steps(opts)
            else:
                for o in opts:
                    o.step()
        runs.append(([p.detach().cpu() for n in nets for p in n.parameters()],
                     [o.state[p]["exp_avg_sq"].cpu() for o, n in zip(opts, nets) for p in n.parameters()]))
    for a, b in zip(runs[0][0] + runs[0][1], runs[1][0] + runs[1][1]):
        assert torch.equal(a, b)
