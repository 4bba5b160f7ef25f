"""The fused training kernel at the bench's scale: one epoch of the critic and of the
continuous actor (mhppo_mlp_train kinds 0 and 1) on the bench workload's real bucketed
batch (4cars 4/1/2, 65 536 envs x 80 steps -> the cross head's ~10.5 M rows, 2 048
per-wave partial gradients folded by k_grad_stage1/2) — on the default split-precision kernel and on
the exact f32-MFMA one (exact_f32) — against a float64 torch autograd of
the same losses (train_model_c, Coop-MH-PPO-scalable.py:778-815) on the same weights.
Bar: max|dg| <= 1e-4 max|g| for every gradient; the loss sums within 1e-6 relative (the
advantage sum, which cancels, within 1e-6 of sum|A|)."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


class _F64(torch.nn.Module):
    """Model_PPO's forward (Coop-MH-PPO-scalable.py:70-93) in float64 on the same weights."""

    def __init__(self, net):
        super().__init__()
        self.kind, self.mean, self.std = net.model_type, net.mean, net.std
        self.layers = torch.nn.ModuleList()
        for lay in (net.layer1, net.layer2, net.layer3, net.layer4):
            m = torch.nn.Linear(lay.in_features, lay.out_features, dtype=torch.float64, device=lay.weight.device)
            with torch.no_grad():
                m.weight.copy_(lay.weight.double())
                m.bias.copy_(lay.bias.double())
            self.layers.append(m)

    def forward(self, x):
        for m in self.layers[:3]:
            x = torch.relu(m(x))
        y = self.layers[3](x)
        return torch.tanh(y) * self.std + self.mean if self.kind == 1 else y


def _f64(net):
    return _F64(net)


def _flat_grad(net, loss):
    gs = torch.autograd.grad(loss, [p for m in net.layers for p in (m.weight, m.bias)])
    return torch.cat([g.reshape(-1) for g in gs])


@pytest.mark.parametrize("exact", [False, True], ids=["bf16x3", "exact_f32"])
def test_fused_epoch_at_bench_scale_vs_float64_autograd(exact):
    from mhppo import ppo
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import bucket_segments
    venv = VecCrosswalk("4cars", 65536, 4, 1, 2, seed_base=0)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
    with torch.no_grad():
        batch = algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0)
    c, _, _ = bucket_segments(batch)
    obs, act, lp, ret = c["obs"], c["act"], c["logp"], c["ret"]
    M = obs.shape[0]
    assert M > 5_000_000
    m = float(M)
    # ---- critic pass (kind 0): MSE gradient, (sum (V-G)^2, sum A, sum A^2), V
    critic, actor = algo.critic_net_cross, algo.actor_net_cross
    gc, sc, V = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m, exact=exact)
    gc, sc = gc.clone(), sc.clone()
    c64 = _f64(critic)
    V64 = torch.squeeze(c64(obs.double()), -1)
    G = ret.double()
    mse = ((V64 - G) ** 2).sum()
    g64 = _flat_grad(c64, mse / m)
    assert float((gc.double() - g64).abs().max()) <= 1e-4 * float(g64.abs().max())
    assert abs(float(sc[0]) - float(mse)) <= 1e-6 * float(mse)
    A64 = G - V64
    assert abs(float(sc[1]) - float(A64.sum())) <= 1e-6 * float(A64.abs().sum())
    assert abs(float(sc[2]) - float((A64 * A64).sum())) <= 1e-6 * float((A64 * A64).sum())
    # ---- actor pass (kind 1): clip surrogate against A normalised with the epoch's critic
    stats = sc[1:3].clone()
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CONT, actor, obs, ret, V, act, lp, stats, m_global=m, exact=exact)
    ga = ga.clone()
    a64 = _f64(actor)
    mean = float(stats[0]) / m
    std = ((float(stats[1]) - float(stats[0]) * mean) / (m - 1)) ** 0.5
    A = ((G - V.double()) - mean) / (std + 1e-10)
    mu = torch.squeeze(a64(obs.double()), -1)
    x = (act.double() - mu) / (0.5 ** 0.5)
    logp = -0.5 * (x * x + torch.log(torch.tensor(2 * torch.pi, dtype=torch.float64))) - 0.5 * torch.log(
        torch.tensor(0.5, dtype=torch.float64))
    r = torch.exp(logp - lp.double())
    surr = -torch.minimum(r * A, r.clamp(0.8, 1.2) * A)
    g64 = _flat_grad(a64, surr.sum() / m)
    assert float((ga.double() - g64).abs().max()) <= 1e-4 * float(g64.abs().max())
    assert abs(float(sa[0]) - float(surr.sum())) <= 1e-6 * float(surr.abs().sum())


def _follow(r, A):
    """Which rows' gradient follows r in -min(rA, clamp(r, .8, 1.2) A) (torch's tie rule: the
    in-range tie gives A): A > 0 up to r = 1.2, A < 0 from r = 0.8 on."""
    return torch.where(A > 0, r <= 1.2, torch.where(A < 0, r >= 0.8, torch.zeros_like(r, dtype=torch.bool)))


@pytest.mark.parametrize("exact", [False, True], ids=["bf16x3", "exact_f32"])
def test_actor_clip_at_bench_scale_vs_float64_autograd(exact):
    """The continuous actor pass on the bench's 10.5 M-row cross bucket with the actor's weights
    moved away from the ones that produced logp_old (as after some epochs), so the ratio spreads
    well past the clip bounds 0.8 / 1.2 (Coop-MH-PPO-scalable.py:803-806): the kernel's gradient
    against a float64 autograd with the reference's float64 ratio, at the 1e-4 max|g| bar.
    The kernel takes the clip branch from the float64 difference lp - logp_old
    (rollout_dev.h surr_and_grad_fd); the test also counts, on torch's float32 lp of the same
    weights, the rows whose branch a float32 ratio expf(lp - logp_old) would flip against the
    float64 one, and the rows whose branch float32 lp itself moves against float64 lp (present in
    the reference too, whose actor is float32) — printed, recorded in DESIGN.md §5."""
    import math
    from mhppo import ppo
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import bucket_segments
    venv = VecCrosswalk("4cars", 65536, 4, 1, 2, seed_base=0)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
    with torch.no_grad():
        batch = algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0)
    c, _, _ = bucket_segments(batch)
    obs, act, lp, ret = c["obs"], c["act"], c["logp"], c["ret"]
    M = obs.shape[0]
    assert M > 5_000_000
    m = float(M)
    critic, actor = algo.critic_net_cross, algo.actor_net_cross
    _, sc, V = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m, exact=exact)
    stats = sc[1:3].clone()
    V = V.clone()
    g = torch.Generator(device=obs.device).manual_seed(1)
    with torch.no_grad():  # the actor after some updates: every weight moved, the output shifted
        for prm in actor.parameters():
            prm.add_(torch.randn(prm.shape, generator=g, device=prm.device) * 0.1 * prm.abs().mean())
        actor.layer4.bias.add_(0.1)
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CONT, actor, obs, ret, V, act, lp, stats, m_global=m, exact=exact)
    ga, sa = ga.clone(), sa.clone()
    a64 = _f64(actor)
    mean = float(stats[0]) / m
    std = ((float(stats[1]) - float(stats[0]) * mean) / (m - 1)) ** 0.5
    A = ((ret.double() - V.double()) - mean) / (std + 1e-10)
    half_logdet = 0.5 * math.log(0.5)
    mu = torch.squeeze(a64(obs.double()), -1)
    x = (act.double() - mu) / (0.5 ** 0.5)
    logp = -0.5 * (x * x + math.log(2 * math.pi)) - half_logdet
    r = torch.exp(logp - lp.double())
    clipped = float(((r < 0.8) | (r > 1.2)).double().mean())
    assert 0.2 < clipped < 0.95, f"ratio spread: {clipped:.3f} of rows outside [0.8, 1.2]"
    surr = -torch.minimum(r * A, r.clamp(0.8, 1.2) * A)
    g64 = _flat_grad(a64, surr.sum() / m)
    err = float((ga.double() - g64).abs().max()) / float(g64.abs().max())
    assert err <= 1e-4, err
    assert abs(float(sa[0]) - float(surr.sum())) <= 1e-6 * float(surr.abs().sum())
    # branch flips, on torch's float32 forward of the same weights (the kernel's lp is not exported)
    with torch.no_grad():
        mu32 = torch.squeeze(actor(obs), -1)
        x32 = (act - mu32) * torch.tensor(1.0 / 0.5 ** 0.5, dtype=torch.float32)
        lp32 = (-0.5 * (x32 * x32 + torch.tensor(math.log(2 * math.pi), dtype=torch.float32))
                - torch.tensor(half_logdet, dtype=torch.float32))
        A32 = A.float()
        f_r32 = _follow(torch.exp(lp32 - lp).double(), A32)       # float32 ratio
        f_r64 = _follow(torch.exp(lp32.double() - lp.double()), A32)  # float64 ratio, float32 lp
        f_64 = _follow(r, A32)                                      # float64 ratio, float64 lp
    flips_ratio = int((f_r32 != f_r64).sum())
    flips_lp = int((f_r64 != f_64).sum())
    rec = dict(kernel="exact_f32" if exact else "bf16x3", lib=os.environ.get("MHPPO_LIB") or "in-tree", rows=M,
               outside_clip=clipped, grad_max_rel_err=err, flips_float32_ratio_vs_float64=flips_ratio,
               flips_float32_lp_vs_float64_lp=flips_lp)
    print("\n" + json.dumps(rec))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(out):
        tag = os.path.basename(os.path.dirname(os.environ["MHPPO_LIB"])) if os.environ.get("MHPPO_LIB") else "tree"
        with open(os.path.join(out, f"clip_scale_{rec['kernel']}_{tag}.json"), "w") as f:
            json.dump(rec, f, indent=1)


def _pair_vs_passes(critic, actor, obs, ret, act, lp, m):
    """One fused pair launch against the actor pass e and the critic pass e + 1 run as two
    launches on the same inputs: gradients, sums and V_{e+1} must be bit-identical."""
    from mhppo import ppo
    _, sc0, V0 = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m)
    stats = sc0[1:3].clone()
    with torch.no_grad():  # the critic's Adam step e (any update of its weights)
        for prm in critic.parameters():
            prm.add_(torch.randn_like(prm) * 1e-3)
    ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CONT, actor, obs, ret, V0, act, lp, stats, m_global=m)
    ga, sa = ga.clone(), sa.clone()
    gc, sc, V1 = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m)
    gc, sc = gc.clone(), sc.clone()
    V = V0.clone()
    sa2 = torch.zeros(3, dtype=torch.float64, device=obs.device)
    sc2 = torch.zeros(3, dtype=torch.float64, device=obs.device)
    ga2, gc2, V = ppo.k_mlp_train_pair(actor, critic, obs, ret, V, act, lp, stats, m, sa2, sc2)
    assert torch.equal(ga2, ga) and torch.equal(gc2, gc)
    assert torch.equal(V, V1)
    assert torch.equal(sa2, sa) and torch.equal(sc2, sc)


def test_pair_launch_bit_identical_to_two_passes():
    """mhppo_mlp_train_pair (actor pass e + critic pass e + 1 in one launch) on the bench's real
    10.5 M-row bucket and on a ragged 70 001-row slice of it."""
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import bucket_segments
    venv = VecCrosswalk("4cars", 65536, 4, 1, 2, seed_base=0)
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)
    with torch.no_grad():
        batch = algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=0)
    c, _, _ = bucket_segments(batch)
    obs, act, lp, ret = c["obs"], c["act"], c["logp"], c["ret"]
    for n in (obs.shape[0], 70001):
        _pair_vs_passes(algo.critic_net_cross, algo.actor_net_cross, obs[:n], ret[:n], act[:n], lp[:n], float(n))


def test_pipelined_epochs_equal_sequential(monkeypatch):
    """Algo_PPO.update's pipelined epochs (ppo.train_epochs: actor e fused with critic e + 1, or
    with PIPELINE_PAIRS off every pass its own launch in the pipelined order) train bit-identical
    nets to the schedule they replace: ten ppo.train_epoch calls (critic passes -> advantage sums
    -> actor passes -> gradient all-reduce -> Adam, epoch by epoch)."""
    from mhppo import ppo
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    pipelined = ppo.train_epochs

    def sequential(heads, n_epochs, bucket=None):
        out = None
        for _ in range(n_epochs):
            out = ppo.train_epoch(heads, bucket)
        return out
    nets = []
    try:
        for arm in ("pairs", "no_pairs", "train_epoch"):
            ppo.PIPELINE_PAIRS = arm == "pairs"
            monkeypatch.setattr(ppo, "train_epochs", sequential if arm == "train_epoch" else pipelined)
            venv = VecCrosswalk("4cars", 2048, 4, 1, 2, seed_base=5)
            torch.manual_seed(0)
            algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=1, save_curves=False)
            algo.train(2)
            nets.append(torch.cat([n.flat() for n in algo.nets()]).cpu())
    finally:
        ppo.PIPELINE_PAIRS = None
    assert torch.equal(nets[0], nets[2]), "pipelined (pairs) vs ten train_epoch calls"
    assert torch.equal(nets[1], nets[2]), "pipelined (no pairs) vs ten train_epoch calls"
