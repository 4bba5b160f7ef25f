"""Data-parallel orchestration on CPU with gloo, world_size 2.

The PPO update's DP logic (mhppo/ppo.py: global row counts, all-reduced
advantage sums, 1/M_global-scaled local gradients, one flat gradient all-reduce,
replicated Adam) must reproduce the single-process full-batch update.  The HIP
loss kernels are replaced by float64-faithful CPU test doubles (tests only; the
product has no CPU path) so the collectives themselves are what is tested.
"""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _install_cpu_doubles(ppo):
    """CPU stand-ins with the kernels' contracts (include/mhppo.h)."""
    import math

    def adv_stats(ret, value):
        a = (ret - value.detach()).double()
        return torch.stack([a.sum(), (a * a).sum()])

    def adv_normalize(ret, value, stats, m):
        mean = stats[0] / m
        var = (stats[1] - stats[0] * mean) / (m - 1)
        a = ret - value.detach()
        return (a - mean.float()) / (var.sqrt().float() + 1e-10)

    def mse(value, ret, m):
        d = (value.detach() - ret).double()
        return (2.0 / m * d).float(), (d * d).sum().reshape(1)

    def ppo_cont(mu, act, lp_old, adv, m):
        diff = (act.double() - mu.detach().double()).float()
        L = math.sqrt(0.5)
        x = diff * (1.0 / L)
        lp = -0.5 * (math.log(2 * math.pi) + x * x) - math.log(L)
        r = torch.exp(lp.double() - lp_old.double())
        A = adv.double()
        s1, s2 = r * A, r.clamp(0.8, 1.2) * A
        inside = ((r >= 0.8) & (r <= 1.2)).double()
        g = torch.where(s1 < s2, A, torch.where(s2 < s1, inside * A, 0.5 * A + 0.5 * inside * A))
        dmu = (1.0 / m) * (-g) * r * x.double() / L
        return dmu.float(), (-torch.minimum(s1, s2)).sum().reshape(1)

    def mlp_train(kind, net, obs, ret, value=None, act=None, lp_old=None, stats=None, counts=None, m_global=1.0):
        m = m_global
        params = list(net.parameters())
        out = torch.squeeze(net(obs), -1)
        if kind == 0:
            dv, loss = mse(out, ret, m)
            st = adv_stats(ret, out)
            sums = torch.cat([loss, st])
            g = torch.autograd.grad(out, params, dv)
            return torch.cat([x.reshape(-1) for x in g]), sums, out.detach()
        adv = adv_normalize(ret, value, stats, m)
        dmu, loss = ppo_cont(out, act, lp_old, adv, m)
        g = torch.autograd.grad(out, params, dmu)
        return torch.cat([x.reshape(-1) for x in g]), torch.cat([loss, torch.zeros(2, dtype=torch.float64)]), None

    ppo.k_adv_stats, ppo.k_adv_normalize, ppo.k_mse, ppo.k_ppo_cont = adv_stats, adv_normalize, mse, ppo_cont
    ppo.k_mlp_train = mlp_train


def _run(rank, world, port, data, out_q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
    from mhppo import ppo
    from mhppo.models import Model_PPO
    _install_cpu_doubles(ppo)
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    actor, critic = Model_PPO(13, 1, 1, mean=-1.0, std=3.0), Model_PPO(13, 1, 0)
    oa, oc = torch.optim.Adam(actor.parameters(), 3e-4), torch.optim.Adam(critic.parameters(), 1e-3)
    obs, act, lp, ret = (torch.tensor(x) for x in data)
    M = obs.shape[0]
    lo, hi = rank * M // world, (rank + 1) * M // world
    m_global = ppo.global_count(hi - lo, "cpu")
    for _ in range(3):
        ppo.train_model_c(actor, critic, oa, oc, obs[lo:hi], act[lo:hi], lp[lo:hi], ret[lo:hi], m_global)
    if rank == 0:
        out_q.put([p.detach().numpy().copy() for p in list(actor.parameters()) + list(critic.parameters())])
    if world > 1:
        dist.destroy_process_group()


def _spawn(world, data):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + world
    procs = [ctx.Process(target=_run, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_dp2_equals_single_process():
    rng = np.random.default_rng(0)
    M = 600
    data = (rng.normal(0, 3, (M, 13)).astype(np.float32), rng.normal(-1, 1, M).astype(np.float32),
            rng.normal(-0.6, 0.3, M).astype(np.float32), rng.normal(-20, 8, M).astype(np.float32))
    single = _spawn(1, data)
    dp2 = _spawn(2, data)
    for a, b in zip(single, dp2):
        np.testing.assert_allclose(a, b, rtol=0, atol=2e-6)
