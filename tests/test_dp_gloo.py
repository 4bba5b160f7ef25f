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

    def choice_loss(probs, lp_old, adv, counts, m):
        """O(M) form of the M x M Categorical surrogate (include/mhppo.h), float64, differentiable."""
        p = probs.double().reshape(-1, 2)
        pn = p / p.sum(1, keepdim=True)
        eps = 1.1920928955078125e-07
        pc = pn.clamp(eps, 1 - eps)
        r = torch.exp(torch.log(pc) - lp_old.double().reshape(-1, 1))
        A = adv.double().reshape(-1, 1)
        f = -torch.minimum(r * A, r.clamp(0.8, 1.2) * A)
        return (f * counts.reshape(1, 2)).sum()

    def mlp_train(kind, net, obs, ret, value=None, act=None, lp_old=None, stats=None, counts=None, m_global=1.0,
                  sums=None, exact=False):
        g, s, v = _mlp_train(kind, net, obs, ret, value, act, lp_old, stats, counts, m_global)
        if sums is None:
            return g, s, v
        sums += s  # the kernel accumulates into the caller's zeroed sums (include/mhppo.h)
        return g, sums, v

    def _mlp_train(kind, net, obs, ret, value, act, lp_old, stats, counts, m_global):
        m = m_global
        params = list(net.parameters())
        out = torch.squeeze(net(obs), -1)
        gf = net.grad_flat()  # the kernel writes the gradient into the net's flat storage
        if kind == 0:
            dv, loss = mse(out, ret, m)
            st = adv_stats(ret, out)
            sums = torch.cat([loss, st])
            g = torch.autograd.grad(out, params, dv, allow_unused=True)
            gf.copy_(torch.cat([(x if x is not None else torch.zeros_like(q)).reshape(-1) for x, q in zip(g, params)]))
            return gf, sums, out.detach()
        adv = adv_normalize(ret, value, stats, m)
        if kind == 2:
            loss = choice_loss(out, lp_old, adv, counts, m)
            g = torch.autograd.grad(loss / (m * m), params, allow_unused=True)
            loss = loss.detach().reshape(1)
        else:
            dmu, loss = ppo_cont(out, act, lp_old, adv, m)
            g = torch.autograd.grad(out, params, dmu, allow_unused=True)
        gf.copy_(torch.cat([(x if x is not None else torch.zeros_like(q)).reshape(-1) for x, q in zip(g, params)]))
        return gf, torch.cat([loss, torch.zeros(2, dtype=torch.float64)]), None

    def mlp_train_pair(actor, critic, obs, ret, value, act, lp_old, stats, m_global, sums_a, sums_c):
        """mhppo_mlp_train_pair's contract: actor pass e on V_e, then critic pass e + 1 into value."""
        mlp_train(1, actor, obs, ret, value, act, lp_old, stats, m_global=m_global, sums=sums_a)
        _, _, v = mlp_train(0, critic, obs, ret, m_global=m_global, sums=sums_c)
        value.copy_(v)
        return actor.grad_flat(), critic.grad_flat(), value

    ppo.k_adv_stats, ppo.k_adv_normalize, ppo.k_mse, ppo.k_ppo_cont = adv_stats, adv_normalize, mse, ppo_cont
    ppo.k_mlp_train = mlp_train
    ppo.k_mlp_train_pair = mlp_train_pair

    # train_epochs' launch helpers (ppo._HeadPlan arguments) on the same doubles
    def critic_pass(p, h, sums, st):
        p.V.copy_(mlp_train(0, h.critic, p.obs, p.ret, m_global=h.m, sums=sums)[2])

    def actor_pass(p, h, stats, sums, st):
        mlp_train(p.akind, h.actor, p.obs, p.ret, p.V, p.act, p.lp, stats, p.counts, m_global=h.m, sums=sums)

    def pair_pass(p, h, stats, sums_a, sums_c, st):
        mlp_train_pair(h.actor, h.critic, p.obs, p.ret, p.V, p.act, p.lp, stats, h.m, sums_a, sums_c)

    ppo._critic_pass, ppo._actor_pass, ppo._pair_pass = critic_pass, actor_pass, pair_pass


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


def _run_joint(rank, world, port, data, shards, out_q, skip=()):
    """Three heads (cross, wait, choice) trained by ppo.train_epoch with a GradBucket: two
    collectives per joint epoch.  `shards[rank]` gives this rank's [lo, hi) rows per head
    (an empty range = an empty shard that must still join every collective).  Heads in `skip`
    are not trained at all (Algo_PPO.update drops a head whose GLOBAL batch is empty): their
    gradient slices hold a sentinel that no collective may touch."""
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
    from mhppo import ppo
    from mhppo.models import Model_PPO
    _install_cpu_doubles(ppo)
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(0)
    nets = [Model_PPO(13, 1, 1, mean=-1.0, std=3.0), Model_PPO(13, 1, 0), Model_PPO(13, 1, 1, mean=-1.0, std=3.0),
            Model_PPO(13, 1, 0), Model_PPO(20, 2, 2), Model_PPO(20, 1, 0)]
    bucket = ppo.GradBucket(nets, "cpu")
    opts = [torch.optim.Adam(n.parameters(), 3e-4 if i % 2 == 0 else 1e-3) for i, n in enumerate(nets)]
    heads = []
    for h, kind in enumerate(("c", "c", "d")):
        if h in skip:
            for n in nets[2 * h:2 * h + 2]:
                n.grad_flat().fill_(1.0)
            continue
        obs, act, lp, ret = (torch.tensor(x) for x in data[h])
        lo, hi = shards[rank][h]
        m = ppo.global_count(hi - lo, "cpu")
        counts = None
        if kind == "d":
            counts = ppo._allreduce_(torch.stack([(act[lo:hi] == 0).sum(), (act[lo:hi] == 1).sum()]).double())
        heads.append(ppo.Head(kind, nets[2 * h], nets[2 * h + 1], opts[2 * h], opts[2 * h + 1], obs[lo:hi],
                              act[lo:hi], lp[lo:hi], ret[lo:hi], m, counts))
    for _ in range(3):
        ppo.train_epoch(heads, bucket)
    if rank == 0:
        out_q.put([p.detach().numpy().copy() for n in nets for p in n.parameters()] +
                  [nets[2 * h + k].grad_flat().numpy().copy() for h in skip for k in (0, 1)])
    if world > 1:
        dist.destroy_process_group()


def _spawn_joint(world, data, shards, skip=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30600 + os.getpid() % 1000 + world + 7 * len(skip)
    procs = [ctx.Process(target=_run_joint, args=(r, world, port, data, shards, q, skip)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_dp2_joint_epoch_with_empty_shard():
    """The joint three-head epoch (one advantage-sum and one gradient-bucket all-reduce per
    epoch) over 2 ranks equals one process; rank 1 holds NO wait rows and still joins."""
    rng = np.random.default_rng(3)
    data = []
    for M, nin, choice in ((500, 13, False), (120, 13, False), (90, 20, True)):
        act = ((rng.uniform(size=M) < 0.4).astype(np.float32) if choice else rng.normal(-1, 1, M).astype(np.float32))
        data.append((rng.normal(0, 3, (M, nin)).astype(np.float32), act, rng.normal(-0.6, 0.3, M).astype(np.float32),
                     rng.normal(-20, 8, M).astype(np.float32)))
    single = _spawn_joint(1, data, [[(0, 500), (0, 120), (0, 90)]])
    dp2 = _spawn_joint(2, data, [[(0, 230), (0, 120), (0, 40)], [(230, 500), (120, 120), (40, 90)]])
    for a, b in zip(single, dp2):
        np.testing.assert_allclose(a, b, rtol=0, atol=2e-6)


def test_dp2_joint_epoch_skipped_middle_head():
    """The wait head (the middle nets of the gradient bucket) is empty on every rank, so
    Algo_PPO.update does not train it: the bucket all-reduce covers the cross and the choice
    gradients in two runs and never sums the wait head's stale slice (it keeps its sentinel,
    not world_size x it); the trained nets equal one process."""
    from mhppo.ppo import GradBucket
    from mhppo.models import Model_PPO
    nets = [Model_PPO(13, 1, 1), Model_PPO(13, 1, 0), Model_PPO(13, 1, 1), Model_PPO(13, 1, 0), Model_PPO(20, 2, 2),
            Model_PPO(20, 1, 0)]
    b = GradBucket(nets, "cpu")
    r = b.runs([nets[0], nets[1], nets[4], nets[5]])
    assert len(r) == 2 and r[0][0] == 0 and r[1][1] == b.buf.numel() and r[0][1] < r[1][0]
    assert b.runs(nets) == [(0, b.buf.numel())]
    rng = np.random.default_rng(4)
    data = []
    for M, nin, choice in ((300, 13, False), (1, 13, False), (80, 20, True)):
        act = ((rng.uniform(size=M) < 0.4).astype(np.float32) if choice else rng.normal(-1, 1, M).astype(np.float32))
        data.append((rng.normal(0, 3, (M, nin)).astype(np.float32), act, rng.normal(-0.6, 0.3, M).astype(np.float32),
                     rng.normal(-20, 8, M).astype(np.float32)))
    single = _spawn_joint(1, data, [[(0, 300), (0, 0), (0, 80)]], skip=(1,))
    dp2 = _spawn_joint(2, data, [[(0, 140), (0, 0), (0, 30)], [(140, 300), (0, 0), (30, 80)]], skip=(1,))
    for a, b_ in zip(single, dp2):
        np.testing.assert_allclose(a, b_, rtol=0, atol=2e-6)
    for g in dp2[-2:]:  # the skipped head's gradient slices: untouched by any collective
        assert np.all(g == 1.0)


# ------------------------------------------------------------------ whole Algo_PPO.train, world 4
class _Cfg:
    car_b = [-4.0, 0.0, 2.0, 0.0]


class _VenvDouble:
    """The attributes Algo_PPO reads from a VecCrosswalk (CPU; no env handle)."""

    def __init__(self, n_envs, env_id_offset, n_slots=2, variant="coop"):
        self.n_envs, self.env_id_offset = n_envs, env_id_offset
        self.max_episode, self.n_slots, self.dt, self.variant = 8, n_slots, 0.5, variant
        self.cfg, self.device = _Cfg(), torch.device("cpu")


def _rollout_double_class(n_total):
    """Env_rollout stand-in: one 'episode' per env, each (env, slot) segment bucketed by its GLOBAL
    env id, so rank r of W owns exactly the global segments [r n, (r + 1) n) of one process.
    Quarter 1 of the envs is all cross, quarter 2 all wait: with 4 ranks, rank 1 has no wait
    rows and rank 2 no cross rows (each still joins every collective)."""

    class RolloutDouble:
        def __init__(self, env, nb_cars, max_steps, dt):
            self.env, self.T = env, max_steps
            self.seed, self.iteration, self.fix_bucket = 0, 0, False
            self.cross = self.wait = self.choice = None

        def reset(self):
            pass

        def iterations_rand(self, *a, **k):
            T, S = self.T, self.env.n_slots
            seg = {"cross": [], "wait": []}
            ch = []
            for g in range(self.env.env_id_offset, self.env.env_id_offset + self.env.n_envs):
                q = 4 * g // n_total
                for s in range(S):
                    rng = np.random.default_rng(1000 * self.iteration + 10 * g + s)
                    b = "cross" if q == 1 else ("wait" if q == 2 else ("cross" if rng.uniform() < 0.5 else "wait"))
                    seg[b].append((rng.normal(0, 3, (T, 13)).astype(np.float32), rng.normal(-1, 1, T).astype(np.float32),
                                   rng.normal(-0.6, 0.3, T).astype(np.float32), rng.normal(-20, 8, T).astype(np.float32),
                                   rng.normal(-1, 0.5, T)))
                    ch.append((rng.normal(0, 2, 20).astype(np.float32), int(rng.uniform() < 0.4),
                               np.float32(rng.normal(-0.7, 0.2)), np.float32(rng.normal(-3, 1))))
            self.iteration += 1
            for b in ("cross", "wait"):
                L = seg[b]
                cat = (lambda i, shape, dt: torch.from_numpy(np.concatenate([x[i] for x in L])) if L
                       else torch.zeros(shape, dtype=dt))
                d = dict(obs=cat(0, (0, 13), torch.float32), act=cat(1, (0,), torch.float32),
                         logp=cat(2, (0,), torch.float32), ret=cat(3, (0,), torch.float32),
                         rew=cat(4, (0,), torch.float64), n_seg=len(L))
                setattr(self, b, d)
            self.choice = dict(obs=torch.from_numpy(np.stack([c[0] for c in ch])),
                               act=torch.tensor([c[1] for c in ch], dtype=torch.int32),
                               logp=torch.tensor([c[2] for c in ch]), ret=torch.tensor([c[3] for c in ch]),
                               n_seg=len(ch))

        def immediate_rewards(self):
            return self.cross["rew"].float(), self.wait["rew"].float(), self.choice["ret"]

    return RolloutDouble


def _run_algo(rank, world, port, n_total, out_q, n_slots=2, variant="coop"):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
    from mhppo import algo as algo_mod
    from mhppo import ppo
    from mhppo.models import Model_PPO
    _install_cpu_doubles(ppo)
    algo_mod.Env_rollout = _rollout_double_class(n_total)
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    n = n_total // world
    torch.manual_seed(0)
    a = algo_mod.Algo_PPO(Model_PPO, _VenvDouble(n, rank * n, n_slots, variant), verbose=False, save_curves=False,
                          num_states_d=20)
    a.train(2)
    if rank == 0:
        out_q.put([p.detach().numpy().copy() for net in a.nets() for p in net.parameters()] +
                  [np.array(x, dtype=np.float64) for x in a.curves()])
    if world > 1:
        dist.destroy_process_group()


def _spawn_algo(world, n_total, n_slots=2, variant="coop"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31700 + os.getpid() % 1000 + world
    procs = [ctx.Process(target=_run_algo, args=(r, world, port, n_total, q, n_slots, variant)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_dp4_algo_train_uneven_shards():
    """Two whole Algo_PPO.train iterations (update: global row and action counts, the joint
    epochs' advantage-sum and gradient-bucket all-reduces, replicated Adam; the reward-curve sum
    all-reduce) over 4 gloo ranks equal one process on all envs.  Rank 1 holds no wait rows and
    rank 2 no cross rows."""
    n_total = 64
    single = _spawn_algo(1, n_total)
    dp4 = _spawn_algo(4, n_total)
    assert len(single) == len(dp4)
    for a, b in zip(single, dp4):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=2e-6)
    assert len(single[-4]) == 2  # two reward-curve entries per head


def test_dp8_algo_train_cfg5_partition():
    """Config 5's partition (BASELINE configs[4]: the scalable env's envs split contiguously over 8
    ranks, rank r owning global env ids [r n, (r + 1) n)) at small N: two whole Algo_PPO.train
    iterations over 8 gloo ranks with 8 car slots per env equal one process on all envs (ranks 2-3
    hold no wait rows, ranks 4-5 no cross rows).  The HIP path's global-id seeding for that partition
    is pinned on one GPU at full size (tests/test_env_fullscale_gpu.py / test_rollout_fullscale_gpu.py,
    cfg5_shard7)."""
    n_total = 64
    single = _spawn_algo(1, n_total, n_slots=8, variant="scalable")
    dp8 = _spawn_algo(8, n_total, n_slots=8, variant="scalable")
    assert len(single) == len(dp8)
    for a, b in zip(single, dp8):
        np.testing.assert_allclose(b, a, rtol=1e-6, atol=2e-6)
