"""PPO update of the multi-head actor-critic (Algo_PPO.train_model_c / _d,
Coop-MH-PPO-scalable.py:778-851), full batch, on the GPU.

Every head's epoch runs on the fused training kernel (mhppo_mlp_train, csrc/mlp_train.hip;
the 13-input heads on its bf16x3 split-precision MFMA path — six bf16 products per f32
product, f32-level accuracy — or, with Algo_PPO(exact_f32=True) (MHPPO_TRAIN_EXACT_F32), on f32
MFMA with k-ordered sums; the choice head on f32 MFMA): a critic pass (forward, MSE gradient, advantage sums) and an
actor pass (forward, clip-surrogate gradient against the advantage normalised with
the start-of-epoch critic, backward, weight gradients); Adam (fused) steps each net.
Epoch semantics follow the reference: the advantage uses the critic of the start of
the epoch (:784-787), the actor-loss gradient never reaches the critic (the reference
zeroes it before the critic step, :810-815).  The small HIP kernels below (advantage
statistics, the clip surrogates, MSE) restate the same losses for the tests'
autograd cross-checks.

Heads are independent nets, so one epoch of every head of an iteration runs together
(train_epoch): the reference's 10 cross/wait epochs and its 10 choice epochs
(:868-882) become 10 joint epochs with identical results.

Data parallel: every rank holds a shard of every head's batch.  Per
joint epoch there are exactly two collectives: one all-reduce (SUM, float64) of all
heads' advantage sums between the critic and the actor passes, and one all-reduce
(SUM) of the gradient bucket — every net's flat gradient lives in one contiguous
GradBucket, so the collective runs in place with no pack/unpack copies.  Each rank's
gradient is that of (global-mean loss restricted to its rows), so the reduced
gradient is the full-batch gradient; Adam then runs replicated.  A rank whose shard
of a head is empty still joins both collectives (the kernel writes a zero gradient).
"""
import contextlib
import os

import torch
import torch.distributed as dist

from . import _lib


_FORCE_COLLECTIVES = False


def set_force_collectives(flag=True):
    """Run the data-parallel collectives even in a one-rank process group (they are skipped
    when world_size == 1): a one-GPU RCCL rehearsal of the exact multi-GPU call sequence
    (bench.py --force-collectives, tests/dp_worker.py --nccl-world1).  Needs an initialised
    process group; a one-rank SUM is the identity, so results equal the plain run's."""
    global _FORCE_COLLECTIVES
    _FORCE_COLLECTIVES = bool(flag)


def _dp():
    if not (dist.is_available() and dist.is_initialized()):
        return False
    return _FORCE_COLLECTIVES or dist.get_world_size() > 1


def _allreduce_(t):
    if _dp():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def global_counts(values, device):
    """All-reduce (SUM) a few per-rank counts at once; one host sync: returns floats."""
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    return [float(x) for x in _allreduce_(t).tolist()]


def global_count(n, device):
    return global_counts([n], device)[0]


class GradBucket:
    """One contiguous float32 buffer holding the flat gradients of several Model_PPOs
    (each net's .grad views alias its slice): the gradient all-reduce of an epoch is
    one in-place collective over a contiguous span of it."""

    def __init__(self, nets, device):
        sizes = [n.flat().numel() for n in nets]
        self.buf = torch.zeros(sum(sizes), dtype=torch.float32, device=device)
        self.span = {}
        off = 0
        for net, n in zip(nets, sizes):
            net.bind_grad(self.buf[off:off + n])
            self.span[id(net)] = (off, off + n)
            off += n

    def runs(self, nets):
        """The maximal contiguous spans of the bucket covered by `nets`' gradients, in order (a
        net that is not trained this epoch — an empty head — splits the span: its stale slice is
        never reduced)."""
        spans = sorted(self.span[id(n)] for n in nets)
        out = []
        for lo, hi in spans:
            if out and out[-1][1] == lo:
                out[-1][1] = hi
            else:
                out.append([lo, hi])
        return [tuple(r) for r in out]

    def allreduce(self, nets):
        """In-place SUM of `nets`' gradients: one collective per maximal contiguous run (one for
        the usual all-heads epoch)."""
        if not _dp() or not nets:
            return
        for n in nets:  # re-link any .grad that autograd / zero_grad rebound
            n.grad_flat()
        for lo, hi in self.runs(nets):
            dist.all_reduce(self.buf[lo:hi], op=dist.ReduceOp.SUM)


def _allreduce_net_grads(*nets):
    """Gradient all-reduce for nets outside a GradBucket (one packed collective)."""
    if not _dp():
        return
    flats = [n.grad_flat() for n in nets]
    flat = torch.cat(flats)
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    off = 0
    for f in flats:
        f.copy_(flat[off:off + f.numel()])
        off += f.numel()


# ---------------------------------------------------------------- kernel layer
# Thin wrappers over the HIP entry points (include/mhppo.h).  Each returns this
# rank's LOCAL contribution; the DP orchestration below decides what is reduced.

def k_adv_stats(ret, value):
    """(sum A, sum A^2) over local rows, float64 [2]."""
    stats = torch.zeros(2, dtype=torch.float64, device=ret.device)
    v = value.detach().contiguous()
    with torch.cuda.device(ret.device):
        _lib.check(_lib.lib().mhppo_adv_stats(_lib.ptr(ret), _lib.ptr(v), ret.numel(), _lib.ptr(stats),
                                              _lib.stream_ptr()))
    return stats


def k_adv_normalize(ret, value, stats, m_global):
    adv = torch.empty_like(ret)
    v = value.detach().contiguous()
    with torch.cuda.device(ret.device):
        _lib.check(_lib.lib().mhppo_adv_normalize(_lib.ptr(ret), _lib.ptr(v), ret.numel(), _lib.ptr(stats),
                                                  float(m_global), _lib.ptr(adv), _lib.stream_ptr()))
    return adv


def k_mse(value, ret, m_global):
    dv = torch.empty_like(ret)
    loss = torch.zeros(1, dtype=torch.float64, device=ret.device)
    v = value.detach().contiguous()
    with torch.cuda.device(ret.device):
        _lib.check(_lib.lib().mhppo_mse_fwd_bwd(_lib.ptr(v), _lib.ptr(ret), ret.numel(), 1.0 / m_global,
                                                _lib.ptr(dv), _lib.ptr(loss), _lib.stream_ptr()))
    return dv, loss


def k_ppo_cont(mu, act, logp_old, adv, m_global):
    dmu = torch.empty_like(adv)
    loss = torch.zeros(1, dtype=torch.float64, device=adv.device)
    m = mu.detach().contiguous()
    with torch.cuda.device(adv.device):
        _lib.check(_lib.lib().mhppo_ppo_cont_fwd_bwd(_lib.ptr(m), _lib.ptr(act), _lib.ptr(logp_old), _lib.ptr(adv),
                                                     adv.numel(), 1.0 / m_global, _lib.ptr(dmu), _lib.ptr(loss),
                                                     _lib.stream_ptr()))
    return dmu, loss


def k_ppo_choice(probs, logp_old, adv, counts, m_global):
    p = probs.detach().contiguous()
    dp = torch.empty_like(p)
    loss = torch.zeros(1, dtype=torch.float64, device=adv.device)
    with torch.cuda.device(adv.device):
        _lib.check(_lib.lib().mhppo_ppo_choice_fwd_bwd(_lib.ptr(p), _lib.ptr(logp_old), _lib.ptr(adv), adv.numel(),
                                                       _lib.ptr(counts), 1.0 / (m_global * m_global), _lib.ptr(dp),
                                                       _lib.ptr(loss), _lib.stream_ptr()))
    return dp, loss


# Optional launch timing (bench.py): when a list, each fused train launch appends
# (kind, n_in, rows, start_event, end_event) recorded on the launch stream.
TRAIN_EVENTS = None


def flops_per_row(n_in, n_out):
    """Algorithmic FLOPs of one row through the fused kernel: forward and
    weight gradient 2 * (32 n_in + 2048 + 2048 + 32 n_out) each, backward data without
    dX 2 * (32 n_out + 2048 + 2048).  13 -> 1: 26,432."""
    macs = 32 * n_in + 2048 + 2048 + 32 * n_out
    return 2 * macs + 2 * (32 * n_out + 4096) + 2 * macs


FLOPS_PER_ROW_CONT = flops_per_row(13, 1)
N_IN_MAX = 64  # the fused kernel's widest input (scalable 8-slot choice head: dc = 54)

KIND_CRITIC, KIND_CONT, KIND_CHOICE = 0, 1, 2
# MHPPO_TRAIN_EXACT_F32 (include/mhppo.h mhppo_mlp_train): a head's passes on the f32-MFMA
# kernel (k-ordered fmaf sums, the exact f32 arithmetic of an fmaf chain) instead of the default
# bf16x3 split-precision one; per head: Head(exact=True), set by Algo_PPO(exact_f32=True)
TRAIN_EXACT_F32 = 0x100


def n_params(n_in, n_out):
    return 32 * n_in + 32 + 64 * 32 + 64 + 32 * 64 + 32 + 32 * n_out + n_out


def k_mlp_train(kind, net, obs, ret, value=None, act=None, logp_old=None, stats=None, counts=None, m_global=1.0,
                exact=False, sums=None):
    """Fused forward/loss/backward of one head (mhppo_mlp_train).
    kind 0 (critic): returns (grad, sums[3] = (sum (V-G)^2, sum A, sum A^2), V).
    kind 1 (continuous actor) / 2 (choice actor): returns (grad, sums[3] = (sum surrogate, 0, 0), None).
    grad is the packed torch-layout gradient (W1 b1 .. W4 b4), written into the net's flat
    .grad storage.  An empty `obs` (an empty data-parallel shard) gives a zero gradient.
    `sums`: optional zeroed float64 [3] the kernel accumulates into (train_epoch passes rows of
    one zeroed tensor: one fill per epoch instead of one per pass).
    exact: the f32-MFMA kernel instead of the split-precision one (any head with n_in <= 54;
    wider choice heads always run on f32 MFMA)."""
    want = {KIND_CRITIC: 0, KIND_CONT: 1, KIND_CHOICE: 2}[kind]
    if net.model_type != want or net.n_in > N_IN_MAX or (kind == KIND_CONT and net.n_in != 13):
        raise ValueError(f"fused kernel kind {kind} cannot train a model_type {net.model_type} "
                         f"{net.n_in}->{net.n_out} Model_PPO")
    dev = obs.device
    M = obs.shape[0]
    obs = obs.float().contiguous()
    if obs.data_ptr() % 16:
        obs = obs.clone()
    ret = ret.float().contiguous()
    V = torch.empty(M, dtype=torch.float32, device=dev) if kind == KIND_CRITIC else value.detach().float().contiguous()
    act = None if act is None else act.float().contiguous()
    logp_old = None if logp_old is None else logp_old.float().contiguous()
    np_ = n_params(net.n_in, net.n_out)
    grad = net.grad_flat()
    if grad.numel() != np_ or grad.device != dev:
        raise ValueError("gradient storage does not match the net / the batch's device")
    if sums is None:
        sums = torch.zeros(3, dtype=torch.float64, device=dev)
    w = net.flat()
    p = _lib.ptr
    ev = None
    if TRAIN_EVENTS is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    flags = TRAIN_EXACT_F32 if exact else 0
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().mhppo_mlp_train(
            kind | flags, net.n_in, p(w), p(obs), M, p(ret), p(V), p(act), p(logp_old), p(stats), p(counts),
            float(m_global), float(net.mean), float(net.std), p(grad), p(sums), _lib.stream_ptr()))
    if ev is not None:
        ev[1].record()
        TRAIN_EVENTS.append((kind, net.n_in, M, ev[0], ev[1]))
    return grad, sums, (V if kind == KIND_CRITIC else None)


def k_mlp_train_pair(actor, critic, obs, ret, value, act, logp_old, stats, m_global, sums_actor, sums_critic):
    """Actor pass of epoch e + critic pass of epoch e + 1 of one continuous head in one launch
    (mhppo_mlp_train_pair): `value` holds V_e (the critic pass e's outputs) and is overwritten
    with V_{e+1}; `stats` are the critic pass e's global advantage sums; the critic's weights
    must already carry its Adam step e.  Gradients go to both nets' flat .grad storage; the
    float64 sums accumulate into sums_actor / sums_critic (zeroed [3] each)."""
    for net, kind in ((actor, 1), (critic, 0)):
        if net.model_type != kind or net.n_in != 13 or net.n_out != 1:
            raise ValueError("the fused pair launch trains a 13 -> 1 continuous actor and its 13 -> 1 critic")
    dev = obs.device
    M = obs.shape[0]
    obs = obs.float().contiguous()
    if obs.data_ptr() % 16:
        obs = obs.clone()
    ret, act, logp_old = ret.float().contiguous(), act.float().contiguous(), logp_old.float().contiguous()
    if value.dtype != torch.float32 or not value.is_contiguous() or value.numel() != M:
        raise ValueError("value must be the float32 [M] buffer of the previous critic pass (updated in place)")
    ga, gc = actor.grad_flat(), critic.grad_flat()
    p = _lib.ptr
    ev = None
    if TRAIN_EVENTS is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().mhppo_mlp_train_pair(
            p(actor.flat()), p(critic.flat()), p(obs), M, p(ret), p(value), p(act), p(logp_old), p(stats),
            float(m_global), float(actor.mean), float(actor.std), p(ga), p(sums_actor), p(gc), p(sums_critic),
            _lib.stream_ptr()))
    if ev is not None:
        ev[1].record()
        TRAIN_EVENTS.append((3, 13, M, ev[0], ev[1]))  # kind 3: a fused pair launch (two passes)
    return ga, gc, value


# ------------------------------------------------------------- DP orchestration

class Head:
    """One actor/critic pair, its Adam optimisers and this rank's shard of its batch.
    kind "c": continuous head (train_model_c, :778-815); "d": choice head (train_model_d,
    :818-851) with the GLOBAL action counts (n0, n1) of the M x M broadcast, or the
    opt-in per-row loss.  m = the global row count.  exact: the head's passes on
    the exact f32-MFMA kernel (Algo_PPO(exact_f32=True))."""

    def __init__(self, kind, actor, critic, opt_actor, opt_critic, obs, act, logp, ret, m, counts=None,
                 per_row=False, exact=False):
        self.kind, self.actor, self.critic = kind, actor, critic
        self.opt_actor, self.opt_critic = opt_actor, opt_critic
        self.obs, self.act, self.logp, self.ret, self.m = obs, act, logp, ret, float(m)
        self.counts = None if counts is None else counts.double().contiguous()
        self.per_row = per_row
        self.exact = bool(exact)


def train_epoch(heads, bucket=None):
    """One full-batch epoch of every head: critic passes -> ONE all-reduce of all heads'
    advantage sums -> actor passes -> ONE gradient all-reduce -> Adam.  Returns this rank's
    (actor, critic) loss sums per head (float64 [1] tensors)."""
    H = len(heads)
    sums = torch.zeros(2 * H, 3, dtype=torch.float64, device=heads[0].obs.device)  # critic rows, actor rows
    crit = [k_mlp_train(KIND_CRITIC, h.critic, h.obs, h.ret, m_global=h.m, sums=sums[i], exact=h.exact)
            for i, h in enumerate(heads)]
    stats = sums[:H, 1:3].reshape(-1).contiguous()
    _allreduce_(stats)
    out = []
    for i, (h, (_, sc, V)) in enumerate(zip(heads, crit)):
        st = stats[2 * i:2 * i + 2]
        sa = sums[H + i]
        if h.kind == "c":
            k_mlp_train(KIND_CONT, h.actor, h.obs, h.ret, V, h.act, h.logp, st, m_global=h.m, sums=sa, exact=h.exact)
        elif h.per_row:
            k_mlp_train(KIND_CHOICE, h.actor, h.obs, h.ret, V, h.act.float(), h.logp, st, None, m_global=h.m,
                        sums=sa, exact=h.exact)
        else:
            k_mlp_train(KIND_CHOICE, h.actor, h.obs, h.ret, V, None, h.logp, st, h.counts, m_global=h.m, sums=sa,
                        exact=h.exact)
        out.append((sa[0:1], sc[0:1]))
    nets = [n for h in heads for n in (h.actor, h.critic)]
    if bucket is not None:
        bucket.allreduce(nets)
    else:
        _allreduce_net_grads(*nets)
    adam_steps([o for h in heads for o in (h.opt_actor, h.opt_critic)])
    return out


# Fuse each continuous head's actor pass e with its critic pass e + 1 (train_epochs) when the head
# has at most PAIR_MAX_ROWS rows (global).  The fused launch shares one input load and saves a
# launch, a weight-staging prologue and a reduction pair per epoch, but with two nets in one wave
# neither can hold its weight fragments in registers: per tile it is 3.6 % slower than the two
# passes (profiles/r04_pair/).  Measured end to end: config 2 (328 k rows per head) 7.92 -> 7.53
# ms per iteration, config 3 (10.5 M rows) 81.9 -> 85.9 ms.  MHPPO_PIPELINE_PAIRS=0 / =1 forces
# it off / on (A/B).
PIPELINE_PAIRS = {"0": False, "1": True}.get(os.environ.get("MHPPO_PIPELINE_PAIRS", ""), None)
PAIR_MAX_ROWS = 2_000_000


def _use_pair(h):
    if h.kind != "c" or h.exact:
        return False
    return PIPELINE_PAIRS if PIPELINE_PAIRS is not None else h.m <= PAIR_MAX_ROWS


class _HeadPlan:
    """One head's launch arguments for a whole train_epochs call, resolved once: the batch as
    contiguous float32 (16-byte aligned rows), the nets' flat weight / gradient pointers (fixed
    while the epochs run: the fused Adam updates them in place) and one V buffer.  Per pass only
    the stats / sums pointers change — the Python cost of a pass is one ctypes call (the per-call
    re-validation in k_mlp_train, ~60 us of host time, left the GPU idle on small batches)."""

    def __init__(self, h):
        for net, kind in ((h.critic, KIND_CRITIC), (h.actor, KIND_CONT if h.kind == "c" else KIND_CHOICE)):
            want = {KIND_CRITIC: 0, KIND_CONT: 1, KIND_CHOICE: 2}[kind]
            if net.model_type != want or net.n_in > N_IN_MAX or (kind == KIND_CONT and net.n_in != 13):
                raise ValueError(f"fused kernel kind {kind} cannot train a model_type {net.model_type} "
                                 f"{net.n_in}->{net.n_out} Model_PPO")
        obs = h.obs.float().contiguous()
        if obs.data_ptr() % 16:
            obs = obs.clone()
        self.obs, self.ret = obs, h.ret.float().contiguous()
        self.M = obs.shape[0]
        self.lp = h.logp.float().contiguous()
        self.act = h.act.float().contiguous() if (h.kind == "c" or h.per_row) else None
        self.counts = None if (h.kind == "c" or h.per_row) else h.counts
        self.V = torch.empty(self.M, dtype=torch.float32, device=obs.device)
        self.n_in = h.actor.n_in
        self.wa, self.wc = h.actor.flat().data_ptr(), h.critic.flat().data_ptr()
        self.ga, self.gc = h.actor.grad_flat().data_ptr(), h.critic.grad_flat().data_ptr()
        self.mean, self.std = float(h.actor.mean), float(h.actor.std)
        self.flags = TRAIN_EXACT_F32 if h.exact else 0
        self.akind = KIND_CONT if h.kind == "c" else KIND_CHOICE
        self.keep = (h.actor.flat(), h.critic.flat())  # the storages the pointers above point into


def _ev_begin():
    if TRAIN_EVENTS is None:
        return None
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    return ev


def _ev_end(ev, kind, n_in, M):
    if ev is not None:
        ev[1].record()
        TRAIN_EVENTS.append((kind, n_in, M, ev[0], ev[1]))


# The three launch helpers of train_epochs (module-level so CPU test doubles can stand in for them:
# tests/test_dp_gloo.py).  sums / stats are float64 views: [3] rows of the step's sums, [2] stats.
def _critic_pass(p, h, sums, st):
    ev = _ev_begin()
    _lib.check(_lib.lib().mhppo_mlp_train(
        KIND_CRITIC | p.flags, p.n_in, p.wc, p.obs.data_ptr(), p.M, p.ret.data_ptr(), p.V.data_ptr(), None, None, None,
        None, h.m, 0.0, 1.0, p.gc, sums.data_ptr(), st))
    _ev_end(ev, KIND_CRITIC, p.n_in, p.M)


def _actor_pass(p, h, stats, sums, st):
    ev = _ev_begin()
    _lib.check(_lib.lib().mhppo_mlp_train(
        p.akind | p.flags, p.n_in, p.wa, p.obs.data_ptr(), p.M, p.ret.data_ptr(), p.V.data_ptr(),
        None if p.act is None else p.act.data_ptr(), p.lp.data_ptr(), stats.data_ptr(),
        None if p.counts is None else p.counts.data_ptr(), h.m, p.mean, p.std, p.ga, sums.data_ptr(), st))
    _ev_end(ev, p.akind, p.n_in, p.M)


def _pair_pass(p, h, stats, sums_a, sums_c, st):
    ev = _ev_begin()
    _lib.check(_lib.lib().mhppo_mlp_train_pair(
        p.wa, p.wc, p.obs.data_ptr(), p.M, p.ret.data_ptr(), p.V.data_ptr(), p.act.data_ptr(), p.lp.data_ptr(),
        stats.data_ptr(), h.m, p.mean, p.std, p.ga, sums_a.data_ptr(), p.gc, sums_c.data_ptr(), st))
    _ev_end(ev, 3, 13, p.M)  # kind 3: a fused pair launch (two passes)


# Heads' passes on alternating streams within an epoch step (train_epochs): head i's passes on
# stream i % TRAIN_STREAMS (a head's actor and critic passes stay in order on one stream: the critic
# pass e + 1 overwrites the V_e the actor pass e reads).  The heads are independent within a step, so
# one head's launch and weight staging overlap the other's tail, partial fold and reduction
# (mhppo_mlp_train keeps a workspace per stream).  Measured -0.7 % per iteration with two streams
# (profiles/r04_streams/), but then each kernel's execution span (rocprofv3) includes the time its
# blocks wait behind the other stream's kernel, so the per-kernel profile no longer matches the
# kernel's own duration: the default stays one stream; MHPPO_TRAIN_STREAMS=2 opts in.
TRAIN_STREAMS = max(1, int(os.environ.get("MHPPO_TRAIN_STREAMS", "1")))
_SIDE_STREAMS = {}


def _side_streams(dev, n):
    if dev.type != "cuda" or n <= 0:
        return []
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), n)
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = [torch.cuda.Stream(device=dev) for _ in range(n)]
    return _SIDE_STREAMS[key]


def train_epochs(heads, n_epochs, bucket=None):
    """n_epochs full-batch epochs of every head, run as a pipeline of n_epochs + 1 steps: step k
    runs the actor passes of epoch k - 1 and the critic passes of epoch k (a continuous head on the
    split-precision kernel: ONE fused launch, mhppo_mlp_train_pair), then one gradient all-reduce
    of the nets trained in the step, one all-reduce of the new critic passes' advantage sums and
    the Adam steps.  The same arithmetic as n_epochs calls of train_epoch: the actor of epoch e
    uses V_e and the advantage sums of the critic pass e (critic weights of epoch e), the critic
    of epoch e + 1 the critic's weights after its Adam step e; each optimiser steps n_epochs
    times.  Returns this rank's (actor, critic) loss sums of the last epoch per head.
    The launches go straight through the C-ABI with each head's arguments resolved once
    (_HeadPlan); an empty head (M == 0) runs k_mlp_train's empty-shard path."""
    H = len(heads)
    dev = heads[0].obs.device
    paired = [_use_pair(h) for h in heads]
    plans = [_HeadPlan(h) if h.obs.shape[0] > 0 else None for h in heads]
    main = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    side = _side_streams(dev, min(TRAIN_STREAMS, H) - 1)
    streams = [main] + side
    stats = None        # all-reduced advantage sums of the previous step's critic passes [2H]
    out = [[None, None] for _ in range(H)]
    for k in range(n_epochs + 1):
        sums = torch.zeros(2 * H, 3, dtype=torch.float64, device=dev)  # critic rows, actor rows
        crit = k < n_epochs
        trained = []
        if side:  # the side streams start after this step's inputs (Adam, sums, stats) on main
            fork = torch.cuda.Event()
            fork.record(main)
            for sd in side:
                sd.wait_event(fork)
        for i, h in enumerate(heads):
            p = plans[i]
            sc, sa = sums[i], sums[H + i]
            sti = streams[i % len(streams)]
            ctx = torch.cuda.stream(sti) if sti is not None else contextlib.nullcontext()
            st = sti.cuda_stream if sti is not None else None
            with ctx:
                stp = stats[2 * i:2 * i + 2] if k > 0 else None
                if p is None:  # an empty shard: zero gradients, sums unchanged (k_mlp_train's M == 0 path)
                    if k > 0:
                        cont = h.kind == "c"
                        k_mlp_train(KIND_CONT if cont else KIND_CHOICE, h.actor, h.obs, h.ret, h.obs.new_empty(0),
                                    h.act if (cont or h.per_row) else None, h.logp, stp,
                                    None if (cont or h.per_row) else h.counts, m_global=h.m, sums=sa, exact=h.exact)
                        trained.append(h.actor)
                        out[i][0] = sums[H + i, 0:1]
                    if crit:
                        k_mlp_train(KIND_CRITIC, h.critic, h.obs, h.ret, m_global=h.m, sums=sc, exact=h.exact)
                        trained.append(h.critic)
                        out[i][1] = sums[i, 0:1]
                    continue
                if k > 0 and crit and paired[i]:
                    _pair_pass(p, h, stp, sa, sc, st)
                    trained += [h.actor, h.critic]
                    out[i] = [sums[H + i, 0:1], sums[i, 0:1]]
                    continue
                if k > 0:  # the actor pass of epoch k - 1
                    _actor_pass(p, h, stp, sa, st)
                    trained.append(h.actor)
                    out[i][0] = sums[H + i, 0:1]
                if crit:  # the critic pass of epoch k
                    _critic_pass(p, h, sc, st)
                    trained.append(h.critic)
                    out[i][1] = sums[i, 0:1]
        for sd in side:  # join
            main.wait_stream(sd)
        if crit:
            stats = sums[:H, 1:3].reshape(-1).contiguous()
            _allreduce_(stats)
        if bucket is not None:
            bucket.allreduce(trained)
        else:
            _allreduce_net_grads(*trained)
        adam_steps([h.opt_actor for h in heads if h.actor in trained] +
                   [h.opt_critic for h in heads if h.critic in trained])
    del plans
    return [tuple(o) for o in out]


def _no_step_hooks(o):
    """No optimizer step hooks (per instance or global): the fast path bypasses Optimizer.step."""
    from torch.optim import optimizer as _opt
    return not (getattr(o, "_optimizer_step_pre_hooks", None) or getattr(o, "_optimizer_step_post_hooks", None)
                or getattr(_opt, "_global_optimizer_pre_hooks", None)
                or getattr(_opt, "_global_optimizer_post_hooks", None))


def _fused_adam_ok(o):
    return (hasattr(torch, "_fused_adam_") and hasattr(torch, "_foreach_add_") and _no_step_hooks(o)
            and isinstance(o, torch.optim.Adam) and getattr(o, "grad_scale", None) is None
            and getattr(o, "found_inf", None) is None
            and all(g.get("fused") and not g.get("amsgrad") and not g.get("capturable") and not g.get("differentiable")
                    and not g.get("decoupled_weight_decay", False) and not isinstance(g["lr"], torch.Tensor)
                    for g in o.param_groups))


class _AdamPlan:
    """The grouped tensor lists of one adam_steps(opts) call, reused while every optimiser keeps
    the same state / param_groups objects, hyper-parameters and .grad tensors (an optimiser's
    load_state_dict replaces those objects; a rebound .grad is a different tensor)."""

    def __init__(self, opts, keys, groups, steps, grads):
        self.opts, self.keys, self.groups, self.steps = opts, keys, groups, steps
        # strong references, compared by identity: an id() of a state dict freed by a later
        # load_state_dict could be reused by a newer one and pass a stale plan
        self.refs = [(o.state, o.param_groups) for o in opts]
        self.grads = grads  # [(param, grad)]

    def valid(self, opts):
        if len(opts) != len(self.refs) or not all(o.state is st and o.param_groups is pg
                                                  for o, (st, pg) in zip(opts, self.refs)):
            return False
        if _group_keys(opts) != self.keys or not all(_no_step_hooks(o) for o in opts):
            return False
        return all(p.grad is g for p, g in self.grads)


def _group_keys(opts):
    return [(float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["weight_decay"]), float(g["eps"]),
             bool(g["maximize"])) for o in opts for g in o.param_groups]


_ADAM_PLANS = {}


def adam_steps(opts):
    """One step of every optimiser in `opts`, bit-identical to calling o.step() on each.  For
    fused torch Adams (the GPU path) whose state exists, the steps of all six nets run as ONE
    step-count increment and one torch._fused_adam_ launch per distinct hyper-parameter set —
    the same per-tensor kernel arithmetic as each optimiser's own step (torch.optim.adam
    _fused_adam), in 1 + (distinct lr) launches instead of 2 per optimiser.  Anything else (CPU,
    the first step, which creates the state, non-default options, registered optimizer step
    hooks, a torch without the private torch._fused_adam_ op) takes o.step().  The fast path
    reads each group's lr at every call, so an LR scheduler's changes apply; it does not run
    Optimizer.step itself (no step hooks — hence the fallback above — and no scheduler
    step-order bookkeeping).  The grouped tensor lists are built once per optimiser set and
    reused (_AdamPlan: ~0.2 ms of host time per call otherwise).  Pinned by
    test_adam_steps_bit_identical_to_per_optimizer_steps."""
    key = tuple(id(o) for o in opts)
    plan = _ADAM_PLANS.get(key)
    if plan is not None and plan.opts == list(opts) and plan.valid(opts):
        _run_adam_plan(plan)
        return
    fast = all(_fused_adam_ok(o) for o in opts)
    groups, steps, grads = {}, [], []
    if fast:
        for o in opts:
            for g in o.param_groups:
                ps = [p for p in g["params"] if p.grad is not None]
                if any(len(o.state[p]) == 0 for p in ps):
                    fast = False
                    break
                if not ps:
                    continue
                hk = (ps[0].device, float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]),
                      float(g["weight_decay"]), float(g["eps"]), bool(g["maximize"]))
                e = groups.setdefault(hk, ([], [], [], [], []))
                for p in ps:
                    st = o.state[p]
                    if p.dtype != torch.float32 or p.device != hk[0]:
                        fast = False
                    e[0].append(p)
                    e[1].append(p.grad)
                    e[2].append(st["exp_avg"])
                    e[3].append(st["exp_avg_sq"])
                    e[4].append(st["step"])
                    steps.append(st["step"])
                    grads.append((p, p.grad))
            if not fast:
                break
    if not fast:
        _ADAM_PLANS.pop(key, None)
        for o in opts:
            o.step()
        return
    plan = _AdamPlan(list(opts), _group_keys(opts), groups, steps, grads)
    if len(_ADAM_PLANS) > 64:
        _ADAM_PLANS.clear()
    _ADAM_PLANS[key] = plan
    _run_adam_plan(plan)


def _run_adam_plan(plan):
    torch._foreach_add_(plan.steps, 1)
    for (_, lr, b1, b2, wd, eps, maximize), (ps, gs, ms, vs, sts) in plan.groups.items():
        torch._fused_adam_(ps, gs, ms, vs, [], sts, amsgrad=False, lr=lr, beta1=b1, beta2=b2, weight_decay=wd,
                           eps=eps, maximize=maximize, grad_scale=None, found_inf=None)


def train_model_c(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, exact=False):
    """One full-batch epoch of Algo_PPO.train_model_c (:778-815) for one head.
    Returns this rank's (actor, critic) loss sums (float64 tensors)."""
    return train_epoch([Head("c", actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global,
                             exact=exact)])[0]


def train_model_d(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, counts, per_row=False,
                  exact=False):
    """One full-batch epoch of Algo_PPO.train_model_d (:818-851) for one head: O(M) form of
    the M x M Categorical surrogate with the global action counts (n0, n1); per_row=True is
    the opt-in bug fix.  Returns this rank's (actor, critic) loss sums."""
    h = Head("d", actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, counts, per_row,
             exact=exact)
    return train_epoch([h])[0]
