"""PPO update of the multi-head actor-critic (Algo_PPO.train_model_c / _d,
Coop-MH-PPO-scalable.py:778-851), full batch, on the GPU.

The MLP forward/backward stays in PyTorch-ROCm (tiny GEMMs + autograd); the
PPO arithmetic around it is hand-written HIP (include/mhppo.h):
  advantage stats + normalisation  (A - mean) / (std_unbiased + 1e-10)   :786-787
  continuous clip surrogate, float64 ratio, dL/dmu                        :795-806
  choice surrogate over the M x M broadcast, exact O(M) form, dL/dprobs   :834-842
  critic MSE and dL/dV                                                    :808-809
Epoch semantics follow the reference: the advantage uses the critic of the
start of the epoch, the actor-loss gradient never reaches the critic (the
reference zeroes it before the critic step, :810-815), Adam for each net.

Data parallel: every rank holds a shard of the batch; advantage sums and the
choice action counts are all-reduced (SUM) so normalisation uses the global
batch, each rank's gradient is the gradient of (global-mean loss restricted to
its rows), and one flat all-reduce (SUM) per update makes it the full-batch
gradient.  Adam then runs replicated.
"""
import torch
import torch.distributed as dist

from . import _lib


def _dp():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _allreduce_(t):
    if _dp():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def _allreduce_net_grads(*nets):
    """One all-reduce (SUM) of the nets' flat gradients (the .grad views alias them)."""
    if not _dp():
        return
    if all(hasattr(n, "grad_flat") for n in nets):
        flats = [n.grad_flat() for n in nets]
        flat = torch.cat(flats)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        off = 0
        for f in flats:
            f.copy_(flat[off:off + f.numel()])
            off += f.numel()
        return
    _allreduce_grads([p for n in nets for p in n.parameters()])


def _allreduce_grads(params):
    if not _dp():
        return
    grads = [p.grad for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def global_count(n, device):
    t = torch.tensor([float(n)], dtype=torch.float64, device=device)
    return float(_allreduce_(t).item())


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
        _lib.check(_lib.lib().mhppo_mse_fwd_bwd(_lib.ptr(v), _lib.ptr(ret), ret.numel(), 1.0 / m_global, _lib.ptr(dv),
                                            _lib.ptr(loss), _lib.stream_ptr()))
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

KIND_CRITIC, KIND_CONT, KIND_CHOICE = 0, 1, 2


def n_params(n_in, n_out):
    return 32 * n_in + 32 + 64 * 32 + 64 + 32 * 64 + 32 + 32 * n_out + n_out


def k_mlp_train(kind, net, obs, ret, value=None, act=None, logp_old=None, stats=None, counts=None, m_global=1.0):
    """Fused forward/loss/backward of one head (mhppo_mlp_train).
    kind 0 (critic): returns (grad, sums[3] = (sum (V-G)^2, sum A, sum A^2), V).
    kind 1 (continuous actor) / 2 (choice actor): returns (grad, sums[3] = (sum surrogate, 0, 0), None).
    grad is the packed torch-layout gradient (W1 b1 .. W4 b4)."""
    want = {KIND_CRITIC: 0, KIND_CONT: 1, KIND_CHOICE: 2}[kind]
    if net.model_type != want or net.n_in > 32 or (kind == KIND_CONT and net.n_in != 13):
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
    # the gradient lands straight in the net's flat .grad storage when it has one
    grad = net.grad_flat() if hasattr(net, "grad_flat") else None
    if grad is None or grad.numel() != np_ or grad.device != dev:
        grad = torch.empty(np_, dtype=torch.float32, device=dev)
    sums = torch.zeros(3, dtype=torch.float64, device=dev)
    w = net.flat() if hasattr(net, "flat") else net.packed()
    p = _lib.ptr
    ev = None
    if TRAIN_EVENTS is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().mhppo_mlp_train(
            kind, net.n_in, p(w), p(obs), M, p(ret), p(V), p(act), p(logp_old), p(stats), p(counts),
            float(m_global), float(net.mean), float(net.std), p(grad), p(sums), _lib.stream_ptr()))
    if ev is not None:
        ev[1].record()
        TRAIN_EVENTS.append((kind, net.n_in, M, ev[0], ev[1]))
    return grad, sums, (V if kind == KIND_CRITIC else None)


# ------------------------------------------------------------- DP orchestration

def normalized_advantage(ret, value, m_global):
    stats = _allreduce_(k_adv_stats(ret, value))
    return k_adv_normalize(ret, value, stats, m_global)


def _set_grads(net, flat):
    if hasattr(net, "_gflat") and flat is net._gflat:
        return  # written in place (k_mlp_train)
    off = 0
    for lay in (net.layer1, net.layer2, net.layer3, net.layer4):
        for p in (lay.weight, lay.bias):
            n = p.numel()
            g = flat[off:off + n].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
            off += n


def train_model_c(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global):
    """One full-batch epoch of Algo_PPO.train_model_c (:778-815) on the fused MFMA kernel:
    critic pass (V, MSE gradient, advantage sums) -> all-reduce of the sums -> actor pass
    (clip-surrogate gradient w.r.t. the start-of-epoch critic's advantage) -> one gradient
    all-reduce -> Adam.  Returns this rank's (actor, critic) loss sums (float64 tensors)."""
    gc, sc, V = k_mlp_train(KIND_CRITIC, critic, obs, ret, m_global=m_global)
    stats = _allreduce_(sc[1:3].clone())
    ga, sa, _ = k_mlp_train(KIND_CONT, actor, obs, ret, V, act, logp_old, stats, m_global=m_global)
    _set_grads(critic, gc)
    _set_grads(actor, ga)
    _allreduce_net_grads(actor, critic)
    opt_actor.step()
    opt_critic.step()
    return sa[0:1], sc[0:1]


def train_model_c_autograd(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global):
    """train_model_c with the MLPs in PyTorch autograd and the PPO arithmetic in HIP
    (kept as the cross-check for the fused kernel)."""
    V = torch.squeeze(critic(obs), -1)
    adv = normalized_advantage(ret, V, m_global)
    mu = torch.squeeze(actor(obs), -1)
    dmu, la = k_ppo_cont(mu, act, logp_old, adv, m_global)
    dv, lc = k_mse(V, ret, m_global)
    opt_actor.zero_grad(set_to_none=False)
    opt_critic.zero_grad(set_to_none=False)
    torch.autograd.backward([mu, V], [dmu, dv])
    _allreduce_grads(list(actor.parameters()) + list(critic.parameters()))
    opt_actor.step()
    opt_critic.step()
    return la, lc  # this rank's loss sums (logging only; reduce if needed)


def train_model_d(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, counts, per_row=False):
    """One full-batch epoch of Algo_PPO.train_model_d (:818-851) on the fused kernel:
    critic pass -> all-reduce of the advantage sums -> choice-actor pass (O(M) form of the
    M x M Categorical surrogate with the global action counts) -> gradient all-reduce ->
    Adam.  counts = global (n0, n1) float64.  per_row=True is the opt-in bug fix (SURVEY
    §8(f)4): the standard per-row PPO surrogate (each row's own action, mean over rows)
    instead of the reference's M x M broadcast.  Returns this rank's (actor, critic) loss sums."""
    if per_row:
        if critic.n_in > 32:
            raise ValueError("per-row choice loss needs the fused kernel (n_in <= 32)")
        gc, sc, V = k_mlp_train(KIND_CRITIC, critic, obs, ret, m_global=m_global)
        stats = _allreduce_(sc[1:3].clone())
        ga, sa, _ = k_mlp_train(KIND_CHOICE, actor, obs, ret, V, act.float(), logp_old, stats, None,
                                m_global=m_global)
        _set_grads(critic, gc)
        _set_grads(actor, ga)
        _allreduce_net_grads(actor, critic)
        opt_actor.step()
        opt_critic.step()
        return sa[0:1], sc[0:1]
    if critic.n_in > 32:
        return train_model_d_autograd(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global,
                                      counts)
    gc, sc, V = k_mlp_train(KIND_CRITIC, critic, obs, ret, m_global=m_global)
    stats = _allreduce_(sc[1:3].clone())
    ga, sa, _ = k_mlp_train(KIND_CHOICE, actor, obs, ret, V, None, logp_old, stats, counts.double().contiguous(),
                            m_global=m_global)
    _set_grads(critic, gc)
    _set_grads(actor, ga)
    _allreduce_net_grads(actor, critic)
    opt_actor.step()
    opt_critic.step()
    return sa[0:1], sc[0:1]


def train_model_d_autograd(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, counts):
    """train_model_d with the MLPs in PyTorch autograd and the PPO arithmetic in HIP (choice
    observations wider than the fused kernel's 32 inputs; cross-check for the fused kernel)."""
    V = torch.squeeze(critic(obs), -1)
    adv = normalized_advantage(ret, V, m_global)
    probs = actor(obs).reshape(-1, 2)
    dp, la = k_ppo_choice(probs, logp_old, adv, counts, m_global)
    dv, lc = k_mse(V, ret, m_global)
    opt_actor.zero_grad(set_to_none=False)
    opt_critic.zero_grad(set_to_none=False)
    torch.autograd.backward([probs, V], [dp, dv])
    _allreduce_grads(list(actor.parameters()) + list(critic.parameters()))
    opt_actor.step()
    opt_critic.step()
    return la, lc  # this rank's loss sums (logging only; reduce if needed)
