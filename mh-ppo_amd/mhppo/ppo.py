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
    _lib.check(_lib.lib().mhppo_adv_stats(_lib.ptr(ret), _lib.ptr(v), ret.numel(), _lib.ptr(stats),
                                          _lib.stream_ptr()))
    return stats


def k_adv_normalize(ret, value, stats, m_global):
    adv = torch.empty_like(ret)
    v = value.detach().contiguous()
    _lib.check(_lib.lib().mhppo_adv_normalize(_lib.ptr(ret), _lib.ptr(v), ret.numel(), _lib.ptr(stats),
                                              float(m_global), _lib.ptr(adv), _lib.stream_ptr()))
    return adv


def k_mse(value, ret, m_global):
    dv = torch.empty_like(ret)
    loss = torch.zeros(1, dtype=torch.float64, device=ret.device)
    v = value.detach().contiguous()
    _lib.check(_lib.lib().mhppo_mse_fwd_bwd(_lib.ptr(v), _lib.ptr(ret), ret.numel(), 1.0 / m_global, _lib.ptr(dv),
                                            _lib.ptr(loss), _lib.stream_ptr()))
    return dv, loss


def k_ppo_cont(mu, act, logp_old, adv, m_global):
    dmu = torch.empty_like(adv)
    loss = torch.zeros(1, dtype=torch.float64, device=adv.device)
    m = mu.detach().contiguous()
    _lib.check(_lib.lib().mhppo_ppo_cont_fwd_bwd(_lib.ptr(m), _lib.ptr(act), _lib.ptr(logp_old), _lib.ptr(adv),
                                                 adv.numel(), 1.0 / m_global, _lib.ptr(dmu), _lib.ptr(loss),
                                                 _lib.stream_ptr()))
    return dmu, loss


def k_ppo_choice(probs, logp_old, adv, counts, m_global):
    p = probs.detach().contiguous()
    dp = torch.empty_like(p)
    loss = torch.zeros(1, dtype=torch.float64, device=adv.device)
    _lib.check(_lib.lib().mhppo_ppo_choice_fwd_bwd(_lib.ptr(p), _lib.ptr(logp_old), _lib.ptr(adv), adv.numel(),
                                                   _lib.ptr(counts), 1.0 / (m_global * m_global), _lib.ptr(dp),
                                                   _lib.ptr(loss), _lib.stream_ptr()))
    return dp, loss


# ------------------------------------------------------------- DP orchestration

def normalized_advantage(ret, value, m_global):
    stats = _allreduce_(k_adv_stats(ret, value))
    return k_adv_normalize(ret, value, stats, m_global)


def train_model_c(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global):
    """One full-batch epoch of Algo_PPO.train_model_c (:778-815). Returns (actor_loss, critic_loss)."""
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


def train_model_d(actor, critic, opt_actor, opt_critic, obs, act, logp_old, ret, m_global, counts):
    """One full-batch epoch of Algo_PPO.train_model_d (:818-851); counts = global (n0, n1) float64."""
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
