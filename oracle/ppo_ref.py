"""ORACLE — test infrastructure only (tests/, smoke(), bench.py cpu_baseline).

PyTorch-CPU restatement of the reference PPO update (Coop-MH-PPO-scalable.py):
  train_model_c  :778-815  continuous heads (MVN(mu, 0.5), float64 ratio)
  train_model_d  :818-851  choice head; the reference's `Categorical.log_prob`
                 of an (M,1) action broadcasts to (M,M) (lp[i,j] = logits[j, a_i]);
                 the loss mean over M^2 equals (1/M^2) sum_j sum_k n_k f(r_jk, A_j)
                 with n_k = #{i: a_i = k}, which is what this restatement computes
                 (exact in real arithmetic; pinned against the reference's own
                 M x M computation by tests/test_oracle_ppo.py).
Pinned against tests/golden/ppo_update.npz (the reference's functions, run unmodified).
"""
import math

import torch


def _mvn_logp(mu, act):
    L = torch.tensor(0.5).sqrt()  # cholesky([[0.5]])
    x = (act.double() - mu.double()).float() * (1.0 / L)
    return -0.5 * (math.log(2 * math.pi) + x * x) - torch.log(L)


def _clip_surrogate(ratio, adv):
    return -torch.min(ratio * adv, torch.clamp(ratio, 0.8, 1.2) * adv)


def train_model_c(actor, critic, opt_a, opt_c, obs, act, logp_old, rtgs):
    V = torch.squeeze(critic(obs), -1)
    A = rtgs - V
    A = (A - A.mean()) / (A.std() + 1e-10)
    mu = torch.squeeze(actor(obs), -1)
    lp = _mvn_logp(mu, act)
    ratio = torch.exp(lp - logp_old.double())
    actor_loss = _clip_surrogate(ratio, A).mean()
    critic_loss = torch.nn.functional.mse_loss(V, rtgs)
    opt_a.zero_grad()
    actor_loss.backward(retain_graph=True)
    opt_a.step()
    opt_c.zero_grad()
    critic_loss.backward()
    opt_c.step()
    return float(actor_loss.detach()), float(critic_loss.detach())


def train_model_d(actor, critic, opt_a, opt_c, obs, act, logp_old, rtgs):
    V = torch.squeeze(critic(obs), -1)
    A = rtgs - V
    A = (A - A.mean()) / (A.std() + 1e-10)
    probs = actor(obs).reshape(-1, 2)
    pn = probs / probs.sum(-1, keepdim=True)
    eps = torch.finfo(torch.float32).eps
    logits = torch.log(pn.clamp(min=eps, max=1 - eps))
    M = obs.shape[0]
    counts = torch.stack([(act == 0).sum(), (act == 1).sum()]).double()
    ratio = torch.exp(logits.double() - logp_old.double()[:, None])           # [M, 2] = r_jk
    f = _clip_surrogate(ratio, A.double()[:, None])                         # [M, 2]
    actor_loss = (f * counts[None, :]).sum() / (M * M)
    critic_loss = torch.nn.functional.mse_loss(V, rtgs)
    opt_a.zero_grad()
    actor_loss.backward(retain_graph=True)
    opt_a.step()
    opt_c.zero_grad()
    critic_loss.backward()
    opt_c.step()
    return float(actor_loss.detach()), float(critic_loss.detach())


def returns_scan(rew_segments, gamma=0.99):
    """futur_rewards (:668-672) on [B, T] float64 -> float32."""
    out = torch.empty(rew_segments.shape, dtype=torch.float32)
    g = torch.zeros(rew_segments.shape[0], dtype=torch.float64)
    for t in range(rew_segments.shape[1] - 1, -1, -1):
        g = rew_segments[:, t] + gamma * g
        out[:, t] = g.float()
    return out
