"""Pin the PPO-update oracle (oracle/ppo_ref.py) against the reference's own
train_model_c / train_model_d run unmodified (tests/golden/ppo_update.npz), and
the O(M) choice-loss restatement against the reference's M x M broadcast."""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mh-ppo_amd"))
from mhppo.models import Model_PPO  # noqa: E402
from oracle import ppo_ref  # noqa: E402

G = os.path.join(ROOT, "tests", "golden", "ppo_update.npz")


def _load(net, g, prefix):
    sd = {k[len(prefix):]: torch.tensor(g[k]) for k in g.files if k.startswith(prefix)}
    net.load_state_dict(sd)


def _check(net, g, prefix, atol):
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(v.numpy(), g[prefix + k], rtol=0, atol=atol, err_msg=prefix + k)


@pytest.mark.parametrize("head", ["c", "d"])
def test_oracle_update_matches_reference(head):
    g = np.load(G)
    if head == "c":
        actor, critic = Model_PPO(13, 1, 1, mean=-1.0, std=3.0), Model_PPO(13, 1, 0)
    else:
        dc = g["d_obs"].shape[1]
        actor, critic = Model_PPO(dc, 2, 2), Model_PPO(dc, 1, 0)
    _load(actor, g, f"{head}_init_actor_")
    _load(critic, g, f"{head}_init_critic_")
    oa = torch.optim.Adam(actor.parameters(), 3e-4)
    oc = torch.optim.Adam(critic.parameters(), 1e-3)
    obs = torch.tensor(g[f"{head}_obs"])
    act = torch.tensor(g[f"{head}_act"])
    lp = torch.tensor(g[f"{head}_logp"])
    rt = torch.tensor(g[f"{head}_rtgs"])
    fn = ppo_ref.train_model_c if head == "c" else ppo_ref.train_model_d
    for ep in range(3):
        la, lc = fn(actor, critic, oa, oc, obs, act, lp, rt)
        ref_a, ref_c = g[f"{head}_losses"][ep]
        assert abs(la - ref_a) <= 1e-6 * max(1.0, abs(ref_a)), (ep, la, ref_a)
        assert abs(lc - ref_c) <= 1e-5 * max(1.0, abs(ref_c)), (ep, lc, ref_c)
        _check(actor, g, f"{head}_ep{ep}_actor_", 2e-6)
        _check(critic, g, f"{head}_ep{ep}_critic_", 2e-6)


def test_choice_O_M_form_equals_M_by_M_broadcast():
    torch.manual_seed(3)
    from torch.distributions import Categorical
    for M in (1, 7, 64, 301):
        probs = torch.softmax(torch.randn(M, 2, dtype=torch.float64), -1)
        a = torch.randint(0, 2, (M, 1)).double()
        old = torch.randn(M, dtype=torch.float64) * 0.3 - 0.7
        A = torch.randn(M, dtype=torch.float64)
        lp = Categorical(probs).log_prob(a)                      # (M, M) broadcast, reference semantics
        r = torch.exp(lp - old)
        ref = (-torch.min(r * A, torch.clamp(r, 0.8, 1.2) * A)).mean()
        pn = probs / probs.sum(-1, keepdim=True)
        logits = torch.log(pn.clamp(min=torch.finfo(torch.float64).eps, max=1 - torch.finfo(torch.float64).eps))
        counts = torch.stack([(a == 0).sum(), (a == 1).sum()]).double()
        rj = torch.exp(logits - old[:, None])
        f = -torch.min(rj * A[:, None], torch.clamp(rj, 0.8, 1.2) * A[:, None])
        mine = (f * counts[None, :]).sum() / (M * M)
        assert abs(float(mine) - float(ref)) <= 1e-12 * max(1.0, abs(float(ref)))
