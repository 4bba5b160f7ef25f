"""The rollout's policy heads on the device vs the reference's own forward: torch-CPU
Model_PPO on batch-1 tensors, as Env_rollout.iterations_rand calls it
(Coop-MH-PPO-scalable.py:403-453).

The device restates glibc tanhf/expf (csrc/libm_glibc.h) so that it matches the C oracle bit
for bit; torch's CPU path is a different float program: its Linear layers sum in MKL's order
and, in this container (torch 2.10, AVX512 capability), a one-element tanh/exp goes through
ATen's vectorised (Sleef) kernel, not glibc.  So against torch the policy outputs agree to
float32 rounding through four layers, not bit for bit, and this test pins exactly that:
probabilities within 1e-5 relative (measured 1.6e-6: a last-bit logit difference grows through
the softmax's exp), actions within 1e-5, and every Categorical draw (u >= p0 / (p0 + p1), the
same recorded u) identical on 4 096 choice rows — the discrete outputs the north star asks to
be exact.  A draw can only flip when u falls within ~1e-6 of the threshold."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _cpu_copy(net):
    import copy
    return copy.deepcopy(net).cpu().float()


def test_policy_heads_vs_torch_batch1():
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    N, S = 2048, 2
    venv = VecCrosswalk("coop", N, 2, 1, 2, seed_base=7000)
    ro = RolloutGPU(venv)
    torch.manual_seed(11)
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    ad = Model_PPO(ro.dc, 2, 2).cuda()
    batch = ro.collect(ac, aw, ad, seed=4, iteration=0)
    torch.cuda.synchronize()
    cac, caw, cad = _cpu_copy(ac), _cpu_copy(aw), _cpu_copy(ad)

    # ---- choice head at t = 0: probabilities and the Categorical draws
    feat_d = batch.feat_d.reshape(N * S, -1).cpu()
    probs_g = ro.probs_d.reshape(N * S, 2).cpu()
    u = ro.u.reshape(N * S).cpu()
    a_g = batch.a_d.reshape(N * S).cpu()
    with torch.no_grad():
        probs_t = torch.stack([cad(feat_d[r:r + 1]).reshape(2) for r in range(N * S)])
    rel = ((probs_g - probs_t).abs() / probs_t.abs().clamp_min(1e-30)).max().item()
    print(f"choice probabilities: max relative difference {rel:.3g}")
    assert rel <= 1e-5, f"choice probabilities differ by {rel:.3g} relative"
    n0 = probs_t[:, 0] / (probs_t[:, 0] + probs_t[:, 1])
    a_t = (u >= n0).to(torch.int32)
    flips = int((a_t != a_g).sum())
    assert flips == 0, f"{flips} Categorical draws differ from torch's batch-1 forward"

    # ---- continuous heads: the step's action a = min(2, mu) + L eps on a sample of rows
    T = ro.T
    rng = np.random.default_rng(0)
    pick = rng.choice(N * S * T, size=3000, replace=False)
    feat = batch.obs_c.reshape(N * S * T, 13).cpu()[pick]
    act_g = batch.act.reshape(N * S * T).cpu()[pick]
    eps = ro.eps.permute(1, 2, 0).reshape(N * S * T).cpu()[pick]
    head = (2 * batch.a_d[:, :, 0].cpu().to(torch.int64) - 1).reshape(N * S)  # action_d[i] (P = 1)
    cross = (head[torch.from_numpy(pick // T)] <= 0)
    L = torch.tensor(math.sqrt(0.5), dtype=torch.float32)
    with torch.no_grad():
        mu = torch.stack([(cac if cross[k] else caw)(feat[k:k + 1]).reshape(()) for k in range(len(pick))])
    loc = torch.minimum(mu, torch.tensor(2.0))
    act_t = loc + L * eps
    err = (act_g - act_t).abs() / (1.0 + act_t.abs())
    print(f"actions: max scaled difference {err.max().item():.3g}, bit-identical {(act_g == act_t).float().mean():.3f}")
    assert err.max().item() <= 1e-5, f"actions differ by {err.max().item():.3g}"
