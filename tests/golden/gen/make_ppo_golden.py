"""tests/golden/ppo_update.npz: the reference's own PPO update math on a fixed batch.

Runs Algo_PPO.train_model_c (Coop-MH-PPO-scalable.py:778-815) and train_model_d
(:818-851) — AST-extracted, unmodified — for 3 epochs each on synthetic batches,
recording initial weights, each epoch's actor/critic loss (captured at
`.backward()`), and the weights after every epoch (Adam, lr 3e-4 / 1e-3).
The choice batch keeps M small enough for the reference's M x M broadcast.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refclasses  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ppo_update.npz")


def params(net):
    return {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}


def main():
    ns = refclasses.scalable_classes(env=None, nb_lines=2)
    Model_PPO, Algo_PPO = ns["Model_PPO"], ns["Algo_PPO"]
    rec = []
    orig_backward = torch.Tensor.backward

    def spy(self, *a, **k):
        rec.append(float(self.detach().double().item()))
        return orig_backward(self, *a, **k)

    torch.Tensor.backward = spy
    rng = np.random.default_rng(7)
    out = {}
    # ---------------- continuous head (cross/wait share the code path)
    torch.manual_seed(11)
    actor = Model_PPO(13, 1, 1, nb_car=4, mean=-1.0, std=3.0)
    critic = Model_PPO(13, 1, 0)
    M = 777
    obs = rng.normal(0, 3, size=(M, 13)).astype(np.float32).astype(np.float64)
    with torch.no_grad():
        mu0 = actor(torch.tensor(obs).float()).numpy().reshape(-1)
    act = (mu0 + np.sqrt(0.5) * rng.normal(size=M).astype(np.float32)).astype(np.float32)
    act = act.astype(np.float64).reshape(M, 1)
    logp = (rng.normal(-0.6, 0.4, size=M)).astype(np.float32).astype(np.float64)
    rtgs = torch.tensor(rng.normal(-30, 15, size=M), dtype=torch.float)
    out.update({f"c_init_actor_{k}": v for k, v in params(actor).items()})
    out.update({f"c_init_critic_{k}": v for k, v in params(critic).items()})
    oa = torch.optim.Adam(actor.parameters(), 3e-4)
    oc = torch.optim.Adam(critic.parameters(), 1e-3)
    cov = torch.diag(torch.full(size=(1,), fill_value=0.5))
    losses = []
    for ep in range(3):
        rec.clear()
        Algo_PPO.train_model_c(None, actor, critic, oa, oc, obs, act, logp, rtgs, cov)
        losses.append(list(rec))
        out.update({f"c_ep{ep}_actor_{k}": v for k, v in params(actor).items()})
        out.update({f"c_ep{ep}_critic_{k}": v for k, v in params(critic).items()})
    out.update(c_obs=obs.astype(np.float32), c_act=act.reshape(-1).astype(np.float32),
               c_logp=logp.astype(np.float32), c_rtgs=rtgs.numpy(), c_losses=np.array(losses))
    # ---------------- choice head (Categorical, M x M broadcast)
    torch.manual_seed(12)
    dc = 27
    actor = Model_PPO(dc, 2, 2)
    critic = Model_PPO(dc, 1, 0)
    M = 333
    obs = rng.normal(0, 3, size=(M, dc)).astype(np.float32).astype(np.float64)
    with torch.no_grad():
        p = actor(torch.tensor(obs).float()).reshape(-1, 2).numpy()
    a = (rng.uniform(size=M) < p[:, 1]).astype(np.float64).reshape(M, 1)
    lp = np.log(np.clip(p[np.arange(M), a.reshape(-1).astype(int)], 1e-7, 1)).astype(np.float32)
    lp = (lp + rng.normal(0, 0.05, size=M).astype(np.float32)).astype(np.float64)
    rtgs = torch.tensor(rng.normal(-5, 4, size=(M, 1)), dtype=torch.float)
    out.update({f"d_init_actor_{k}": v for k, v in params(actor).items()})
    out.update({f"d_init_critic_{k}": v for k, v in params(critic).items()})
    oa = torch.optim.Adam(actor.parameters(), 3e-4)
    oc = torch.optim.Adam(critic.parameters(), 1e-3)
    losses = []
    for ep in range(3):
        rec.clear()
        Algo_PPO.train_model_d(None, actor, critic, oa, oc, obs, a, lp, rtgs, None)
        losses.append(list(rec))
        out.update({f"d_ep{ep}_actor_{k}": v for k, v in params(actor).items()})
        out.update({f"d_ep{ep}_critic_{k}": v for k, v in params(critic).items()})
    out.update(d_obs=obs.astype(np.float32), d_act=a.reshape(-1).astype(np.int32), d_logp=lp.astype(np.float32),
               d_rtgs=rtgs.numpy().reshape(-1), d_losses=np.array(losses))
    torch.Tensor.backward = orig_backward
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "losses c", out["c_losses"].tolist(), "d", out["d_losses"].tolist())


if __name__ == "__main__":
    main()
