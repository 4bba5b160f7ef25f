"""tests/golden/rollout_<name>.npz: the reference rollout collector on recorded noise.

For each episode e: the reference's Env_rollout.iterations_rand (scalable driver:
Coop-MH-PPO-scalable.py:357-517; coop driver: Coop-MH-PPO.ipynb cell 0; naif:
MH-PPO.ipynb cell 1), AST-extracted and unmodified, runs ONE 80-step episode
(batch_size=80) of an env on the CPython random stream random.seed(seed_base+e).
Its torch draws are replaced by recorded ones: MultivariateNormal's
_standard_normal returns eps[t, e, i] in call order, Categorical.sample returns
a_d[e, i, p].  Actor weights: Model_PPO (same extraction) under torch.manual_seed.
Recorded: the bucketed batch_* lists and futur_rewards(), per episode.
"""
import contextlib
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refharness as R  # noqa: E402
import refclasses  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CASES = {  # name: (driver, variant, nb_car, nb_ped, nb_lines, episodes, seed_base, torch_seed)
    "coop_212": ("coop", "coop", 2, 1, 2, 6, 700, 1),
    "coop_422": ("coop", "coop", 4, 2, 2, 4, 720, 2),
    "scalable_814": ("scalable", "scalable", 8, 1, 4, 6, 740, 3),
    "scalable_422": ("scalable", "scalable", 4, 2, 2, 4, 760, 4),
    "naif_111": ("naif", "naif", 1, 1, 1, 6, 780, 5),
}


def packed(net):
    return torch.cat([p.detach().reshape(-1) for lay in (net.layer1, net.layer2, net.layer3, net.layer4)
                      for p in (lay.weight, lay.bias)]).numpy()


def run(driver, variant, nc, npd, nl, E, seed_base, tseed):
    env = R.make(variant, nc, npd, nl)
    S = 2 * nl if variant == "scalable" else nc
    glob = dict(env=env, nb_lines=nl, nb_car=nc, nb_ped=npd)
    ns = refclasses.scalable_classes(**glob) if driver == "scalable" else refclasses.notebook_classes(driver, **glob)
    Model_PPO, Env_rollout = ns["Model_PPO"], ns["Env_rollout"]
    dc = 2 + 6 * (S - 1) + 10 if driver == "scalable" else 2 + 5 * (S - 1) + 10
    torch.manual_seed(tseed)
    ac = Model_PPO(13, 1, 1, nb_car=S, mean=-1.0, std=3.0)
    aw = Model_PPO(13, 1, 1, nb_car=S, mean=-1.0, std=3.0)
    ad = Model_PPO(dc, 2, 2)
    rng = np.random.default_rng(seed_base)
    eps = rng.normal(size=(80, E, S)).astype(np.float32)
    a_d = (rng.uniform(size=(E, S, npd)) < 0.5).astype(np.int32)
    cov = torch.diag(torch.full(size=(1,), fill_value=0.5))
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        ro = Env_rollout(env, S, 80, 0.3)
    import torch.distributions.multivariate_normal as mvn
    from torch.distributions import Categorical
    orig_sn, orig_cs = mvn._standard_normal, Categorical.sample
    recs = []
    for e in range(E):
        ctr = {"n": 0, "c": 0}

        def sn(shape, dtype, device):
            t, i = divmod(ctr["n"], S)
            ctr["n"] += 1
            return torch.tensor([eps[t, e, i]], dtype=dtype).reshape(shape)

        def cs(self, sample_shape=torch.Size()):
            i, p = divmod(ctr["c"], npd)
            ctr["c"] += 1
            return torch.tensor(int(a_d[e, i, p]))

        mvn._standard_normal, Categorical.sample = sn, cs
        try:
            with contextlib.redirect_stdout(open(os.devnull, "w")):
                ro.reset()  # consumes draws from whatever stream is current (uses the global env)
            st = R.Stream(seed_base + e)
            with st.active():
                ro.iterations_rand(ac, aw, ad, cov, None, 80)
                rc, rw, rd = ro.futur_rewards()
        finally:
            mvn._standard_normal, Categorical.sample = orig_sn, orig_cs
        assert ctr["n"] == 80 * S and ctr["c"] == S * npd, (ctr, S)
        cars_exist = [bool(getattr(c, "exist", True)) for c in env.cars]
        recs.append(dict(
            obs_cross=np.array(ro.batch_obs_cross, np.float64).reshape(-1, 13),
            act_cross=np.array(ro.batch_acts_cross, np.float64).reshape(-1),
            logp_cross=np.array(ro.batch_log_probs_cross, np.float64).reshape(-1),
            rew_cross=np.array(ro.batch_rews_cross, np.float64).reshape(-1),
            obs_wait=np.array(ro.batch_obs_wait, np.float64).reshape(-1, 13),
            act_wait=np.array(ro.batch_acts_wait, np.float64).reshape(-1),
            logp_wait=np.array(ro.batch_log_probs_wait, np.float64).reshape(-1),
            rew_wait=np.array(ro.batch_rews_wait, np.float64).reshape(-1),
            obs_choice=np.array(ro.batch_obs_choice, np.float64).reshape(-1, dc),
            act_choice=np.array(ro.batch_acts_choice, np.float64).reshape(-1),
            logp_choice=np.array(ro.batch_log_probs_choice, np.float64).reshape(-1),
            rew_choice=np.array(ro.batch_rews_choice, np.float64).reshape(-1),
            ret_cross=rc.numpy().reshape(-1), ret_wait=rw.numpy().reshape(-1), ret_choice=rd.numpy().reshape(-1),
            exist=np.array(cars_exist[:S], np.uint8)))
    out = dict(driver=driver, variant=variant, nb_car=nc, nb_ped=npd, nb_lines=nl, seed_base=seed_base,
               w_cross=packed(ac), w_wait=packed(aw), w_choice=packed(ad), eps=eps, a_d=a_d)
    for k in recs[0]:
        out[k] = np.concatenate([r[k] for r in recs]) if recs[0][k].ndim else np.array([r[k] for r in recs])
        out["n_" + k] = np.array([len(r[k]) for r in recs])
    return out


def main():
    for name, case in CASES.items():
        d = run(*case)
        path = os.path.join(OUT, f"rollout_{name}.npz")
        np.savez_compressed(path, **d)
        print(name, "cross rows", d["obs_cross"].shape, "wait rows", d["obs_wait"].shape, "choice",
              d["obs_choice"].shape, os.path.getsize(path))


if __name__ == "__main__":
    main()
