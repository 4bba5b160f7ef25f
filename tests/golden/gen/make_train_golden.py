"""tests/golden/train_<name>.npz: one whole reference training iteration, end to end.

For each case, in the BUILD container only:
  1. The reference driver's classes (scalable: Coop-MH-PPO-scalable.py; coop:
     Coop-MH-PPO.ipynb cell 0), AST-extracted and unmodified, build
     Algo_PPO(Model_PPO, env, ...) as the driver does (:1036-1052) under
     torch.manual_seed(tseed); the six nets' initial weights are recorded.
  2. Env e of E envs runs on its own CPython stream random.seed(seed_base + e) and
     sees what env e of the batched product sees: the reset of Env_rollout.__init__
     (:107), the reset of Algo_PPO.train's rollout.reset() (:861 -> :129), then one
     80-step episode of Env_rollout.iterations_rand (:357-517) with batch_size 80,
     its torch draws replaced by recorded ones (MultivariateNormal eps[t, e, i],
     Categorical a_d[e, i, p]).  The episodes' batch_* lists are concatenated in env
     order — the batch one Algo_PPO.train iteration collects (:489-507).
  3. Algo_PPO.train(1) runs UNMODIFIED on that batch (its rollout.reset /
     iterations_rand are pointed at the recorded batch): futur_rewards (:658-684),
     10 epochs of train_model_c cross + wait (:868-877), 10 epochs of train_model_d
     (:879-882), reward curves.  Final weights of all six nets are recorded.
Outputs: initial/final weights, the noise, the bucketed batches (obs/act/logp/rtgs per
head), the reward-curve entries.
"""
import contextlib
import io
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refharness as R  # noqa: E402
import refclasses  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CASES = {  # name: (driver, variant, nb_car, nb_ped, nb_lines, E, seed_base, torch_seed)
    "coop_212": ("coop", "coop", 2, 1, 2, 16, 800, 21),
    "scalable_814": ("scalable", "scalable", 8, 1, 4, 16, 820, 22),
}
NETS = ("actor_net_cross", "actor_net_wait", "actor_net_choice", "critic_net_cross", "critic_net_wait",
        "critic_net_choice")
LISTS = ("batch_obs_cross", "batch_obs_wait", "batch_obs_choice", "batch_acts_cross", "batch_acts_wait",
         "batch_acts_choice", "batch_log_probs_cross", "batch_log_probs_wait", "batch_log_probs_choice",
         "batch_rews_cross", "batch_rews_wait", "batch_rews_choice")


def run(driver, variant, nc, npd, nl, E, seed_base, tseed):
    env = R.make(variant, nc, npd, nl)
    S = 2 * nl if variant == "scalable" else nc
    glob = dict(env=env, nb_lines=nl, nb_car=nc, nb_ped=npd)
    ns = refclasses.scalable_classes(**glob) if driver == "scalable" else refclasses.notebook_classes(driver, **glob)
    Model_PPO, Algo_PPO = ns["Model_PPO"], ns["Algo_PPO"]
    dc = 2 + 6 * (S - 1) + 10 if driver == "scalable" else 2 + 5 * (S - 1) + 10
    torch.manual_seed(tseed)
    with contextlib.redirect_stdout(io.StringIO()):
        algo = Algo_PPO(Model_PPO, env, num_algo=100 * npd + 10 * nc + nl, num_states_c=13, num_states_d=dc,
                        num_actions=1, mean=-1.0, std=3.0, nb_cars=nc, dt=0.3)
    out = dict(driver=driver, variant=variant, nb_car=nc, nb_ped=npd, nb_lines=nl, seed_base=seed_base, E=E)
    for n in NETS:
        out.update({f"{n}_init_{k}": v.detach().numpy().copy() for k, v in getattr(algo, n).state_dict().items()})
    rng = np.random.default_rng(seed_base)
    eps = rng.normal(size=(80, E, S)).astype(np.float32)
    a_d = (rng.uniform(size=(E, S, npd)) < 0.5).astype(np.int32)
    import torch.distributions.multivariate_normal as mvn
    from torch.distributions import Categorical
    orig_sn, orig_cs = mvn._standard_normal, Categorical.sample
    ro = algo.rollout
    acc = {k: [] for k in LISTS}
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
            st = R.Stream(seed_base + e)
            with st.active():
                env.reset()   # Env_rollout.__init__ (:107)
                ro.reset()    # Algo_PPO.train -> rollout.reset() (:861, :129)
                ro.iterations_rand(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, algo.cov_mat,
                                   algo.cov_mat_d, 80)
        finally:
            mvn._standard_normal, Categorical.sample = orig_sn, orig_cs
        assert ctr["n"] == 80 * S and ctr["c"] == S * npd, (ctr, S)
        for k in LISTS:
            acc[k] += list(getattr(ro, k))

    def install(*a, **k):  # the recorded batch stands in for this iteration's collection
        for name in LISTS:
            setattr(ro, name, list(acc[name]))

    ro.iterations_rand = install
    ro.reset = lambda: None
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "load_model", "parameters"))
        os.chdir(tmp)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                install()
                rtgs = ro.futur_rewards()
                algo.train(1)
        finally:
            os.chdir(cwd)
    for n in NETS:
        out.update({f"{n}_final_{k}": v.detach().numpy().copy() for k, v in getattr(algo, n).state_dict().items()})
    out.update(eps=eps, a_d=a_d,
               obs_cross=np.array(acc["batch_obs_cross"], np.float64).reshape(-1, 13).astype(np.float32),
               obs_wait=np.array(acc["batch_obs_wait"], np.float64).reshape(-1, 13).astype(np.float32),
               obs_choice=np.array(acc["batch_obs_choice"], np.float64).reshape(-1, dc).astype(np.float32),
               act_cross=np.array(acc["batch_acts_cross"], np.float64).reshape(-1),
               act_wait=np.array(acc["batch_acts_wait"], np.float64).reshape(-1),
               act_choice=np.array(acc["batch_acts_choice"], np.float64).reshape(-1),
               logp_cross=np.array(acc["batch_log_probs_cross"], np.float64).reshape(-1),
               logp_wait=np.array(acc["batch_log_probs_wait"], np.float64).reshape(-1),
               logp_choice=np.array(acc["batch_log_probs_choice"], np.float64).reshape(-1),
               rtgs_cross=rtgs[0].numpy().reshape(-1), rtgs_wait=rtgs[1].numpy().reshape(-1),
               rtgs_choice=rtgs[2].numpy().reshape(-1),
               ep_reward_cross=np.array(algo.ep_reward_cross, np.float64),
               ep_reward_wait=np.array(algo.ep_reward_wait, np.float64),
               ep_reward_choice=np.array(algo.ep_reward_choice, np.float64),
               scenario_balance=np.array(algo.ep_scenario_balance, np.int64))
    return out


def main():
    for name, case in CASES.items():
        d = run(*case)
        path = os.path.join(OUT, f"train_{name}.npz")
        np.savez_compressed(path, **d)
        print(name, "cross", d["obs_cross"].shape, "wait", d["obs_wait"].shape, "choice", d["obs_choice"].shape,
              "balance", d["scenario_balance"].tolist(), os.path.getsize(path))


if __name__ == "__main__":
    main()
