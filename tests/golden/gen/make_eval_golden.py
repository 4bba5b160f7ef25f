"""tests/golden/eval_<name>.npz: the reference's deterministic evaluation on the shipped weights.

For each env e: the reference's Env_rollout.iterations (scalable driver:
Coop-MH-PPO-scalable.py:152-252; coop driver: Coop-MH-PPO.ipynb cell 0; naif:
MH-PPO.ipynb cell 1) — AST-extracted and unmodified, the routine Algo_PPO.evaluate
(:738-747) calls — plays `episodes` consecutive episodes on the CPython random stream
random.seed(seed_base + e), with the actor heads loaded from the reference's shipped
checkpoints (load_model/weights/*.pth, torch.load(weights_only=True), the files
Algo_PPO.loading (:935-955) reads).  Deterministic: argmax choice, mean actions.
Recorded per env: the five tensors iterations returns (states, actions, rews_c,
rews_d, waiting times).  The weights travel as packed float32 arrays (data, not code).
"""
import contextlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import refharness as R  # noqa: E402
import refclasses  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
WDIR = "/root/reference/load_model/weights"
CASES = {  # name: (driver, variant, nb_car, nb_ped, nb_lines, envs, episodes, seed_base, weights prefix)
    "coop_212": ("coop", "coop", 2, 1, 2, 4, 2, 900, "pappo-coop-{h}-122-{k}-step-3000.pth"),
    "naif_111": ("naif", "naif", 1, 1, 1, 4, 2, 910, "pappo-coop-{h}-111-{k}-step-1000.pth"),
    "scalable_211": ("scalable", "scalable", 2, 1, 1, 4, 2, 920, "pappo-scalable-coop-{h}-111-{k}-step-1000.pth"),
    # nb_ped 2: envs drawing ped_traffic = 1 < nb_ped re-decide every step (:218-220)
    "scalable_221": ("scalable", "scalable", 2, 2, 1, 4, 2, 930, "pappo-scalable-coop-{h}-111-{k}-step-1000.pth"),
    # evaluate(n, choix=True): Env_rollout.choix_test (:629-633) after every reset (:170-172)
    "scalable_choix_211": ("scalable", "scalable", 2, 1, 1, 4, 2, 940, "pappo-scalable-coop-{h}-111-{k}-step-1000.pth",
                           True),
    "scalable_choix_221": ("scalable", "scalable", 2, 2, 1, 4, 2, 950, "pappo-scalable-coop-{h}-111-{k}-step-1000.pth",
                           True),
    # two lanes (choix_test puts car 1 on lane 1): no shipped weights of that width, so the
    # heads are torch.manual_seed(960) random inits (packed into the fixture like the others)
    "scalable_choix_422": ("scalable", "scalable", 4, 2, 2, 4, 2, 960, None, True),
}


def packed(net):
    return torch.cat([p.detach().reshape(-1) for lay in (net.layer1, net.layer2, net.layer3, net.layer4)
                      for p in (lay.weight, lay.bias)]).numpy()


def run(driver, variant, nc, npd, nl, E, K, seed_base, wfmt, choix=False):
    env = R.make(variant, nc, npd, nl)
    S = 2 * nl if variant == "scalable" else nc
    glob = dict(env=env, nb_lines=nl, nb_car=nc, nb_ped=npd)
    ns = refclasses.scalable_classes(**glob) if driver == "scalable" else refclasses.notebook_classes(driver, **glob)
    Model_PPO, Env_rollout = ns["Model_PPO"], ns["Env_rollout"]
    dc = 2 + 6 * (S - 1) + 10 if driver == "scalable" else 2 + 5 * (S - 1) + 10
    torch.manual_seed(seed_base)
    ac = Model_PPO(13, 1, 1, nb_car=S, mean=-1.0, std=3.0)
    aw = Model_PPO(13, 1, 1, nb_car=S, mean=-1.0, std=3.0)
    ad = Model_PPO(dc, 2, 2)
    for net, h in ((ac, "cross"), (aw, "wait"), (ad, "choice")) if wfmt else ():
        sd = torch.load(os.path.join(WDIR, wfmt.format(h=h, k="actor")), weights_only=True, map_location="cpu")
        net.load_state_dict(sd)
    with contextlib.redirect_stdout(open(os.devnull, "w")):
        ro = Env_rollout(env, S, 80, 0.3)
    recs = []
    for e in range(E):
        st = R.Stream(seed_base + e)
        with st.active():
            ro.reset()
            obs, acts, rc, rd, wt = ro.iterations(ac, aw, ad, K, choix=choix)
        recs.append(dict(obs=obs.numpy(), acts=acts.numpy().reshape(len(obs), -1), rews_c=rc.numpy(),
                         rews_d=rd.numpy().reshape(-1, S), waiting=wt.numpy().reshape(-1)))
    out = dict(driver=driver, variant=variant, nb_car=nc, nb_ped=npd, nb_lines=nl, seed_base=seed_base,
               episodes=K, choix=bool(choix), w_cross=packed(ac), w_wait=packed(aw), w_choice=packed(ad))
    for k in recs[0]:
        out[k] = np.concatenate([r[k] for r in recs])
        out["n_" + k] = np.array([len(r[k]) for r in recs])
    return out


def main(only=None):
    for name, case in CASES.items():
        if only and name not in only:
            continue
        d = run(*case)
        path = os.path.join(OUT, f"eval_{name}.npz")
        np.savez_compressed(path, **d)
        print(name, {k: d[k].shape for k in ("obs", "acts", "rews_c", "rews_d", "waiting")},
              "saves/env", d["n_rews_d"], os.path.getsize(path))


if __name__ == "__main__":
    main(sys.argv[1:])
