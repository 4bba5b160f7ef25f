"""GPU env parity diagnostic: HIP env vs reference fixtures and vs the C oracle.

Usage (GPU box): python tools/env_parity_diag.py [N_random]
Reports per case: exact-match fraction of obs / rewards / reward_light / state,
first divergence, and max abs error on continuous fields.
"""
import glob
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo.env import VecCrosswalk  # noqa: E402
from oracle import OracleEnv  # noqa: E402


def compare_fixture(path):
    g = np.load(path)
    v = str(g["variant"])
    nc, npd, nl = int(g["nb_car"]), int(g["nb_ped"]), int(g["nb_lines"])
    E, T = g["obs"].shape[:2]
    env = VecCrosswalk(v, E, nc, npd, nl, seed_base=int(g["seed_base"]))
    o0 = env.reset().cpu().numpy()
    res = {"obs0": int((o0 != g["obs0"]).sum())}
    nob = nre = nrl = nst = nd = 0
    first = None
    S = env.n_slots
    for t in range(T):
        a = torch.from_numpy(g["actions"][:, t]).cuda()
        o, r, rl, d = env.step(a)
        st = env.get_state().cpu().numpy()
        o, r, rl, d = o.cpu().numpy(), r.cpu().numpy(), rl.cpu().numpy(), d.cpu().numpy()
        dm = g["dump"][:, t]
        k = dm.shape[1]
        bo, br, bl, bs = (o != g["obs"][:, t]), (r != g["rewards"][:, t]), (rl != g["reward_light"][:, t]), (st[:, :k] != dm)
        nob += bo.sum(); nre += br.sum(); nrl += bl.sum(); nst += bs.sum(); nd += (d != g["done"][:, t]).sum()
        if first is None and (bo.any() or br.any() or bl.any() or bs.any()):
            e = int(np.nonzero(bo.any(1) | br.any(1) | bl.any(1) | bs.any(1))[0][0])
            first = dict(t=t, e=e, obs_idx=np.nonzero(bo[e])[0][:6].tolist(),
                         rew=(r[e] - g["rewards"][e, t]).tolist(), rl=(rl[e] - g["reward_light"][e, t]).tolist(),
                         st_idx=np.nonzero(bs[e])[0][:8].tolist(),
                         st_gpu=st[e, np.nonzero(bs[e])[0][:8]].tolist(), st_ref=dm[e, np.nonzero(bs[e])[0][:8]].tolist())
    mt, mti = env.get_rng()
    mt = mt.cpu().numpy().view(np.uint32)
    res.update(obs=int(nob), rew=int(nre), rl=int(nrl), state=int(nst), done=int(nd),
               final_mt=int((mt != g["final_mt"]).sum()), first=first)
    return res


def compare_oracle(variant, nc, npd, nl, N, T=80, seed_base=1000):
    env = VecCrosswalk(variant, N, nc, npd, nl, seed_base=seed_base)
    S = env.n_slots
    rng = np.random.default_rng(seed_base)
    orc = [OracleEnv(variant, nc, npd, nl, seed=seed_base + e) for e in range(N)]
    go = env.reset().cpu().numpy()
    oo = np.stack([o.reset() for o in orc])
    stats = dict(obs0=int((go != oo).sum()))
    light = rng.choice([-1.0, 1.0], size=(N, S))
    diverged = np.zeros(N, bool)
    maxerr = 0.0
    nexact = ntot = 0
    for t in range(T):
        acc = rng.uniform(-4.5, 2.5, size=(N, S)).astype(np.float32).astype(np.float64)
        a = np.concatenate([acc, light], 1)
        o, r, rl, d = env.step(torch.from_numpy(a).cuda())
        o, r, rl = o.cpu().numpy(), r.cpu().numpy(), rl.cpu().numpy()
        for e in range(N):
            oo_, ro, rlo, do = orc[e].step(a[e])
            ex = np.array_equal(oo_, o[e]) and np.array_equal(ro, r[e]) and np.array_equal(rlo, rl[e])
            nexact += ex; ntot += 1
            if not ex:
                err = max(np.abs(oo_.astype(np.float64) - o[e]).max(), np.abs(ro - r[e]).max(), np.abs(rlo - rl[e]).max())
                maxerr = max(maxerr, float(err))
                if err > 1e-6:
                    diverged[e] = True
    stats.update(exact_env_steps=nexact, total=ntot, diverged_envs=int(diverged.sum()), max_abs_err=maxerr)
    return stats


def main():
    torch.cuda.init()
    for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "env_*.npz"))):
        print(os.path.basename(f), compare_fixture(f), flush=True)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for case in [("coop", 2, 1, 2), ("4cars", 4, 1, 2), ("scalable", 8, 1, 4), ("naif", 1, 1, 1), ("coop", 4, 3, 2)]:
        t0 = time.time()
        print("oracle", case, compare_oracle(*case, N=n), f"{time.time()-t0:.1f}s", flush=True)


if __name__ == "__main__":
    main()
