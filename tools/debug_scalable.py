import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo.env import VecCrosswalk
from oracle import OracleEnv
np.set_printoptions(linewidth=200, precision=6)
for (nc, npd, nl, sb) in [(4, 3, 2, 450), (8, 1, 4, 400)]:
    env = VecCrosswalk("scalable", 8, nc, npd, nl, seed_base=sb)
    o = env.reset().cpu().numpy(); st = env.get_state().cpu().numpy(); mt, mti = env.get_rng()
    for e in range(4):
        orc = OracleEnv("scalable", nc, npd, nl, seed=sb + e)
        oo = orc.reset(); d = orc.dump(); omt, omti = orc.rng_state()
        print("env", e, "mti gpu", int(mti[e]), "oracle", omti, "obs diff idx", np.nonzero(oo != o[e])[0])
        k = 20 * npd
        print(" gpu cars Sc/exist", st[e, k + 2:k + 8 * env.n_slots:8], st[e, k + 7:k + 8 * env.n_slots:8])
        print(" orc cars Sc/exist", d[k + 2::8], d[k + 7::8])
        print(" gpu tail", st[e, -4:], " peds gpu", st[e, :20 * npd].reshape(npd, 20)[:, [0, 1, 15, 18]].ravel())
        print(" peds orc", d[:20 * npd].reshape(npd, 20)[:, [0, 1, 15, 18]].ravel())
