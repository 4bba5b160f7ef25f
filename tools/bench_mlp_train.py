"""Micro-benchmark of the fused continuous-head train kernel (mhppo_mlp_train_cont):
both passes at M rows, HIP-event timed on the launch stream; prints TFLOP/s."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
import torch  # noqa: E402

from mhppo import ppo  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10485760)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--exact", action="store_true", help="the exact f32-MFMA kernel (MHPPO_TRAIN_EXACT_F32)")
ap.add_argument("--pair", action="store_true", help="also time the fused actor+critic launch (mhppo_mlp_train_pair)")
ap.add_argument("--choice", type=int, default=0, help="also time a choice head with this many inputs, split vs exact")
ap.add_argument("--choice-rows", type=int, default=655360)
ap.add_argument("--sweep", action="store_true",
                help="per-launch time of critic / actor passes at 1, 2, 4 ... 64 tiles per wave (kernel only, "
                     "HIP events around the x3 launch are not separable: reported per k_mlp_train call)")
ap.add_argument("--data", default="randn", choices=("randn", "zero", "coarse"),
                help="the observation rows: N(0, 9) (default), all zero, or N(0, 9) rounded to integers "
                     "(MFMA timing does not depend on the data; a change here is the chip's power / clock state)")
a = ap.parse_args()
if a.sweep:
    torch.manual_seed(0)
    act_ = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    cri_ = Model_PPO(13, 1, 0).cuda()
    for tpw in (1, 2, 4, 8, 16, 32, 64):
        Ms = 32 * 1024 * tpw
        xo = torch.randn(Ms, 13, device="cuda") * 3
        xr = torch.randn(Ms, device="cuda") * 8 - 20
        xa = torch.randn(Ms, device="cuda") - 1
        xl = torch.randn(Ms, device="cuda") * 0.3 - 0.9
        res = []
        for kind in (0, 1):
            ppo.TRAIN_EVENTS = []
            for r in range(a.reps + 2):
                if r == 2:
                    torch.cuda.synchronize()
                    ppo.TRAIN_EVENTS = []
                if kind == 0:
                    _, sc_, V_ = ppo.k_mlp_train(0, cri_, xo, xr, m_global=float(Ms))
                else:
                    ppo.k_mlp_train(1, act_, xo, xr, V_, xa, xl, sc_[1:3].clone(), m_global=float(Ms))
            torch.cuda.synchronize()
            res.append(sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in ppo.TRAIN_EVENTS) / a.reps * 1e3)
        print(f"tiles/wave {tpw:3d} rows {Ms:8d}: critic {res[0]:8.1f} us  actor {res[1]:8.1f} us", flush=True)
    ppo.TRAIN_EVENTS = None
    sys.exit(0)
M = a.rows
torch.manual_seed(0)
actor = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
critic = Model_PPO(13, 1, 0).cuda()
obs = torch.randn(M, 13, device="cuda") * 3
if a.data == "zero":
    obs.zero_()
elif a.data == "coarse":
    obs.round_()
ret = torch.randn(M, device="cuda") * 8 - 20
act = torch.randn(M, device="cuda") - 1
lp = torch.randn(M, device="cuda") * 0.3 - 0.9
for kind in (0, 1, 0, 1):
    gc, sc, V = ppo.k_mlp_train(0, critic, obs, ret, m_global=float(M), exact=a.exact)
    ga, sa, _ = ppo.k_mlp_train(1, actor, obs, ret, V, act, lp, sc[1:3].clone(), m_global=float(M), exact=a.exact)
torch.cuda.synchronize()
for kind in (0, 1):
    ppo.TRAIN_EVENTS = []
    for _ in range(a.reps):
        if kind == 0:
            ppo.k_mlp_train(0, critic, obs, ret, m_global=float(M), exact=a.exact)
        else:
            ppo.k_mlp_train(1, actor, obs, ret, V, act, lp, sc[1:3].clone(), m_global=float(M), exact=a.exact)
    torch.cuda.synchronize()
    ms = sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in ppo.TRAIN_EVENTS) / a.reps
    tf = ppo.FLOPS_PER_ROW_CONT * M / (ms * 1e-3) / 1e12
    print(f"kind {kind} rows {M}: {ms:.3f} ms  {tf:.1f} TFLOP/s "
          f"({100 * tf / 157.3:.1f}% of f32 MFMA peak)", flush=True)
if a.pair:
    V2 = V.clone()
    sa2, sc2 = (torch.zeros(3, dtype=torch.float64, device="cuda") for _ in range(2))
    st = sc[1:3].clone()
    for _ in range(2):
        ppo.k_mlp_train_pair(actor, critic, obs, ret, V2, act, lp, st, float(M), sa2, sc2)
    torch.cuda.synchronize()
    ppo.TRAIN_EVENTS = []
    for _ in range(a.reps):
        ppo.k_mlp_train_pair(actor, critic, obs, ret, V2, act, lp, st, float(M), sa2, sc2)
    torch.cuda.synchronize()
    ms = sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in ppo.TRAIN_EVENTS) / a.reps
    tf = 2 * ppo.FLOPS_PER_ROW_CONT * M / (ms * 1e-3) / 1e12
    print(f"pair rows {M}: {ms:.3f} ms (both passes)  {tf:.1f} TFLOP/s", flush=True)
if a.choice:
    dc, Mc = a.choice, a.choice_rows
    ca = Model_PPO(dc, 2, 2).cuda()
    cc = Model_PPO(dc, 1, 0).cuda()
    xo = torch.randn(Mc, dc, device="cuda") * 2
    xr = torch.randn(Mc, device="cuda") * 3 - 5
    xa = (torch.rand(Mc, device="cuda") < 0.4).float()
    xl = torch.log(torch.rand(Mc, device="cuda") * 0.8 + 0.1)
    cnt = torch.stack([(xa == 0).sum(), (xa == 1).sum()]).double()
    flops = 6 * (dc * 32 + 32 * 64 + 64 * 32 + 32 * 2)  # fwd + bwd(dX, dW) multiply-adds x 2
    for exact in (False, True):
        for kind in (0, 2):
            ppo.TRAIN_EVENTS = []
            for r in range(a.reps + 2):
                if r == 2:
                    torch.cuda.synchronize()
                    ppo.TRAIN_EVENTS = []
                _, scc, Vc = ppo.k_mlp_train(0, cc, xo, xr, m_global=float(Mc), exact=exact) if kind == 0 else (0, scc, Vc)
                if kind == 2:
                    ppo.k_mlp_train(2, ca, xo, xr, Vc, None, xl, scc[1:3].clone(), cnt, m_global=float(Mc), exact=exact)
            torch.cuda.synchronize()
            ms = sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in ppo.TRAIN_EVENTS) / a.reps
            print(f"choice dc {dc} kind {kind} {'exact' if exact else 'split'} rows {Mc}: {ms:.4f} ms "
                  f"{flops * Mc / (ms * 1e-3) / 1e12:.1f} TFLOP/s", flush=True)
ppo.TRAIN_EVENTS = None
