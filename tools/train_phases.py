"""Per-phase share of the fused train kernel (k_mlp_train<KIND,7,true>) from a timing build:
  tools/ab_build.sh timing -DMHPPO_TIMING
  MHPPO_LIB=build_ab/timing/libmhppo.so python tools/train_phases.py
Stamps serialise what the real kernel overlaps: read the SHARES, not the length."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo import _lib, ppo  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

PH = {1: "tile inputs wait", 2: "forward L1-L4", 3: "loss gradient", 4: "L4 bwd + dW3 + dH2",
      5: "dW2 + dH1", 6: "dW1"}
M = 10485760
torch.manual_seed(0)
actor = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
critic = Model_PPO(13, 1, 0).cuda()
obs = torch.randn(M, 13, device="cuda") * 3
ret = torch.randn(M, device="cuda") * 8 - 20
act = torch.randn(M, device="cuda") - 1
lp = torch.randn(M, device="cuda") * 0.3 - 0.9
fn = _lib.lib().mhppo_debug_timing_train
fn.restype, fn.argtypes = ctypes.c_int32, [ctypes.c_void_p]
buf = (ctypes.c_uint64 * 16)()
gc, sc, V = ppo.k_mlp_train(0, critic, obs, ret, m_global=float(M))
torch.cuda.synchronize()
for kind in (0, 1):
    fn(buf)
    if kind == 0:
        ppo.k_mlp_train(0, critic, obs, ret, m_global=float(M))
    else:
        ppo.k_mlp_train(1, actor, obs, ret, V, act, lp, sc[1:3].clone(), m_global=float(M))
    torch.cuda.synchronize()
    fn(buf)
    tot = sum(buf[k] for k in PH)
    print(f"kind {kind}: {buf[15]} waves")
    for k, n in PH.items():
        print(f"  {n:22s} {100.0 * buf[k] / tot:5.1f} %  ({buf[k] / max(buf[15], 1) / (M / 32 / buf[15]):8.0f} cycles/tile)")
