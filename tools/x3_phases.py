"""Per-phase share of the split-precision train kernel (k_mlp_train_x3) from a timing build:
  tools/ab_build.sh timing -DMHPPO_TIMING
  MHPPO_LIB=build_ab/timing/libmhppo.so python tools/x3_phases.py
Stamps serialise what the real kernel overlaps across phase borders: read the SHARES."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]
from mhppo import _lib, ppo  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402

# the hand-placed passes (SCH, the default): marks after each MFMA block of Pass::fwd_s / bwd_s;
# MHPPO_X3_SCH=0 builds: the phase-by-phase marks
PH_SCH = {1: "tile inputs wait", 2: "layer 1 (+h1 s0 split)", 3: "layer 2 (+payload)", 4: "layer 3 (+payload)",
          5: "loss + d3 + d3 s0 split", 6: "A dH2 (+payload)", 7: "B dW3 (+payload)", 8: "C dH1 (+payload)",
          9: "D dW2 (+payload)"}  # E (dW1) runs in the next tile's layer 1
PH_OLD = {1: "tile inputs wait", 2: "layer 1", 3: "layer 2", 4: "layer 3", 5: "loss + dW4/dB3 sums",
          6: "dW3", 7: "dH2 + masks + dB2 sums", 8: "dW2 + dH1", 9: "dW1"}
PH = PH_OLD if os.environ.get("X3_PHASES_OLD") else PH_SCH
if os.environ.get("X3_PHASES_ALL"):  # masked-mark builds: every slot, by number
    PH = {k: f"slot {k}" for k in range(1, 14)}
M = 10485760
torch.manual_seed(0)
actor = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
critic = Model_PPO(13, 1, 0).cuda()
obs = torch.randn(M, 13, device="cuda") * 3
ret = torch.randn(M, device="cuda") * 8 - 20
act = torch.randn(M, device="cuda") - 1
lp = torch.randn(M, device="cuda") * 0.3 - 0.9
fn = _lib.lib().mhppo_debug_timing_train
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p]
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
    waves = max(buf[15], 1)
    tiles = M / 32 / waves
    tot = sum(buf[k] for k in PH)
    print(f"kind {kind}: {buf[15]} waves, {tot / waves / tiles:.0f} stamped cycles/tile")
    for k, n in PH.items():
        print(f"  {n:24s} {100.0 * buf[k] / tot:5.1f} %  ({buf[k] / waves / tiles:7.0f} cycles/tile)")
