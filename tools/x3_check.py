"""Split-precision (bf16x3) training kernel vs the exact f32-MFMA kernel vs float64 autograd,
and launch timing (GPU box): python tools/x3_check.py [M]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from mhppo import ppo  # noqa: E402
from mhppo.models import Model_PPO  # noqa: E402
from test_update_scale_gpu import _f64, _flat_grad  # noqa: E402


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    torch.manual_seed(0)
    actor = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    critic = Model_PPO(13, 1, 0).cuda()
    obs = (torch.randn(M, 13) * 3).cuda()
    ret = (torch.randn(M) * 8 - 20).cuda()
    act = (torch.randn(M) - 1).cuda()
    lp = (torch.randn(M) * 0.3 - 0.9).cuda()
    m = float(M)
    res = {}
    for exact in (True, False):
        gc, sc, V = ppo.k_mlp_train(ppo.KIND_CRITIC, critic, obs, ret, m_global=m, exact=exact)
        gc, sc, V = gc.clone(), sc.clone(), V.clone()
        st = sc[1:3].clone()
        ga, sa, _ = ppo.k_mlp_train(ppo.KIND_CONT, actor, obs, ret, V, act, lp, st, m_global=m, exact=exact)
        res[exact] = (gc, sc, V, ga.clone(), sa.clone())
    c64 = _f64(critic)
    V64 = torch.squeeze(c64(obs.double()), -1)
    g64 = _flat_grad(c64, ((V64 - ret.double()) ** 2).sum() / m)
    for exact in (True, False):
        gc, sc, V, ga, sa = res[exact]
        print(f"exact={exact}: V maxrel {float(((V.double() - V64).abs() / V64.abs().clamp(min=1e-3)).max()):.3e} "
              f"critic grad max|d|/max|g| {float((gc.double() - g64).abs().max() / g64.abs().max()):.3e} "
              f"mse rel {abs(float(sc[0]) / float(((V64 - ret.double()) ** 2).sum()) - 1):.3e}")
    gce, _, Ve, gae, sae = res[True]
    gcx, _, Vx, gax, sax = res[False]
    print(f"split vs exact: V maxabs {float((Vx - Ve).abs().max()):.3e}  critic grad {float((gcx - gce).abs().max() / gce.abs().max()):.3e}"
          f"  actor grad {float((gax - gae).abs().max() / gae.abs().max()):.3e}  actor loss rel "
          f"{abs(float(sax[0]) / float(sae[0]) - 1):.3e}")
    for exact in (True, False):
        for kind in (ppo.KIND_CRITIC, ppo.KIND_CONT):
            net = critic if kind == ppo.KIND_CRITIC else actor
            args = (kind, net, obs, ret) if kind == ppo.KIND_CRITIC else (kind, net, obs, ret, V, act, lp, st)
            for _ in range(3):
                ppo.k_mlp_train(*args, m_global=m, exact=exact)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n = 10
            for _ in range(n):
                ppo.k_mlp_train(*args, m_global=m, exact=exact)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / n
            print(f"exact={exact} kind={kind}: {ms:.3f} ms/launch (incl. grad reduction) = "
                  f"{ppo.FLOPS_PER_ROW_CONT * M / ms / 1e9:.1f} TFLOP/s algorithmic", flush=True)


if __name__ == "__main__":
    main()
