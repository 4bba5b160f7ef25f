"""Full-scale parity of the POLICY-DRIVEN rollout (RolloutGPU.collect) against the C rollout
oracle (oracle_rollout_episode over OpenMP), at the bench's env count.

Env_rollout.iterations_rand (Coop-MH-PPO-scalable.py:357-517): the choice head's Categorical
draws at t = 0 (:403-428), then 80 steps of cross/wait actor forward -> torch.min over
pedestrians -> MVN sample (:430-453) -> env.step (:460) -> episodic min (:461).  Both sides get
the same per-env CPython streams, the same random-init Model_PPO weights and the same Philox
draws (Categorical uniforms u, MVN standard normals eps); the policy outputs feed back into the
env, so a one-ulp difference in a device transcendental (tanhf of the continuous head, expf of
the choice softmax) moves positions and can flip a gap-acceptance decision downstream.

Discrete, per env, exactly (north_star: "bit-exact discrete action indices / collision masks"):
the t = 0 choice actions a_d, the closest pedestrian, car existence, bucket membership (derived),
every discrete pedestrian / car field of the final env state (decision, at_crossing, left,
in_cross, accident, time_stop, stop, line, need_to_stop, direction, follow_rule, light,
exist), the episode's per-env event counters (detection's prints: accidents, near misses, ...) and
the final MT19937 state + cursor (every data-dependent draw of the episode).  An env
whose rewards move by more than 1e-3 at some step is also counted (an accident or decision
flip changes a reward by O(1)).  Continuous outputs of the undiverged envs: actions, log-probs,
features, rewards within the 256-env test's tolerances; bit-different fractions reported.
Records: gpurun_out/parity_rollout_fullscale_<variant>.json (profiles/r03_parity_rollout_fullscale/).
"""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DISCRETE_PED = [4, 5, 6, 7, 8, 9, 10, 11, 17, 18, 19]
DISCRETE_CAR = [3, 7]  # light, exist


def _report(name, rec):
    out = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(out):
        with open(os.path.join(out, f"parity_rollout_fullscale_{name}.json"), "w") as f:
            json.dump(rec, f, indent=1)
    print(name, json.dumps(rec))


def _bitdiff(a, b):
    return int((a != b).sum().item())


# cfg5_shard7: config 5's last rank (global env ids 458 752 .. 524 287, env_id_offset 7 x 65 536):
# env streams and Philox policy noise keyed by global id (tests/test_env_fullscale_gpu.py)
@pytest.mark.parametrize("case", [("4cars", 4, 1, 2, 0), ("scalable", 8, 1, 4, 0), ("scalable", 8, 1, 4, 7 * 65536)],
                         ids=["cfg3_4cars", "cfg4_scalable", "cfg5_shard7_scalable"])
def test_policy_rollout_fullscale_parity(case):
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo.rollout import RolloutGPU
    from oracle import OracleBatch, set_threads
    set_threads(min(16, os.cpu_count() or 1))
    v, nc, npd, nl, off = case
    N, T, seed = int(os.environ.get("MHPPO_FULLSCALE_ENVS", "65536")), 80, 41000
    venv = VecCrosswalk(v, N, nc, npd, nl, seed_base=seed, env_id_offset=off)
    ro = RolloutGPU(venv)
    torch.manual_seed(5)
    ac = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    aw = Model_PPO(13, 1, 1, mean=-1.0, std=3.0).cuda()
    ad = Model_PPO(ro.dc, 2, 2).cuda()
    b = ro.collect(ac, aw, ad, seed=3, iteration=0)
    torch.cuda.synchronize()
    S, P = ro.S, ro.P
    orc = OracleBatch(v, N, nc, npd, nl, seed_base=seed + off)  # oracle env e = global id off + e
    o = orc.rollout(ac.packed().cpu().numpy(), aw.packed().cpu().numpy(), ad.packed().cpu().numpy(),
                    u=ro.u.cpu().numpy(), eps=ro.eps.cpu().numpy(), T=T)
    dev = venv.device
    g = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    # ---- discrete, per env
    bad_ad = (b.a_d != g(o["a_d"])).reshape(N, -1).any(1)
    bad_cl = (b.closest != g(o["closest"])).any(1)
    bad_ex = (b.exist != g(o["exist"])).any(1)
    act_d_g = 2 * b.a_d.reshape(N, S * P)[:, :S] - 1
    act_d_o = 2 * g(o["a_d"]).reshape(N, S * P)[:, :S] - 1
    bucket_g = torch.where(b.exist.bool(), (act_d_g > 0).to(torch.int8), torch.full_like(act_d_g, -1, dtype=torch.int8))
    bucket_o = torch.where(g(o["exist"]).bool(), (act_d_o > 0).to(torch.int8),
                           torch.full_like(act_d_o, -1, dtype=torch.int8))
    bad_bk = (bucket_g != bucket_o).any(1)
    mt_g, mti_g = venv.get_rng()
    mt_o, mti_o = orc.rng_state()
    bad_mt = (mt_g.view(torch.int32) != g(mt_o.view(np.int32))).any(1) | (mti_g != g(mti_o))
    k = orc.dump_dim
    st = venv.get_state()[:, :k]
    dm = g(orc.dump())
    ped_g = st[:, :20 * npd].reshape(N, npd, 20)[:, :, DISCRETE_PED].reshape(N, -1)
    ped_o = dm[:, :20 * npd].reshape(N, npd, 20)[:, :, DISCRETE_PED].reshape(N, -1)
    car_g = st[:, 20 * npd:].reshape(N, -1, 8)[:, :, DISCRETE_CAR].reshape(N, -1)
    car_o = dm[:, 20 * npd:].reshape(N, -1, 8)[:, :, DISCRETE_CAR].reshape(N, -1)
    bad_st = (ped_g != ped_o).any(1) | (car_g != car_o).any(1)
    ev_g = venv.events()  # the episode's detection prints (accident, near miss, ...) per env
    bad_ev = (ev_g != g(orc.events().astype(np.int32))).any(1)
    rew_g = b.rew  # [N, S, T] f64 view
    rew_o = g(o["rew"])
    # an accident / decision flip moves a reward by O(1); only present car slots have records (the
    # scalable env's compact record layout stores none for absent slots, include/mhppo.h rec_of)
    present = b.exist.bool()
    rew_jump = ((rew_g - rew_o).abs() > 1e-3) & present.unsqueeze(-1)
    bad_rw = rew_jump.reshape(N, -1).any(1)
    div = bad_ad | bad_cl | bad_ex | bad_bk | bad_mt | bad_st | bad_rw | bad_ev
    jt = rew_jump.any(1)  # [N, T]
    first_t = torch.where(jt.any(1), jt.float().argmax(1), torch.full((N,), -1, device=dev))
    ok = ~div
    # ---- continuous, undiverged envs
    cont = {}
    for name, x, y, tol in (("act", b.act, g(o["act"]), 1e-5), ("logp", b.logp, g(o["logp"]), 1e-5),
                            ("logp_d", b.logp_d, g(o["logp_d"]), 1e-5), ("feat_d", b.feat_d, g(o["feat_d"]), 1e-5),
                            ("obs_c", b.obs_c, g(o["obs_c"]), 1e-4), ("rew", b.rew, g(o["rew"]), 1e-5),
                            ("ep_min", b.ep_min, g(o["ep_min"]), 1e-5)):
        if name in ("act", "logp", "obs_c", "rew"):  # per-(env, slot, t) records: present slots only
            xs, ys = x[ok][present[ok]].double(), y[ok][present[ok]].double()
        else:
            xs, ys = x[ok].double(), y[ok].double()
        err = ((xs - ys).abs() / ys.abs().clamp_min(1.0)).max().item() if xs.numel() else 0.0
        cont[name] = dict(bit_different=_bitdiff(xs, ys), total=int(xs.numel()), max_rel_err=err, tol=tol)
    rec = dict(config=f"{v} {nc}/{npd}/{nl}", envs=N, steps=T, policy="random-init Model_PPO (torch.manual_seed(5))",
               noise="Philox seed 3 iteration 0 (u, eps shared with the oracle)",
               diverged_envs=int(div.sum().item()),
               by_check=dict(a_d=int(bad_ad.sum()), closest=int(bad_cl.sum()), exist=int(bad_ex.sum()),
                             bucket=int(bad_bk.sum()), mt_state=int(bad_mt.sum()),
                             final_discrete_state=int(bad_st.sum()), reward_jump=int(bad_rw.sum()),
                             event_counts=int(bad_ev.sum())),
               event_counts_gpu=dict(zip(("accident", "possible_accident", "small_mistake", "not_waiting",
                                          "bad_green"), ev_g.sum(0).tolist())),
               diverged_env_ids=torch.nonzero(div).flatten()[:20].tolist(),
               first_reward_jump_steps=first_t[div][:20].tolist(), continuous_undiverged=cont)
    rec["env_id_offset"] = off
    _report(v + (f"_offset{off}" if off else ""), rec)
    assert rec["diverged_envs"] == 0, rec
    for name, c in cont.items():
        assert c["max_rel_err"] <= c["tol"], (name, c)
