#!/usr/bin/env python3
"""MH-PPO hot-path benchmark on MI355X (driver contract: see task README).

One bench "step" = one full PPO iteration on this rank's shard:
    reset N envs -> 80 rollout steps (choice head at t=0; per step: policy
    kernel + fused sample/env-step kernel) -> returns scan -> bucketing ->
    10 epochs (cross, wait) + 10 epochs (choice) of full-batch PPO updates.
Workload (BASELINE.json configs[2], the metric's "65536 envs x 4 agents"):
    Env_hybrid_multi_coop_4cars, 4 AVs (+4 IDM followers), 1 pedestrian,
    2 lanes, 65536 envs per GPU (weak scaling over ranks), T = 80.
value = (all ranks' envs) * 80 env-steps / max-over-ranks iteration time.

Extra JSON fields:
  roofline     — the dominant kernel, the fused continuous-head train kernel
                 (mhppo_mlp_train_cont, ~60 % of GPU time): algorithmic FLOPs per
                 row x rows / launch duration, from HIP events on
                 its stream inside the timed region, summed over all launches;
                 f32 MFMA peak 157.3 TFLOP/s (exact-f32 matrix rate on gfx950).
  roofline_env — the fused sample+env-step kernel (mhppo_rollout_sample_env):
                 algorithmic bytes per env-step x N / its mean duration; 8 TB/s.
  cpu_baseline — the C oracle (same env + rollout, glibc) + PyTorch-CPU update
                 on a bounded sample of the same workload, rank 0, N=1 only.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec at 65536 envs × 4 agents, 1/2/4/8 MI355X + %HBM roofline"
HBM_PEAK_GBS = 8000.0
F32_MFMA_PEAK_TFLOPS = 157.3


def env_step_bytes(S, nC, P, obs_dim, T=80):
    """Algorithmic HBM bytes one env moves in one fused sample+env-step launch.
    With one pedestrian the policy kernel writes the step's feature record in place
    (include/mhppo.h), so this kernel neither reads feat_c nor writes obs_c."""
    car = nC * 11 * 8 + nC * 6 * 8 + S * 3 * 8      # read 11 fields/car, write 6 dynamic (+3 detection fields per AV)
    ped = P * (17 * 8 + 4) + P * (10 * 8 + 4)      # read 17 f64 + flags, write 10 dynamic f64 + flags
    env = 8 + 8 + 4 + 4 + 4 + 4 + 8               # cross, time r/w, mti r/w, block bits, ped_traffic, RNG words
    feat = 0 if P == 1 else 2 * S * 13 * 4          # selected feature row: read feat_c, write obs_c
    io_in = S * P * 4 + S * 4 + S * P * 4 + S * 4 + S * 8   # out_c, eps, a_d, closest, ep_min
    io_out = S * 4 + S * 4 + S * 8 + S * 8 + obs_dim * 4     # act, logp, rew, ep_min, obs
    return car + ped + env + feat + io_in + io_out


def pmc_traffic(*patterns):
    """Mean HBM bytes per launch over the kernels matching `patterns`, from the committed
    rocprofv3 PMC summary (profiles/pmc_traffic.json, made by tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench; reads = 2 x FETCH_SIZE on
    gfx950).  None when absent."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        ks = json.load(open(path))["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    vals = [v["hbm_bytes_per_launch"] for k, v in ks.items()
            if any(p in k for p in patterns) and v.get("hbm_bytes_per_launch")]
    return sum(vals) / len(vals) if vals else None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--variant", default="4cars")
    ap.add_argument("--nb-car", type=int, default=4)
    ap.add_argument("--nb-ped", type=int, default=1)
    ap.add_argument("--nb-lines", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-envs", type=int, default=256)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse several ranks on one GPU")
    return ap.parse_args()


def cpu_baseline(a, seconds_cap=30.0):
    """Oracle rollout (C, glibc) + PyTorch-CPU PPO update on a bounded env sample."""
    try:
        from oracle import cpu_iteration
    except Exception as ex:  # pragma: no cover - reported, never silently substituted
        return {"value": None, "unit": "env-steps/s", "cores": 0, "kind": "port", "sample": f"unavailable: {ex}"}
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    n = a.cpu_sample_envs
    t0 = time.perf_counter()
    iters = 0
    while True:
        cpu_iteration(a.variant, n, a.nb_car, a.nb_ped, a.nb_lines, seed=iters)
        iters += 1
        if time.perf_counter() - t0 > min(seconds_cap, 10.0) or iters >= 3:
            break
    dt = (time.perf_counter() - t0) / iters
    return {"value": n * 80 / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs x 80 steps x {iters} iterations (oracle env+rollout in C, 1 thread; "
                      f"update PyTorch-CPU {threads} threads), {dt:.2f} s/iteration"}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank; with fewer GPUs than ranks (a rehearsal) ranks share them round-robin
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.dist_backend)
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO
    from mhppo import ppo

    N, T = a.envs, 80
    venv = VecCrosswalk(a.variant, N, a.nb_car, a.nb_ped, a.nb_lines, seed_base=0, env_id_offset=rank * N,
                        device=f"cuda:{local}")
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0)

    def iteration(events=None):
        algo.rollout.reset()
        with torch.no_grad():
            algo.rollout.batch = algo.rollout.gpu.collect(algo.actor_net_cross, algo.actor_net_wait,
                                                          algo.actor_net_choice, seed=0,
                                                          iteration=algo.rollout.iteration, step_events=events)
        algo.rollout.iteration += 1
        from mhppo.rollout import bucket_segments
        algo.rollout.cross, algo.rollout.wait, algo.rollout.choice = bucket_segments(algo.rollout.batch)
        algo.update()

    for _ in range(a.warmup):
        iteration()
    events = [[[torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)] for _ in range(T)]
              for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ppo.TRAIN_EVENTS = []
    t0 = time.perf_counter()
    for k in range(a.steps):
        iteration(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / a.steps * 1e3
    value = world * N * T / (dt / a.steps)
    kern_ms = sum(ev[0].elapsed_time(ev[1]) for evs in events for ev in evs) / (a.steps * T)
    S = venv.n_slots
    nC = 2 * S if a.variant == "4cars" else S
    per_env = env_step_bytes(S, nC, a.nb_ped, venv.obs_dim)
    achieved = per_env * N / (kern_ms * 1e-3) / 1e9
    tr = [e for e in ppo.TRAIN_EVENTS if e[1] == 13]  # the continuous heads' launches
    ppo.TRAIN_EVENTS = None
    tr_ms = sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in tr)
    tr_rows = sum(m for _, _, m, _, _ in tr)
    tr_flops = ppo.FLOPS_PER_ROW_CONT * tr_rows
    tr_tflops = tr_flops / (tr_ms * 1e-3) / 1e12
    traffic = pmc_traffic("k_mlp_train<0, 7, true>", "k_mlp_train<1, 7, true>")
    traffic_env = pmc_traffic("k_sample_env")
    line = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64 env / f32 nets", "data": "synthetic (random-init Model_PPO heads, CPython-MT19937 env streams, "
                                            "Philox policy noise)",
        "config": {"workload": f"{a.variant} nb_car={a.nb_car} nb_ped={a.nb_ped} nb_lines={a.nb_lines}, "
                               f"{N} envs/GPU x 80 steps, full PPO iteration (rollout + returns + 10+10 epochs)",
                   "envs_per_gpu": N, "agents": S, "T": T, "parallelism": f"dp{world}"},
        "roofline": {"bound": "mfma", "kernel": "k_mlp_train (fused continuous-head fwd/loss/bwd/wgrad, f32 MFMA)",
                     "achieved": tr_tflops, "peak": F32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tr_tflops / F32_MFMA_PEAK_TFLOPS, "traffic": traffic, "traffic_unit": "B/launch",
                     "flops_per_row": ppo.FLOPS_PER_ROW_CONT, "rows_per_launch": tr_rows / max(len(tr), 1),
                     "launches": len(tr), "launch_ms": tr_ms / max(len(tr), 1)},
        "roofline_env": {"bound": "hbm", "kernel": "k_sample_env (fused select/MVN/env.step)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic_env, "traffic_unit": "B/launch",
                         "bytes_per_launch": per_env * N, "bytes_per_env_step": per_env,
                         "kernel_ms": kern_ms},
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(a)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
