#!/usr/bin/env python3
"""MH-PPO hot-path benchmark on MI355X (driver contract: see task README).

One bench "step" = one full PPO iteration on this rank's shard: one call of the product's
Algo_PPO.train(1) (Coop-MH-PPO-scalable.py:854-917), reward-curve file writing off:
    rollout.reset() -> reset N envs + 80 rollout steps (choice head at t=0; per step:
    policy kernel + fused sample/env-step kernel, two env halves on two streams; at small N
    one chain replayed from a HIP graph) -> returns scan -> bucketing -> 10 joint epochs of
    the three heads (cross, wait, choice) ->
    immediate rewards, the
    reward-sum all-reduce and its host read (the reward curves) -> rollout.reset().
Default workload (BASELINE.json configs[2], the metric's "65536 envs x 4 agents"):
    Env_hybrid_multi_coop_4cars, 4 AVs (+4 IDM followers), 1 pedestrian, 2 lanes,
    65536 envs per GPU (weak scaling over ranks), T = 80.
    `--config 4`: Env_hybrid_multi_coop_scalable 8/1/4, ragged 1-8 agents (configs[3]).
value = (all ranks' envs) * 80 env-steps / max-over-ranks iteration time.

Multi-GPU: `python bench.py --gpus N` with N > 1 and no WORLD_SIZE in the environment
starts N ranks itself (torch.distributed.run, one process per GPU, RCCL) before this
process touches the GPU, and relays rank 0's JSON line; under an external launcher
(WORLD_SIZE set) it is one rank.  Envs shard by global id: rank r owns env ids
[r*N, (r+1)*N).

Extra JSON fields:
  roofline     — the dominant kernel, the fused continuous-head train kernel (k_mlp_train,
                 ~85 % of GPU time): algorithmic FLOPs per row x rows /
                 launch duration, from HIP events on its stream around each launch of one
                 extra training iteration run right after the timed region with the passes on
                 one stream (the timed region carries no per-launch events; with
                 MHPPO_TRAIN_STREAMS=2 its concurrent launches would blur them).  The kernel runs the bf16x3 split path
                 (six bf16 MFMAs per f32 product, f32-level accuracy), so its
                 ceiling is the bf16 dense MFMA peak / 6 = 419.4 TFLOP/s of f32-equivalent
                 work; the fraction of the f32-MFMA peak (157.3) is reported beside it.
                 With --exact-f32 (Algo_PPO(exact_f32=True): the f32-MFMA kernel) the peak is
                 the f32 one.
  roofline_env — the fused sample+env-step kernel: SURVEY §8(d)'s algorithmic bytes per
                 env-step (cfg3 1515 B, cfg4 1615 B) x N / its mean duration over the timed
                 region's launches, from HIP events attached to each launch's dispatch
                 packet (mhppo_kernel_timing_begin/_end: hipExtLaunchKernelGGL start/stop
                 events, i.e. the kernel's execution as rocprofv3 times it, without the
                 event packets' queue gaps); 8 TB/s.
  cpu_baseline — the C oracle (same env + rollout, glibc, OpenMP over envs on the box's
                 cores) + the PyTorch-CPU update (same thread count) on a bounded sample
                 of the same workload, rank 0, N=1 only; legs timed separately.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mh-ppo_amd")]

import torch  # noqa: E402  (importing torch does not initialise the GPU)
import torch.distributed as dist  # noqa: E402

METRIC = "env-steps/sec at 65536 envs × 4 agents, 1/2/4/8 MI355X + %HBM roofline"
HBM_PEAK_GBS = 8000.0
F32_MFMA_PEAK_TFLOPS = 157.3   # 256 CU x 4 SIMD x 64 FLOP/clk (32x32x2 f32) x 2.4 GHz
X3_MFMA_PEAK_TFLOPS = 2516.6 / 6  # bf16 32x32x16: 1024 FLOP/clk/SIMD; six per split product
CONFIGS = {3: ("4cars", 4, 1, 2), 4: ("scalable", 8, 1, 4), 2: ("coop", 2, 1, 2)}


def env_step_bytes(S, P, A_ctl, obs_dim):
    """algorithmic HBM bytes of one env-step of the step kernel —
    dynamic state read + written in fp64 (car 56 B, ped 88 B, env 12 B), static state
    read once (car 2 B, ped 78 B, env 12 B), actions 2 A_ctl floats in, obs_dim floats
    + rewards/reward_light (8 A_ctl) + done out, 8 B of RNG words.
    cfg3 (S 8, P 1, A 4, obs 60): 1515 B; cfg4 (S 8, P 1, A 8, obs 69): 1615 B."""
    return 2 * (S * 56 + P * 88 + 12) + (S * 2 + P * 78 + 12) + 4 * 2 * A_ctl + 4 * obs_dim + 8 * A_ctl + 1 + 8


CONFIG = 3  # the workload of this run (set in main): PMC summaries are per config


def pmc_traffic(*patterns, required=True):
    """Mean HBM bytes per launch over the kernels matching `patterns`, from the committed
    rocprofv3 PMC summary of this config (profiles/pmc_traffic_cfg<N>.json, made by
    tools/gpu_pmc.sh <tag> <config> -> tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench; reads = 2 x FETCH_SIZE on
    gfx950).  None when absent."""
    path = os.path.join(ROOT, "profiles", f"pmc_traffic_cfg{CONFIG}.json")
    if not os.path.exists(path):
        return None  # no PMC summary committed for this config: reported as null
    ks = json.load(open(path))["kernels"]
    # a pattern is a substring or a tuple of substrings that must all occur in the kernel's name
    match = lambda k, p: all(q in k for q in p) if isinstance(p, tuple) else p in k  # noqa: E731
    vals = [v["hbm_bytes_per_launch"] for k, v in ks.items()
            if any(match(k, p) for p in patterns) and v.get("hbm_bytes_per_launch")]
    if not vals:  # a stale summary (kernel renamed since it was taken) must not pass as "no data"
        if not required:  # a non-default kernel the committed summary never covered (--exact-f32)
            return None
        raise RuntimeError(f"{path}: no PMC entry matches {patterns}; re-take it (tools/gpu_pmc.sh)")
    return sum(vals) / len(vals)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS),
                    help="BASELINE.json config: 3 = 4cars 4/1/2 (the metric), 4 = scalable 8/1/4, 2 = coop 2/1/2")
    ap.add_argument("--envs", type=int, default=None,
                    help="envs per GPU (default: BASELINE.json's for the config: 4096 for config 2, else 65536)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-envs", type=int, default=4096)
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL, one GPU per rank); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--force-collectives", action="store_true",
                    help="one rank: init a one-rank RCCL group and run every data-parallel collective "
                         "anyway (the multi-GPU call sequence on one GPU; identity sums)")
    ap.add_argument("--save-nets", default=None, help="rank 0 saves every net's flat weights here (tests)")
    ap.add_argument("--exact-f32", action="store_true",
                    help="continuous heads on the exact f32-MFMA train kernel (Algo_PPO(exact_f32=True))")
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """Start `--gpus` ranks (one process per GPU) as children and relay their output.
    Runs before this process makes any GPU call; returns the children's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def cpu_baseline(a, variant, nc, npd, nl):
    """Oracle env + rollout (C, glibc, OpenMP over envs) + PyTorch-CPU update on a bounded
    sample of the same workload: one untimed small iteration, then one timed iteration of
    `--cpu-sample-envs` envs (10-30 s of CPU work on the box's share of cores)."""
    try:
        import oracle
    except Exception as ex:  # pragma: no cover - reported, never silently substituted
        return {"value": None, "unit": "env-steps/s", "cores": 0, "kind": "port", "sample": f"unavailable: {ex}"}
    threads = int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)
    oracle.set_threads(threads)
    torch.set_num_threads(threads)
    oracle.cpu_iteration(variant, 64, nc, npd, nl, seed=999)  # warm caches / torch CPU init (untimed)
    n = a.cpu_sample_envs
    tm = {}
    t0 = time.perf_counter()
    oracle.cpu_iteration(variant, n, nc, npd, nl, seed=0, timings=tm)
    dt = time.perf_counter() - t0
    return {"value": n * 80 / dt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} envs x 80 steps, 1 full iteration (C oracle env+rollout, OpenMP {threads} threads: "
                      f"{tm['rollout']:.2f} s = {n * 80 / tm['rollout']:.0f} env-steps/s; PyTorch-CPU update "
                      f"10+10 epochs, {threads} threads: {tm['update']:.2f} s), {dt:.2f} s total",
            "rollout_s": tm["rollout"], "update_s": tm["update"], "threads_rollout": threads,
            "threads_update": threads}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    # one GPU per rank; with fewer GPUs than ranks (a gloo rehearsal) ranks share them round-robin
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(a.dist_backend)
    elif a.force_collectives:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(29700 + os.getpid() % 200))
        dist.init_process_group(a.dist_backend, rank=0, world_size=1,
                                device_id=torch.device("cuda", local) if a.dist_backend == "nccl" else None)
    from mhppo import ppo
    if a.force_collectives:
        ppo.set_force_collectives(True)
    from mhppo.algo import Algo_PPO
    from mhppo.env import VecCrosswalk
    from mhppo.models import Model_PPO

    global CONFIG
    CONFIG = a.config
    variant, nc, npd, nl = CONFIGS[a.config]
    if a.envs is None:
        a.envs = 4096 if a.config == 2 else 65536
    N, T = a.envs, 80
    venv = VecCrosswalk(variant, N, nc, npd, nl, seed_base=0, env_id_offset=rank * N, device=f"cuda:{local}")
    torch.manual_seed(0)
    algo = Algo_PPO(Model_PPO, venv, verbose=False, seed=0, save_curves=False, exact_f32=a.exact_f32)

    def iteration():
        """One product training iteration (mhppo/algo.py Algo_PPO.train)."""
        algo.train(1)

    for _ in range(a.warmup):
        iteration()
    from mhppo import _lib
    L = _lib.lib()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # per-iteration GPU times (events on the current stream at the iteration boundaries: no extra
    # synchronisation inside the timed region), so clock / power drift over the run is visible
    marks = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
    t0 = time.perf_counter()
    marks[0].record()
    for k in range(a.steps):
        iteration()
        marks[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / a.steps * 1e3
    iter_ms = [round(marks[k].elapsed_time(marks[k + 1]), 3) for k in range(a.steps)]
    value = world * N * T / (dt / a.steps)
    # After the timed region (same process, same workload): (0) one more training iteration with the
    # train passes on ONE stream and torch events around each launch -> roofline (the product runs
    # the heads' passes on two streams, where one launch's events would span the other's kernel);
    # (1) the env-step kernel over all N envs
    # with HIP events attached to its 80 launches' dispatch packets (hipExtLaunchKernelGGL: the
    # kernel's own execution, as rocprofv3 reports it) -> roofline_env; (2) the rollout's wall time
    # per step (policy + env step) with the one-chain loop and with the product's two-stream parts
    # (RolloutGPU.parts), from torch events around whole collects.
    streams_product = ppo.TRAIN_STREAMS
    ppo.TRAIN_STREAMS, ppo.TRAIN_EVENTS = 1, []
    iteration()
    torch.cuda.synchronize()
    ppo.TRAIN_STREAMS = streams_product
    gpu = algo.rollout.gpu
    env_ms, env_n = ctypes.c_double(0.0), ctypes.c_int32(0)
    step_us = {}
    modes = [("one_chain", 1)] + ([("parts", gpu.parts)] if gpu.parts > 1 else []) + [("product", None)]
    with torch.no_grad():
        for name, parts in modes:
            algo.rollout.reset()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            timed = name == "one_chain"
            if timed:
                _lib.check(L.mhppo_kernel_timing_begin(T))
            e0.record()
            gpu.collect(algo.actor_net_cross, algo.actor_net_wait, algo.actor_net_choice, seed=7, iteration=0,
                        parts=parts, graph=None if name == "product" else False)
            e1.record()
            torch.cuda.synchronize()
            if timed:
                ms_, n_ = ctypes.c_double(0.0), ctypes.c_int32(0)
                _lib.check(L.mhppo_kernel_timing_end(ctypes.byref(ms_), ctypes.byref(n_)))
                if n_.value != T:
                    raise RuntimeError(f"timed {n_.value} step launches, expected {T}")
                env_ms, env_n = ms_, n_
            step_us[name] = e0.elapsed_time(e1) * 1e3 / T
    kern_ms = env_ms.value / env_n.value
    S = venv.n_slots
    S_all = 2 * S if variant == "4cars" else S  # car slots incl. the 4cars IDM followers
    per_env = env_step_bytes(S_all, npd, S, venv.obs_dim)
    achieved = per_env * N / (kern_ms * 1e-3) / 1e9
    tr = [e for e in ppo.TRAIN_EVENTS if e[1] == 13]  # the continuous heads' launches
    ppo.TRAIN_EVENTS = None
    tr_ms = sum(e0.elapsed_time(e1) for _, _, _, e0, e1 in tr)
    # a fused pair launch (kind 3: actor pass e + critic pass e + 1) runs two passes over its rows
    tr_rows = sum(m * (2 if k == 3 else 1) for k, _, m, _, _ in tr)
    tr_flops = ppo.FLOPS_PER_ROW_CONT * tr_rows
    tr_tflops = tr_flops / (tr_ms * 1e-3) / 1e12
    split = not algo.exact_f32
    peak = X3_MFMA_PEAK_TFLOPS if split else F32_MFMA_PEAK_TFLOPS
    traffic = (pmc_traffic(("k_mlp_train_x3<0", "Geo<16, 1, 13"), ("k_mlp_train_x3<1", "Geo<16, 1, 13")) if split else
               pmc_traffic("k_mlp_train<0, 7, true>", "k_mlp_train<1, 7, true>", required=False))
    traffic_env = pmc_traffic("k_sample_env")
    agents = "ragged 1-8 existing of 8 slots" if variant == "scalable" else S
    line = {
        "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64 env / f32 nets", "data": "synthetic (random-init Model_PPO heads, CPython-MT19937 env streams, "
                                            "Philox policy noise)",
        "config": {"workload": f"config {a.config}: {variant} nb_car={nc} nb_ped={npd} nb_lines={nl}, {N} envs/GPU x "
                               f"80 steps, full PPO iteration (rollout + returns + 10+10 epochs)",
                   "envs_per_gpu": N, "agents": agents, "T": T, "parallelism": f"dp{world}"},
        "dist": {"world_size": world, "backend": (a.dist_backend if dist.is_initialized() else None),
                 "env_ranges": [[r * N, (r + 1) * N] for r in range(world)],
                 "collectives": "forced (one rank)" if a.force_collectives and world == 1 else
                 ("per epoch: advantage sums + gradient bucket" if world > 1 else "none (one rank)")},
        "roofline": {"bound": "mfma",
                     "kernel": ("k_mlp_train_x3 (fused continuous-head fwd/loss/bwd/wgrad, bf16x3-split MFMA, "
                                "f32-equivalent FLOPs)" if split else
                                "k_mlp_train (fused continuous-head fwd/loss/bwd/wgrad, f32 MFMA)"),
                     "achieved": tr_tflops, "peak": peak, "unit": "TFLOP/s",
                     "frac": tr_tflops / peak, "frac_of_f32_mfma_peak": tr_tflops / F32_MFMA_PEAK_TFLOPS,
                     "traffic": traffic, "traffic_unit": "B/launch",
                     "flops_per_row": ppo.FLOPS_PER_ROW_CONT, "rows_per_launch": tr_rows / max(len(tr), 1),
                     "launches": len(tr), "passes": sum(2 if k == 3 else 1 for k, _, _, _, _ in tr),
                     "launch_ms": tr_ms / max(len(tr), 1),
                     "measured_on": "one extra training iteration after the timed region, its passes on one "
                                    f"stream (the product: heads on {streams_product} streams)"},
        "roofline_env": {"bound": "hbm", "kernel": "k_sample_env (fused select/MVN/env.step)", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic_env, "traffic_unit": "B/launch",
                         "bytes_per_launch": per_env * N, "bytes_per_env_step": per_env,
                         "kernel_ms": kern_ms, "step_kernel_env_steps_per_s": N / (kern_ms * 1e-3),
                         "measured_on": "one extra 80-step rollout after the timed region, all N envs per launch"},
        "rollout_step_us": {**step_us, "parts_n": gpu.parts,
                            "product_path": ("parts" if gpu.parts > 1 else "one_chain") +
                            (" (HIP graph)" if gpu.use_graph and (gpu.parts == 1 or gpu.use_graph == 2) else ""),
                            "note": "wall time per rollout step, torch events around a whole 80-step collect: "
                                    "one_chain = policy + env-step launches, parts = those on two streams "
                                    "(env halves), product = the product's collect (its step loop replays a "
                                    "captured HIP graph at small N)"},
        "iter_ms": iter_ms,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(a, variant, nc, npd, nl)
    if rank == 0 and a.save_nets:
        import numpy as np
        np.save(a.save_nets, np.concatenate([net.flat().cpu().numpy() for net in algo.nets()]))
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
