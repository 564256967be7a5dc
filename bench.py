#!/usr/bin/env python
"""Benchmark: env-steps/s of the batched gym-TD step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Workload (BASELINE.json configs[1]/[3] shape, per GPU): TD-def-small (10x10),
``--boards`` boards per GPU (default 65,536 = the metric's batch), built-in lv1
opponent, uniform random defender actions over [0, 601) drawn on the device
before the timed region, auto-reset on.  Boards are seeded base + global index
(trajectories do not depend on the GPU count) and burned in ``--burnin`` steps
(half an episode) untimed, so the timed steps see mid-episode tower counts.
Scaling is weak: every rank owns its own boards; the only collective is the
timing all-reduce and the episode-stat gather after the timed region.

One JSON line on rank 0: metric/value/unit, ``roofline`` for the step kernel
(HIP events on the launch stream, algorithmic bytes per launch) and
``cpu_baseline`` (the oracle port timed on this host's cores, rank 0, N=1).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "gym-td_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def algorithmic_bytes(L, mode="def", multi=False):
    """obs f32 (45 L L) + action int64 + reward f64 + done u8 per env-step."""
    obs = 45 * L * L * 4
    act = (6 * L * L * 8 if multi else 8) if mode != "atk" else 0
    act += 3 * 8 * 8 if mode != "def" else 0
    return obs + act + 8 + 1


# --------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    L, seconds, seed = args
    from oracle import td_oracle as O
    import warnings
    warnings.simplefilter("ignore")
    rng = np.random.RandomState(seed)
    s = seed
    while True:
        try:
            env = O.Env(L, O.MODE_DEF, 1, s, s, road_attempts=20000)
            break
        except O.RoadGenError:
            s += 100003
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(50):
            _, _, d, _ = env.step(int(rng.randint(0, 6 * L * L + 1)))
            n += 1
            if d:
                while True:  # the reference raises here for a few L=10 draws; draw again
                    try:
                        env.reset()
                        break
                    except O.RoadGenError:
                        pass
    return n, time.perf_counter() - t0


def cpu_baseline(L, seconds, procs):
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(L, seconds, 90001 + i) for i in range(procs)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "sample": "oracle/td_oracle.py (Python restatement of the reference step, parity-pinned) TD-def-small "
                      "random defender actions, %d processes x %.0f s, %d env-steps" % (procs, seconds, steps)}


def host_cores():
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:  # noqa: BLE001
        n = os.cpu_count() or 1
    return max(1, min(16, n))


# --------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--boards", type=int, default=65536, help="boards per GPU")
    ap.add_argument("--map-size", type=int, default=10)
    ap.add_argument("--burnin", type=int, default=600)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--autoreset", type=int, default=1, help="diagnostic: 0 keeps finished boards stepping (not the metric)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from gym_TD.engine import TDEngine
    from gym_TD import shard

    B, L, K, W = args.boards, args.map_size, args.steps, args.warmup
    seeds = shard.shard_seeds(args.seed, rank, B)
    eng = TDEngine(L, B, "def", False, 1, device=dev, np_seeds=seeds, py_seeds=seeds, autoreset=bool(args.autoreset), info=True)
    obs, _ = eng.reset_all()  # failing road draws (the reference raises/hangs) are redrawn
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    n_act = 6 * L * L + 1
    burn = torch.randint(0, n_act, (max(args.burnin, 1), B), device=dev, generator=g, dtype=torch.int64)
    for k in range(args.burnin):
        eng.step(def_act=burn[k])
    warm = torch.randint(0, n_act, (max(W, 1), B), device=dev, generator=g, dtype=torch.int64)
    for k in range(W):
        eng.step(def_act=warm[k])
    acts = torch.randint(0, n_act, (K, B), device=dev, generator=g, dtype=torch.int64)
    del burn, warm
    stream = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    eng.episode_stats(clear=True)  # the device accumulates finished episodes of the timed steps

    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        ev[k][0].record(stream)
        eng.step(def_act=acts[k])
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    kern_ms = [s.elapsed_time(e) for s, e in ev]
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    # after timing: MAX of the clocks over ranks, and the episode statistics of the
    # timed steps gathered to rank 0 (the only exchange; RCCL on GPUs)
    flags = eng.flags()
    t = shard.max_over_ranks(torch.tensor([elapsed, avg_kernel_s], dtype=torch.float64, device=dev))
    per_rank = shard.gather_stats(eng.episode_stats(clear=True))
    elapsed, avg_kernel_s = float(t[0]), float(t[1])

    if rank == 0:
        total_steps = world * B * K
        value = total_steps / elapsed
        bpe = algorithmic_bytes(L)
        achieved = B * bpe / avg_kernel_s / 1e9
        traffic = None
        tp = os.path.join(HERE, "profiles", "pmc_traffic.json")
        if os.path.exists(tp):
            try:
                tj = json.load(open(tp))
                key = "L%d_B%d" % (L, B)
                if key in tj:
                    traffic = tj[key]["hbm_bytes_per_launch"]
            except Exception:  # noqa: BLE001
                traffic = None
        out = {
            "metric": "env-steps/sec (whole node), 10x10 board, batch=65k, at 1/2/4/8 MI355X",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64",
            "data": "synthetic: uniform random defender actions, built-in lv1 opponent, seeded boards",
            "config": {"workload": "TD-def-small-v0 (10x10), %d boards per GPU, auto-reset, burn-in %d steps"
                                   % (B, args.burnin), "global_batch": world * B, "boards_per_gpu": B,
                       "map_size": L, "parallelism": "boards sharded per GPU (dp%d)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "td_step_kernel<10>", "avg_kernel_us": avg_kernel_s * 1e6,
                         "algorithmic_bytes_per_launch": B * bpe},
            "board_flags_nonzero": int((flags != 0).sum()),
            "episodes": {"finished": int(per_rank[:, 0].sum()),
                         "mean_return": float(per_rank[:, 1].sum() / max(float(per_rank[:, 0].sum()), 1.0)),
                         "per_rank": [int(v) for v in per_rank[:, 0].tolist()]},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(L, args.cpu_seconds, host_cores())
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
