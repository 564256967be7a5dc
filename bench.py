#!/usr/bin/env python
"""Benchmark: env-steps/s of the batched gym-TD step on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

``--gpus N`` with N > 1 and no WORLD_SIZE in the environment starts the N ranks itself
(``torch.distributed.run`` as a child process, before anything touches the GPU) and
exits with its status; under a launcher, WORLD_SIZE must equal ``--gpus``.

Workload: TD-def-small (10x10), built-in lv1 opponent, uniform random defender
actions over [0, 601) drawn on the device before the timed region, auto-reset on.
Scaling is STRONG by default, as BASELINE.json's metric and configs[3] state it:
the global batch (default 65,536 boards = "batch=65k") is split over the N ranks,
65,536 / N boards per GPU (8,192 at N = 8), contiguous global board blocks per
rank.  ``--boards-per-gpu B`` instead runs B boards on every rank (weak scaling)
and labels its line as such.  ``--workload`` selects the other SURVEY.md 8(d)
shapes for their own lines (not the metric): ``2p-middle-multi`` (configs[2]:
16,384 x TD-2p 20x20, multi-action defender flags uniform in {0,1,2}, attacker
clusters uniform in {0..4}) and ``def-large`` (configs[4]: 131,072 x TD-def 30x30
over the node).  Boards are seeded base + global index (trajectories do not
depend on the GPU count) and burned in ``--burnin`` steps untimed.  The burn-in
staggers the episodes: at burn-in step k the boards whose global index is k
modulo the episode limit (1,200 steps) are reset explicitly, so after a full
burn-in the boards' episode phases are spread uniformly and the timed steps see
the steady state of a long rollout -- about B / 1,200 auto-resets (layout draws
included) per step and every tower count of an episode -- instead of the
synchronised start of a fresh batch, where every board would reset in the same
step.  There is no collective on the data path: the only ones are the timing
MAX and the episode-stat gather after the timed region (RCCL on GPUs).

One JSON line on rank 0: metric/value/unit (the metric string, ``global_batch``,
``boards_per_gpu`` and ``scaling`` follow what actually ran), ``roofline`` for
the step kernel (its average duration from HIP timing events bound to the own
dispatch of every k-th launch of the timed region on the launch stream -- the
timestamps rocprofv3's kernel trace reports; k from the warm-up's step time,
``event_every`` -- and the algorithmic bytes per launch;
``traffic`` is the PMC-measured HBM bytes per launch of the same kernel build at
the same boards per GPU, with its source, or null) and ``cpu_baseline`` (the C
restatement oracle/td_cpu.c on this host's cores, rank 0, N=1;
``cpu_baseline_python`` times the Python restatement the same way).
"""
import argparse
import json
import math
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


# name -> (map size, mode, multi-action, default GLOBAL batch (split over the ranks), BASELINE config)
WORKLOADS = {
    "def-small": (10, "def", False, 65536, "configs[1]/[3]"),
    "2p-middle-multi": (20, "2p", True, 16384, "configs[2]"),
    "def-large": (30, "def", False, 131072, "configs[4]"),
}
# BASELINE.json's metric, quoted verbatim when the run is exactly its configuration
BASELINE_METRIC = "env-steps/sec (whole node), 10\u00d710 board, batch=65k, at 1/2/4/8 MI355X"
ENV_ID = {"def-small": "TD-def-small-v0", "2p-middle-multi": "TD-2p-middle-v0 (allow_multiple_actions)",
          "def-large": "TD-def-large-v0"}
DATA = {("def", False): "synthetic: uniform random defender actions, built-in lv1 opponent, seeded boards",
        ("2p", True): "synthetic: defender flags uniform in {0,1,2} (6,L,L), attacker clusters uniform in {0..4} (3,8), "
                      "seeded boards"}
N_ACTION_BUFS = 8  # distinct pre-drawn action batches cycled through the timed steps (multi-action shapes)
EVENT_EVERY = 8  # timed steps per sampled kernel duration when the warm-up gives no step time (--warmup 0)

FLAG_BITS = (("enemy_overflow", 1), ("tower_overflow", 2), ("bad_action", 4), ("no_layout", 8), ("bad_move", 16),
             ("claim_timeout", 32))

# The step kernel is sampled inside the timed region itself, on every k-th launch.  A
# launch bound to a timing-event pair (td_kernel_timing) delays the next dispatch by about
# EVENT_COST_US (~3 us at 65,536 and at 8,192 boards with events on every launch,
# scripts/probe_timing.py in r05/s1; 4,096 boards with every 2nd: +1 us per step, r05/s10),
# so k is chosen from the warm-up's wall time per step to keep that cost below
# EVENT_PERTURB of the step, and at most half the timed steps apart (two samples at least).
# Passes sampled outside the timed region measured another window of the rollout: 20-step
# windows of the same run differ by up to 10 % (65,536 boards: 208.5 us per step after
# 1,200 burn-in steps, 228.0 after 1,456, 231.9 after 1,520, r05/s10).
EVENT_COST_US = 3.0
EVENT_PERTURB = 0.01
MIN_SAMPLES = 4  # sampled launches per rank at least (when the timed steps allow it)


def event_every(steps, warm_step_us=None, override=None):
    """Timed launches per sampled kernel duration: the smallest k with EVENT_COST_US / k
    below EVENT_PERTURB of the warm-up's step time, at least 2, but never so large that the
    timed steps hold fewer than MIN_SAMPLES samples (k <= steps // MIN_SAMPLES, at least 1).
    The driver's 20 steps at 65,536 boards (~204 us): every 2nd launch, 10 samples; at the
    N = 8 share (8,192 boards, ~32 us) every 5th, 4 samples per rank.
    Without a warm-up step time: every EVENT_EVERY-th, within the same cap."""
    if override:
        return max(1, int(override))
    cap = max(1, steps // MIN_SAMPLES)
    if not (warm_step_us and warm_step_us > 0):
        return int(min(EVENT_EVERY, cap))
    k = max(2, math.ceil(EVENT_COST_US / (EVENT_PERTURB * warm_step_us)))
    return int(min(k, cap))


def timed_region(run, sync, barrier=None, clock=time.perf_counter):
    """Time run() -- the K timed steps -- on this rank.  Opening: sync, barrier (every rank
    starts together), sync, clock.  Closing: sync, clock -- the rank's own steps end there --
    then the closing barrier and a sync, timed on their own.  The closing barrier is outside
    the timed region: at N = 8 a rank times only ~20 x 32 us, and a
    barrier's latency and release skew would be charged to the metric; the MAX over ranks of
    the returned times is the whole job's.  Returns (elapsed s, closing barrier s)."""
    sync()
    if barrier is not None:
        barrier()
    sync()
    t0 = clock()
    run()
    sync()
    elapsed = clock() - t0
    barrier_s = 0.0
    if barrier is not None:
        tb = clock()
        barrier()
        sync()
        barrier_s = clock() - tb
    return elapsed, barrier_s


def kernel_vs_step(avg_kernel_us, step_us):
    """A step kernel cannot take longer than a step: the sampled mean is held against the
    timed region's wall time per step (ms_per_step), the steps it was sampled in.
    When the mean exceeds it the kernel figure is not trusted and the roofline fraction is
    withheld (None) with the reason."""
    if not (avg_kernel_us == avg_kernel_us) or not (step_us > 0):  # nan: not timed
        return False, None
    return avg_kernel_us > step_us, ("mean sampled kernel %.2f us exceeds the timed region's %.2f us wall time per "
                                     "step" % (avg_kernel_us, step_us)) if avg_kernel_us > step_us else None


def algorithmic_bytes(L, mode="def", multi=False):
    """obs f32 (45 L L) + action int64 + reward f64 + done u8 per env-step."""
    obs = 45 * L * L * 4
    act = (6 * L * L * 8 if multi else 8) if mode != "atk" else 0
    act += 3 * 8 * 8 if mode != "def" else 0
    return obs + act + 8 + 1


def stagger_mask(k, gidx, period):
    """The burn-in's explicit resets before step k: the boards whose global index is k modulo
    the episode limit (``period``, 1,200 steps), for 0 < k < period, so that after a full
    burn-in the episode phases are spread uniformly.  None when no board is reset."""
    if k <= 0 or k >= period:
        return None
    m = (np.asarray(gidx) % period) == k
    return m if m.any() else None


def partition(workload, world, global_batch=None, boards_per_gpu=None):
    """Boards per rank and the scaling mode of a run.

    Strong scaling (default): the global batch -- BASELINE's 65,536 boards for the
    metric -- is split evenly over the ranks.  Weak scaling: ``boards_per_gpu`` on
    every rank.  Returns (boards per rank, global batch, "strong" | "weak")."""
    if boards_per_gpu is not None:
        if boards_per_gpu < 1:
            raise ValueError("--boards-per-gpu must be >= 1")
        return int(boards_per_gpu), int(boards_per_gpu) * world, "weak"
    g = int(global_batch or WORKLOADS[workload][3])
    if g < world or g % world:
        raise ValueError("global batch %d does not split evenly over %d ranks" % (g, world))
    return g // world, g, "strong"


def metric_label(workload, global_batch, scaling):
    """The metric string of what ran: BASELINE.json's own metric only for its config."""
    L = WORKLOADS[workload][0]
    if workload == "def-small" and global_batch == 65536 and scaling == "strong":
        return BASELINE_METRIC
    kind = {"def-small": "TD-def", "def-large": "TD-def", "2p-middle-multi": "TD-2p multi-action"}[workload]
    return "env-steps/sec (whole node), %s %dx%d board, batch=%d (%s scaling)" % (kind, L, L, global_batch, scaling)


def kernel_source_hash():
    """sha256 (16 hex) of the library's sources (td_step.hip, td_capi.hip -- which picks
    the kernel, the store policy and the refill cadence -- and the headers): a PMC
    traffic record of the step kernel is quoted only for the build it was measured on."""
    import hashlib
    h = hashlib.sha256()
    d = os.path.join(HERE, "gym-td_amd", "csrc")
    for f in sorted(os.listdir(d)):
        if f.endswith(".hip") or f.endswith(".h"):
            h.update(open(os.path.join(d, f), "rb").read())
    h.update(open(os.path.join(HERE, "include", "tdstep.h"), "rb").read())
    return h.hexdigest()[:16]


def measured_traffic(workload, boards, kernel, obs_alloc, path=None):
    """(bytes per launch, source) from profiles/pmc_traffic.json when that file holds a
    PMC measurement of this workload at these boards per GPU on this build (kernel source
    hash), of this step kernel, with the observation allocated the same way (contiguous /
    plain: the write stream's placement changes the kernel).  Else (None, None)."""
    tp = path or os.path.join(HERE, "profiles", "pmc_traffic.json")
    try:
        rec = json.load(open(tp)).get("%s_B%d" % (workload, boards))
    except Exception:  # noqa: BLE001
        return None, None
    if not rec or rec.get("kernel_src") != kernel_source_hash():
        return None, None
    if rec.get("kernel") != kernel or rec.get("obs_alloc") != obs_alloc:
        return None, None
    return rec["hbm_bytes_per_launch"], "profiles/pmc_traffic.json[%s_B%d] (%s, rocprofv3 --pmc FETCH_SIZE / " \
        "WRITE_SIZE passes of bench.py at the same boards per GPU, kernel sources %s, %s observation)" % (
            workload, boards, rec.get("round", "?"), rec["kernel_src"], obs_alloc)


# --------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    L, mode, multi, seconds, seed = args
    from oracle import td_oracle as O
    import warnings
    warnings.simplefilter("ignore")
    rng = np.random.RandomState(seed)
    s = seed
    omode = {"def": O.MODE_DEF, "atk": O.MODE_ATK, "2p": O.MODE_2P}[mode]
    while True:
        try:
            env = O.Env(L, omode, 1, s, s, O.Config(), O.Hyper(allow_multiple_actions=multi), road_attempts=20000)
            break
        except O.RoadGenError:
            s += 100003
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(50):
            da = aa = None
            if mode != "atk":
                da = rng.randint(0, 3, size=(6, L, L)) if multi else int(rng.randint(0, 6 * L * L + 1))
            if mode != "def":
                aa = rng.randint(0, 5, size=(3, 8))
            _, _, d, _ = env.step(da, aa)
            n += 1
            if d:
                while True:  # the reference raises here for a few L=10 draws; draw again
                    try:
                        env.reset()
                        break
                    except O.RoadGenError:
                        pass
    return n, time.perf_counter() - t0


def cpu_baseline_python(L, mode, multi, seconds, procs, workload):
    """The Python restatement (oracle/td_oracle.py), one process per core."""
    with mp.get_context("spawn").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(L, mode, multi, seconds, 90001 + i) for i in range(procs)])
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "sample": "oracle/td_oracle.py (Python restatement of the reference step, parity-pinned) %s "
                      "random actions, %d processes x %.0f s, %d env-steps" % (workload, procs, seconds, steps)}


def cpu_baseline(L, mode, multi, seconds, threads, workload):
    """The plain-C restatement (oracle/td_cpu.c, golden-pinned), OpenMP over the host
    cores: 16 envs per thread, random actions, auto-reset, every observation built."""
    from oracle import td_cpu
    n_envs = 16 * threads
    steps, wall = td_cpu.bench(L, mode, multi, n_envs, seconds, threads)
    return {"value": steps / wall, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": "oracle/td_cpu.c (C restatement of the reference step, pinned by the golden vectors) %s, "
                      "%d envs on %d OpenMP threads x %.0f s, random actions, auto-reset, %d env-steps"
                      % (workload, n_envs, threads, seconds, steps)}


def host_cores():
    """Every core this process may run on (its affinity mask; SURVEY 8(d): the CPU
    baseline runs on all host cores and states the count)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:  # noqa: BLE001
        n = os.cpu_count() or 1
    return max(1, n)


def baseline_threads():
    """(threads, affinity cores, quota cores) of the CPU baseline: one thread per core the
    process may run on, bounded by the CPU time the box grants it.  On the MI355X boxes the
    affinity mask lists 256 cores and the cgroup grants 16 cores' worth of time
    (cpu.max 1600000 / 100000, profiles/r04/s1/host.log): 256 OpenMP threads there measured
    3.3 M env-steps/s, 16 threads 8.2 M -- throttled time slices, not a larger host."""
    affinity, quota = host_cores(), cpu_quota()
    threads = affinity if not quota else max(1, min(affinity, int(quota)))
    return threads, affinity, quota


def baseline_note(value, threads, affinity, quota):
    """The core accounting of a CPU-baseline line: what it ran on, what the host has, and
    the whole host's rate at the measured per-core rate (a linear projection, labelled)."""
    per_core = value / threads
    return {"affinity_cores": affinity, "cpu_quota_cores": quota, "value_per_core": per_core,
            "all_affinity_cores_projection": {
                "value": per_core * affinity, "cores": affinity,
                "note": "linear projection of the measured per-core rate to every core of the affinity mask "
                        "(not measured: the cgroup grants %s cores' worth of CPU time)" % (quota,)}}


def cpu_quota():
    """The cgroup CPU bandwidth limit in cores (cgroup v2 cpu.max / v1 cfs quota), or None
    when there is none.  A box may give a process fewer cores' worth of time than its
    affinity mask lists; the baseline line states both."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except Exception:  # noqa: BLE001
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / p
    except Exception:  # noqa: BLE001
        return None


# --------------------------------------------------------------------------- launch
def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """Run this script on n ranks (one process per GPU) with torch.distributed.run as a
    child process; returns its exit status.  Nothing here touches the GPU, so the ranks
    start fresh (no exec from a process that has initialised HIP)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def check_world(gpus, env):
    """The rank count a run has: WORLD_SIZE under a launcher (which must equal --gpus),
    else None when bench.py must start --gpus ranks itself, else 1."""
    w = env.get("WORLD_SIZE")
    if w is not None:
        if int(w) != gpus:
            raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (gpus, w))
        return int(w)
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return None if gpus > 1 else 1


# --------------------------------------------------------------------------- ranks
def init_dist(gpu, backend="nccl"):
    """The rank's process group (RANK / WORLD_SIZE / MASTER_* from the launcher's env): RCCL
    (backend "nccl") bound to the rank's GPU, or gloo for CPU-side rehearsals.  Returns the
    device the collectives' tensors live on.  tests/test_gpu_rccl.py runs this very call at
    world size 1 on the GPU box."""
    torch.cuda.set_device(gpu)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        return torch.device("cuda", gpu)
    dist.init_process_group(backend)
    return torch.device("cpu")


def collect(elapsed, avg_kernel_s, warm_step_s, ep_stats, ep_recs, coll, barrier_s=0.0):
    """After the timed region: the MAX of the clocks over ranks (one all_reduce), each
    rank's own clocks (elapsed, kernel mean, warm-up step, closing barrier; f64 [4]), the
    timed steps' episode statistics (per-rank count / return sum, f64 [2]) and per-board
    last-episode records (16 B per board) gathered to rank 0 -- the only exchange of a run,
    over RCCL on GPUs.  Returns ((elapsed, avg_kernel_s, warm_step_s), per_rank [W, 2],
    (ret, length, win), clocks [W, 4]); the last three are None off rank 0."""
    from gym_TD import shard
    mine = torch.tensor([elapsed, avg_kernel_s, warm_step_s, barrier_s], dtype=torch.float64, device=coll)
    clocks = shard.gather_stats(mine.clone())
    t = shard.max_over_ranks(mine[:3].clone())
    per_rank = shard.gather_stats(ep_stats.to(coll))
    recs = shard.gather_episode_records(*[x.to(coll) for x in ep_recs])
    return tuple(float(v) for v in t.cpu()), per_rank, recs, (clocks.cpu().numpy() if clocks is not None else None)


# --------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="def-small", choices=sorted(WORKLOADS))
    ap.add_argument("--global-batch", type=int, default=None,
                    help="boards over all ranks, split evenly (strong scaling; default: the workload's)")
    ap.add_argument("--boards-per-gpu", "--boards", dest="boards_per_gpu", type=int, default=None,
                    help="boards on every rank (weak scaling, its own labelled line)")
    ap.add_argument("--burnin", type=int, default=1200)
    ap.add_argument("--stagger", type=int, default=1, help="stagger episode phases during burn-in (see docstring)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--py-cpu-seconds", type=float, default=5.0, help="Python restatement leg (0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--autoreset", type=int, default=1, help="diagnostic: 0 keeps finished boards stepping (not the metric)")
    ap.add_argument("--timing", default="dispatch", choices=("dispatch", "marker", "none"),
                    help="step-kernel durations: 'dispatch' = events bound to every k-th timed launch "
                         "(td_kernel_timing, the dispatch-packet timestamps rocprofv3 reports; k: --event-every); "
                         "'marker' = torch event pairs around every k-th launch (adds the marker packets' "
                         "overhead); 'none' = no kernel timing (diagnostic A/B of the step rate)")
    ap.add_argument("--step-kernel", default="auto", choices=("auto", "large", "small", "small2"),
                    help="diagnostic: force a step kernel (td_set_step_kernel); default td_create's rule")
    ap.add_argument("--event-every", type=int, default=None,
                    help="timed launches per sampled kernel duration (default: event_every, from the warm-up's "
                         "step time; every launch perturbs the step)")
    ap.add_argument("--refill-interval", type=int, default=None,
                    help="diagnostic: steps between layout-refill launches in the timed region (0 = none)")
    args = ap.parse_args()

    world = check_world(args.gpus, os.environ)
    if world is None:  # --gpus N > 1 without a launcher: start the N ranks here
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TD_BENCH_DIST_BACKEND=gloo + TD_BENCH_SAME_DEVICE=1: rehearsal of the N > 1 control
    # flow with every rank on cuda:0 of a one-GPU box (never the measured configuration)
    backend = os.environ.get("TD_BENCH_DIST_BACKEND", "nccl")
    gpu = 0 if os.environ.get("TD_BENCH_SAME_DEVICE") == "1" else local
    dev = torch.device("cuda", gpu if world > 1 else 0)
    coll = init_dist(gpu, backend) if world > 1 else dev  # where the collectives' tensors live
    torch.cuda.set_device(dev)

    from gym_TD.engine import TDEngine
    from gym_TD import shard
    from gym_TD import params as P

    L, mode, multi, _, base_cfg = WORKLOADS[args.workload]
    B, global_batch, scaling = partition(args.workload, world, args.global_batch, args.boards_per_gpu)
    metric = metric_label(args.workload, global_batch, scaling)
    K, W = args.steps, args.warmup
    seeds = shard.shard_seeds(args.seed, rank, B)
    # info tensors (win, allow-next, fail codes, real actions, episode totals) are written
    # every step -- except in multi-action mode, where the reference itself cannot build
    # its info dict (TDDefense.py:87, TDMulti.py:134-135 raise) and SURVEY 8(d) config 3
    # is the board-level step
    eng = TDEngine(L, B, mode, multi, 1, device=dev, np_seeds=seeds, py_seeds=seeds, autoreset=bool(args.autoreset),
                   info=not multi, step_kernel=args.step_kernel)
    obs, _ = eng.reset_all()  # failing road draws (the reference raises/hangs) are redrawn
    g = torch.Generator(device=dev).manual_seed(1234 + rank)

    def draw(n):
        """n pre-drawn (defender, attacker) action batches on the device."""
        out = []
        for _ in range(n):
            d = a = None
            if mode != "atk":
                d = (torch.randint(0, 3, (B, 6, L, L), device=dev, generator=g, dtype=torch.int64) if multi
                     else torch.randint(0, 6 * L * L + 1, (B,), device=dev, generator=g, dtype=torch.int64))
            if mode != "def":
                a = torch.randint(0, 5, (B, 3, 8), device=dev, generator=g, dtype=torch.int64)
            out.append((d, a))
        return out

    # the discrete shapes draw every step's actions up front; the multi-action shapes
    # (315 MB of int64 flags per step at 20x20) cycle N_ACTION_BUFS batches, each
    # larger than the L2s and the 256 MiB MALL, so every step still reads its actions from HBM
    pool = draw(N_ACTION_BUFS) if multi else None
    period = P.hyper_parameters.max_episode_steps
    gidx = np.arange(B) + rank * B
    for k in range(args.burnin):
        m = stagger_mask(k, gidx, period) if args.stagger else None
        if m is not None:
            eng.reset(m)  # the boards' next staged layouts (tests/test_gpu_steady.py checks this recipe)
        d, a = (pool[k % N_ACTION_BUFS] if multi else draw(1)[0])
        eng.step(def_act=d, atk_act=a)
    acts = pool if multi else draw(K)
    stream = torch.cuda.current_stream(dev)
    if args.refill_interval is not None:
        eng.set_refill_interval(args.refill_interval)
    sampled, ev = set(), {}  # --timing marker: torch event pairs around the sampled steps

    def run_steps(n, first):
        for k in range(n):
            if first + k in sampled:
                ev[first + k][0].record(stream)
            d, a = acts[(first + k) % len(acts)]
            eng.step(def_act=d, atk_act=a)
            if first + k in sampled:
                ev[first + k][1].record(stream)

    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    run_steps(W, 0)  # warm-up: its wall time per step sets the sampling stride
    torch.cuda.synchronize(dev)
    warm_step_s = (time.perf_counter() - t1) / W if W > 0 else float("nan")
    # HIP events bound to every `every`-th step kernel of the timed region (their own
    # dispatch's timestamps): the kernel's duration is sampled live in the steps timed
    every = event_every(K, warm_step_s * 1e6 if W > 0 else None, args.event_every)
    n_samples = (K + every - 1) // every
    if args.timing == "dispatch":
        eng.kernel_timing(n_samples, every)
    elif args.timing == "marker":
        sampled = set(range(0, K, every))
        ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for k in sampled}
    eng.episode_stats(clear=True)  # the device accumulates finished episodes of the timed steps

    elapsed, barrier_s = timed_region(lambda: run_steps(K, 0), lambda: torch.cuda.synchronize(dev),
                                      dist.barrier if world > 1 else None)

    # snapshots of the timed steps' episode statistics and flags (stream-ordered copies)
    flags = eng.flags()
    ep_stats = eng.episode_stats(clear=True)
    ep_recs = eng.episode_records()
    if args.timing == "dispatch":
        kern_ms = (eng.kernel_times().astype(np.float64) / 1e3).tolist()
        eng.kernel_timing(0)
    elif args.timing == "marker":
        kern_ms = [s.elapsed_time(e) for s, e in ev.values()]
    else:
        kern_ms = [float("nan")]
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3 if kern_ms else float("nan")
    # after timing: MAX of the clocks over ranks, and the episode statistics of the
    # timed steps gathered to rank 0 (the only exchange; RCCL on GPUs)
    guard_to = eng.guard_timeouts()
    (elapsed, avg_kernel_s, warm_step_s), per_rank, recs, clocks = collect(
        elapsed, avg_kernel_s, warm_step_s, ep_stats, ep_recs, coll, barrier_s)
    reported_world = dist.get_world_size() if world > 1 else 1  # what the process group (RCCL) reports

    if rank == 0:
        total_steps = world * B * K
        value = total_steps / elapsed
        bpe = algorithmic_bytes(L, mode, multi)
        achieved = B * bpe / avg_kernel_s / 1e9
        exceeds, why = kernel_vs_step(avg_kernel_s * 1e6, elapsed / K * 1e6)
        traffic, traffic_src = measured_traffic(args.workload, B, eng.step_kernel_name, eng.obs_alloc)
        out = {
            "metric": metric,
            "value": value, "unit": "env-steps/s", "n_gpus": world, "world_size_reported": reported_world,
            "steps": K, "warmup": W,
            "ms_per_step": elapsed / K * 1e3, "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "dtype": "f64",
            "data": DATA[mode, multi],
            "config": {"workload": "%s (%dx%d), %d boards over %d GPU(s) = %d per GPU (%s scaling; BASELINE %s), "
                                   "auto-reset, burn-in %d steps%s"
                                   % (ENV_ID[args.workload], L, L, global_batch, world, B, scaling, base_cfg,
                                      args.burnin, ", episode phases staggered" if args.stagger else ""),
                       "global_batch": global_batch, "boards_per_gpu": B, "obs_alloc": eng.obs_alloc,
                       "map_size": L, "parallelism": "boards sharded per GPU (dp%d), no data-path collective" % world},
            "roofline": {"bound": "hbm", "achieved": None if exceeds else achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": None if exceeds else achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": eng.step_kernel_name,
                         "avg_kernel_us": avg_kernel_s * 1e6,
                         "kernel_samples": len(kern_ms) * world,
                         "kernel_samples_per_rank": len(kern_ms),
                         "low_sample_count": len(kern_ms) < MIN_SAMPLES,
                         "kernel_exceeds_step": exceeds,
                         "kernel_timing": {"dispatch": "dispatch-packet timestamps (td_kernel_timing) of every %dth launch "
                                                       "of the timed region (%d samples; warm-up %.2f us per step)" % (
                                                           every, len(kern_ms), warm_step_s * 1e6),
                                           "marker": "torch event pairs around every %dth launch of the timed region" % every,
                                           "none": "not timed"}[args.timing],
                         "algorithmic_bytes_per_launch": B * bpe},
            "per_rank_ms_per_step": [float(c[0]) / K * 1e3 for c in clocks],
            "per_rank_avg_kernel_us": [float(c[1]) * 1e6 for c in clocks],
            "closing_barrier_us": [float(c[3]) * 1e6 for c in clocks],
            "timed_region": "each rank's clock from the opening barrier + synchronize to its own synchronize after "
                            "its K steps (the closing barrier follows, outside it: closing_barrier_us); value uses "
                            "the MAX over ranks",
            "board_flags_nonzero": int((flags != 0).sum()),
            "guard_timeouts_rank0": int(guard_to),
            "board_flags": {name: int(((flags & bit) != 0).sum()) for name, bit in FLAG_BITS if ((flags & bit) != 0).any()},
            "episodes": {"finished": int(per_rank[:, 0].sum()),
                         "mean_return": float(per_rank[:, 1].sum() / max(float(per_rank[:, 0].sum()), 1.0)),
                         "per_rank": [int(v) for v in per_rank[:, 0].tolist()],
                         "boards_with_a_finished_episode": int((recs[2] >= 0).sum()),
                         "last_episode_win_rate": float((recs[2] == 1).sum()) / max(int((recs[2] >= 0).sum()), 1)},
        }
        if exceeds:
            out["roofline"]["frac_withheld"] = why
        if world == 1 and not args.no_cpu_baseline:
            threads, affinity, quota = baseline_threads()
            cb = cpu_baseline(L, mode, multi, args.cpu_seconds, threads, args.workload)
            cb.update(baseline_note(cb["value"], threads, affinity, quota))
            out["cpu_baseline"] = cb
            if args.py_cpu_seconds > 0:
                out["cpu_baseline_python"] = cpu_baseline_python(L, mode, multi, args.py_cpu_seconds, min(threads, 64),
                                                                 args.workload)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
