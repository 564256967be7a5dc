"""The N > 1 path on CPU (gloo, world sizes 2 and 4): board sharding and the episode-stats
gather that bench.py runs over RCCL on GPUs.

Each rank steps its own contiguous block of boards (here with the oracle, the
same per-board algorithm the HIP path is checked against), accumulates the
finished episodes with ``gym_TD.shard.episode_stats`` and gathers them to rank 0;
rank 0 checks the totals against one process stepping every board.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as tmp

from gym_TD import shard
from oracle import td_oracle as O

L, BOARDS_PER_RANK, STEPS = 10, 3, 80  # seeds 2000..2005 and 2008..2019: every layout draw of these runs succeeds


def _run_boards(seeds):
    """Oracle TD-def boards with 1-LP bases (short episodes): per-step done / ep_return arrays."""
    cfg = O.Config(base_LP=1)
    envs = [O.Env(L, O.MODE_DEF, 1, int(s), int(s), cfg, O.Hyper(), road_attempts=20000) for s in seeds]
    rngs = [np.random.RandomState(int(s) + 1) for s in seeds]  # board-owned action streams
    ret = np.zeros(len(envs))
    out = []
    for _ in range(STEPS):
        acts = [r.randint(0, 6 * L * L + 1) for r in rngs]
        done = np.zeros(len(envs), bool)
        ep = np.zeros(len(envs))
        ln = np.zeros(len(envs), np.int32)
        win = np.full(len(envs), -1, np.int32)
        for i, (e, a) in enumerate(zip(envs, acts)):
            _, r, d, info = e.step(int(a))
            ret[i] += r
            if d:
                done[i], ep[i], ln[i], win[i] = True, ret[i], e._board.steps, int(info["Win"])
                ret[i] = 0.0
                e.reset()
        out.append((done, ep, ln, win))
    return out


def _last_records(trace):
    """Each board's last finished episode (td_episode_records' payload)."""
    n = len(trace[0][0])
    ret, ln, win = np.zeros(n), np.zeros(n, np.int32), np.full(n, -1, np.int32)
    for done, ep, l, w in trace:
        ret[done], ln[done], win[done] = ep[done], l[done], w[done]
    return torch.from_numpy(ret), torch.from_numpy(ln), torch.from_numpy(win)


def _stats(trace):
    tot = torch.zeros(2, dtype=torch.float64)
    for done, ep, _, _ in trace:
        tot += shard.episode_stats(torch.from_numpy(done), torch.from_numpy(ep))
    return tot


def _worker(rank, world, port, q, base):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        seeds = shard.shard_seeds(base, rank, BOARDS_PER_RANK)
        trace = _run_boards(seeds)
        stats = _stats(trace)
        t = shard.max_over_ranks(torch.tensor([float(rank + 1)], dtype=torch.float64))
        got = shard.gather_stats(stats)
        recs = shard.gather_episode_records(*_last_records(trace))
        if rank == 0:
            q.put((got.numpy().tolist(), float(t[0]), [r.numpy().tolist() for r in recs]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_partition():
    for world in (1, 2, 4, 8):
        blocks = [shard.shard_seeds(5, r, 16) for r in range(world)]
        assert np.array_equal(np.concatenate(blocks), np.arange(5, 5 + 16 * world))
        assert shard.shard_range(world - 1, 16) == (16 * (world - 1), 16 * world)


@pytest.mark.parametrize("world,base", [(2, 2000), (4, 2008)])
def test_gloo_ranks_match_one_process(world, base):
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, base)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        per_rank, tmax, recs = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert tmax == float(world)
    trace = _run_boards(shard.shard_seeds(base, 0, world * BOARDS_PER_RANK))
    one = _stats(trace)
    want = [r.numpy().tolist() for r in _last_records(trace)]
    assert recs == want  # per-board records, 16 B each, in global board order
    per_rank = np.asarray(per_rank)
    assert per_rank.shape == (world, 2)
    assert per_rank[:, 0].sum() == float(one[0]) > 0
    assert per_rank[:, 1].sum() == pytest.approx(float(one[1]), rel=1e-12, abs=1e-9)


def _timing_worker(rank, world, port, q):
    """bench.py's timed region and collect() over gloo: rank r's steps take 10 + 40 r ms."""
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        elapsed, barrier_s = bench.timed_region(lambda: time.sleep(0.010 + 0.040 * rank), lambda: None, dist.barrier)
        stats = torch.tensor([float(rank), 2.0 * rank], dtype=torch.float64)
        recs = (torch.zeros(3, dtype=torch.float64), torch.zeros(3, dtype=torch.int32),
                torch.full((3,), -1, dtype=torch.int32))
        (el, ak, ws), per_rank, _, clocks = bench.collect(elapsed, 1e-5 * (rank + 1), 2e-5, stats, recs,
                                                          torch.device("cpu"), barrier_s)
        if rank == 0:
            q.put((el, ak, clocks.tolist(), per_rank.numpy().tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_timed_region_and_per_rank_clocks():
    """N > 1 timing: each rank's clock ends at its own steps, the fast
    rank's wait for the slow one shows as its closing barrier, and the reported time is
    the MAX over ranks -- the slowest rank's steps, not steps + barrier."""
    world = 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_timing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        el, ak, clocks, per_rank = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    clocks = np.asarray(clocks)
    assert clocks.shape == (world, 4)
    assert 0.010 <= clocks[0, 0] < 0.045  # rank 0: its own 10-ms steps
    assert 0.050 <= clocks[1, 0] < 0.090  # rank 1: 50 ms
    assert clocks[0, 3] >= 0.030  # rank 0 waited for rank 1 in the closing barrier, outside its clock
    assert el == clocks[:, 0].max() and ak == pytest.approx(2e-5)
    assert per_rank == [[0.0, 0.0], [1.0, 2.0]]
