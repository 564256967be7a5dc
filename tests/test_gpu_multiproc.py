"""The N > 1 path with the product on the device: two ranks (spawned processes, gloo
process group, both on cuda:0 of a one-GPU box) each step their contiguous block of the
global batch through libtdstep.so with auto-reset, then gather the device-accumulated
episode statistics (td_episode_stats) and the per-board last-episode records
(td_episode_records) to rank 0 with the helpers bench.py uses over RCCL
(gym_TD.shard).  Rank 0 checks them, and every rank's final observation, against one
process stepping the whole batch: sharding changes nothing."""
import copy
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as tmp  # noqa: E402

L, B_RANK, STEPS, BASE = 10, 256, 300, 5000


def _actions(k, lo, hi):
    """Step k's actions of global boards [lo, hi): a stream per step, sliced by board."""
    return np.random.RandomState(10007 + k).randint(0, 6 * L * L + 1, size=2 * B_RANK)[lo:hi].astype(np.int64)


def _run(lo, hi):
    """Boards [lo, hi) of the global batch on cuda:0: (episode stats, records, obs)."""
    from gym_TD import params as P
    from gym_TD.engine import TDEngine
    cfg = copy.deepcopy(P.config)
    cfg.base_LP = 1  # short episodes: many auto-resets in 300 steps
    seeds = np.arange(lo, hi) + BASE
    eng = TDEngine(L, hi - lo, "def", False, 1, device=0, np_seeds=seeds, py_seeds=seeds, autoreset=True, cfg=cfg)
    try:
        eng.reset_all()
        eng.episode_stats(clear=True)
        for k in range(STEPS):
            eng.step(def_act=torch.from_numpy(_actions(k, lo, hi)).cuda())
        torch.cuda.synchronize()
        stats = eng.episode_stats().cpu()
        recs = [t.cpu() for t in eng.episode_records()]
        obs = eng.obs.cpu().clone()
        assert (eng.flags() == 0).all()
        return stats, recs, obs
    finally:
        eng.close()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gym_TD import shard
        lo, hi = shard.shard_range(rank, B_RANK)
        stats, recs, obs = _run(lo, hi)
        per_rank = shard.gather_stats(stats)
        all_recs = shard.gather_episode_records(*recs)
        out = [torch.zeros_like(obs) for _ in range(world)] if rank == 0 else None
        dist.gather(obs, out, dst=0)
        if rank == 0:
            q.put((per_rank.numpy().tolist(), [r.numpy().tolist() for r in all_recs], torch.cat(out).numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_match_one_process():
    world = 2
    ctx = tmp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        per_rank, recs, obs = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    stats, want_recs, want_obs = _run(0, world * B_RANK)
    per_rank = np.asarray(per_rank)
    assert per_rank.shape == (world, 2)
    assert per_rank[:, 0].sum() == float(stats[0]) > B_RANK // 4  # episodes finished and auto-reset on both ranks
    assert per_rank[:, 1].sum() == pytest.approx(float(stats[1]), rel=1e-12, abs=1e-9)  # atomics: order differs
    assert recs == [r.numpy().tolist() for r in want_recs]  # 16 B per board, global board order, bit-exact
    assert np.array_equal(obs, want_obs.numpy())
