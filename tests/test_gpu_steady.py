"""Every board of the state bench.py times.

bench.py times the metric's 65,536 TD-def 10x10 boards (and the 8,192-board N = 8 share,
configs[1]'s 4,096, configs[2]'s 16,384 TD-2p 20x20 multi-action and configs[4]'s 16,384
30x30 per GPU) after its burn-in recipe: explicit resets staggered over the first 1,200 steps
(bench.stagger_mask: board i is reset before step i mod 1,200), 1,200 steps with
auto-reset, uniform random defender actions.  In that steady state every episode phase is
present, about B / 1,200 boards auto-reset per step and enemies are upgraded past progress
0.75.  This test runs that recipe on the device (through libtdstep.so, the kernel
td_create picks) and on the batched C restatement (oracle/td_cpu.c tdc_batch_*, OpenMP)
side by side, then compares EVERY board's reward bits, done flag and observation bytes at
every step of a 16-step window, and the board flags at the end.

Reference: TDBoard.step / get_states (gym_TD/envs/TDBoard.py:295-368, :85-144),
TDGymBasic.reset at every episode end (TDGymBasic.py:37-55)."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

import bench  # noqa: E402
from gym_TD import params as P  # noqa: E402
from gym_TD import shard  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402
from oracle import td_cpu as C  # noqa: E402

WINDOW = 16


def _threads():
    """One checker thread per CPU the process is granted (the GPU box: a 16-core quota)."""
    t, _, _ = bench.baseline_threads()
    return max(1, min(t, 32))


# the metric's N = 1 line, the N = 8 share, configs[1], configs[2] (TD-2p 20x20 multi-action)
# and configs[4] per GPU (30x30), each on the kernel td_create picks on a 256-CU MI355X
@pytest.mark.parametrize("L,B,mode,multi,want", [
    (10, 65536, "def", False, "small2"), (10, 8192, "def", False, "small"), (10, 4096, "def", False, "small2"),
    (20, 16384, "2p", True, "small2"), (30, 16384, "def", False, "small2"),
    # the other modes at 10x10 (not BASELINE lines): TD-atk (a random attacker against the
    # built-in random_tower_lv1) and TD-2p discrete, on whatever kernel td_create picks
    (10, 16384, "atk", False, None), (10, 4096, "2p", False, None)])
def test_steady_state_every_board(L, B, mode, multi, want):
    period = P.hyper_parameters.max_episode_steps
    burnin = period
    seeds = shard.shard_seeds(0, 0, B)  # bench.py's seeds at N = 1 (base 0 + global index)
    eng = TDEngine(L, B, mode, multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, info=not multi)
    bt = None
    try:
        if want and torch.cuda.get_device_properties(0).multi_processor_count == 256:
            assert eng.step_kernel == want, eng.step_kernel_name  # the kernel the bench line times
        eng.reset_all()  # failing first draws skipped (bench.py)
        bt = C.Batch(L, B, mode, 1, seeds, seeds, multi=multi, threads=_threads())
        assert bt.initial_failed == []
        assert np.array_equal(eng.obs.cpu().numpy(), bt.obs()), "initial observations differ"
        gidx = np.arange(B)
        rng = np.random.RandomState(20260)
        # the multi-action shape cycles bench.py's N_ACTION_BUFS pre-drawn batches (host + device)
        pool = []
        if multi:
            for _ in range(bench.N_ACTION_BUFS):
                d = rng.randint(0, 3, size=(B, 6, L, L)).astype(np.int64)
                a = rng.randint(0, 5, size=(B, 3, 8)).astype(np.int64)
                pool.append((d, a, torch.from_numpy(d).to(eng.device), torch.from_numpy(a).to(eng.device)))
        obs_c = np.empty((B, 45, L, L), dtype=np.float32)
        finished, resets = 0, 0
        for k in range(burnin + WINDOW):
            m = bench.stagger_mask(k, gidx, period)
            if m is not None:
                eng.reset(m)
                assert bt.reset(m) == 0
                resets += int(m.sum())
            if multi:
                acts, atk, dd, ad = pool[k % len(pool)]
                eng.step(def_act=dd, atk_act=ad)
            else:
                acts = rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64) if mode != "atk" else None
                atk = rng.randint(0, 5, size=(B, 3, 8)).astype(np.int64) if mode != "def" else None
                eng.step(def_act=None if acts is None else torch.from_numpy(acts).to(eng.device),
                         atk_act=None if atk is None else torch.from_numpy(atk).to(eng.device))
            if k < burnin:
                bt.step(acts, atk)  # (the burn-in's observations are not built on the CPU side)
                continue
            rw_c, dn_c = bt.step(acts, atk, obs=obs_c)
            rw = eng.reward.cpu().numpy()
            dn = eng.done.cpu().numpy()
            bad = np.flatnonzero(rw.view(np.uint64) != rw_c.view(np.uint64))
            assert bad.size == 0, ("reward bits", k, bad[:8].tolist())
            bad = np.flatnonzero(dn != dn_c)
            assert bad.size == 0, ("done", k, bad[:8].tolist())
            ob = eng.obs.cpu().numpy()
            diff = (ob.view(np.uint32) != obs_c.view(np.uint32)).reshape(B, -1).any(axis=1)
            assert not diff.any(), ("observation bytes", k, np.flatnonzero(diff)[:8].tolist())
            finished += int(dn.sum())
            del ob
        assert resets == int((gidx % period != 0).sum())  # every board not in phase 0 had its staggered reset
        # the steady state: about B / 1,200 auto-resets per step over the window
        assert finished >= WINDOW * B // period // 2, finished
        fl = eng.flags()
        assert (fl == 0).all(), np.unique(fl, return_counts=True)
        assert not bt.no_layout().any()
    finally:
        eng.close()
        if bt is not None:
            bt.close()
