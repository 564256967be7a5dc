"""Deep-in-time batched parity: 64-128 boards stepped 1,300 times in one launch per
step with auto-reset on, against the C restatement (oracle/td_cpu.c, golden-pinned)
bit for bit -- rewards, done, every observation byte every step, the canonical state
of every board every 25 steps.

The episodes run to the 1,200-step limit (base_LP raised so leaks never end them), so
every board crosses the enemy-upgrade threshold (progress >= 0.75, TDBoard.py:201),
finishes its episode and auto-resets onto its next staged layout (failing draws
skipped on both sides).  The two shapes are chosen so that boards carry more than
64 live enemies (10x10, an idle defender against a fast attacker) and more than 16
towers (20x20, a builder defender): the step kernel prefetches 16 enemy and 16 tower
slots with the header and loads the rest afterwards (the large kernel loads exactly the
live slots once the header is in), and lanes hold enemies l and l + 64 (td_step.hip
prefetch_issue / load_board / board_step).  Each shape runs on all three step kernels."""
import copy

import numpy as np
import pytest
import torch

from oracle import canon
from oracle import td_cpu as C
from oracle import td_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import params as P  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

ROAD_ATTEMPTS = 1000  # td_kernels.h kRoadAttempts
LAYOUT_RETRIES = 64   # td_kernels.h kLayoutRetries


def _policy(rng, L, roads, p_build):
    """p_build > 0: with probability p_build an arrow tower (the cheapest, TDParam
    tower_cost[0]) on a random cell within 2 of a road cell, else a uniform action over
    [0, 6 L^2].  p_build == 0: a mostly idle defender (90 % the empty action 6 L^2)."""
    if p_build == 0.0:
        return 6 * L * L if rng.random_sample() < 0.9 else int(rng.randint(0, 6 * L * L + 1))
    if rng.random_sample() < p_build:
        rr, cc = roads
        k = rng.randint(len(rr))
        r = min(max(int(rr[k]) + rng.randint(-2, 3), 0), L - 1)
        c = min(max(int(cc[k]) + rng.randint(-2, 3), 0), L - 1)
        return r * L + c
    return int(rng.randint(0, 6 * L * L + 1))


def _reset_skipping(env):
    """Auto-reset's layout: the next draw that succeeds (TDGymBasic.reset, failing draws skipped)."""
    for _ in range(LAYOUT_RETRIES + 1):
        try:
            return env.reset()
        except C.RoadGenError:
            pass
    raise AssertionError("no layout in %d draws" % (LAYOUT_RETRIES + 1))


# 10x10: an idle defender against a fast attacker (cost rates 4 -> 8 per step): 25-65 live
# enemies per board late in the episode, past the 16 prefetched slots and past lane 63.
# 20x20: a builder defender: up to ~24 towers per board.
@pytest.mark.parametrize("kernel", ("large", "small", "small2"))
@pytest.mark.parametrize("L,B,p_build,over", [
    (10, 128, 0.0, dict(attacker_cost_init_rate=4, attacker_cost_final_rate=8)),
    (20, 64, 0.8, {})])
def test_deep_batched_autoreset_vs_c_oracle(L, B, p_build, over, kernel):
    steps, every = 1300, 25
    over = dict(over, base_LP=10 ** 6)
    cfg = O.Config(**over)
    seeds, orc = [], []
    s = 20000 + L
    while len(seeds) < B:
        try:
            orc.append(C.Env(L, "def", 1, s, s, cfg, road_attempts=ROAD_ATTEMPTS))
            seeds.append(s)
        except C.RoadGenError:
            pass
        s += 1
    dcfg = copy.deepcopy(P.config)
    for key, v in over.items():
        setattr(dcfg, key, v)
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, cfg=dcfg,
                   step_kernel=kernel)
    try:
        assert eng.step_kernel == kernel
        obs, failed = eng.reset()
        assert not failed
        ob = obs.cpu().numpy()
        for b in range(B):
            assert np.array_equal(ob[b], orc[b].obs()), b
        roads = [np.nonzero(o.layout()[0][0]) for o in orc]
        rng = np.random.RandomState(L)
        max_en = max_tw = 0
        resets = 0
        for k in range(steps):
            acts = np.array([_policy(rng, L, roads[b], p_build) for b in range(B)], dtype=np.int64)
            eng.step(def_act=torch.from_numpy(acts))
            ob = eng.obs.cpu().numpy()
            rw = eng.reward.cpu().numpy()
            dn = eng.done.cpu().numpy()
            for b in range(B):
                wo, wr, wd = orc[b].step(int(acts[b]))
                assert canon.fhex(rw[b]) == canon.fhex(wr), (L, k, b)
                assert bool(dn[b]) == wd, (L, k, b)
                if wd:  # the device returns the next episode's first observation
                    wo = _reset_skipping(orc[b])
                    roads[b] = np.nonzero(orc[b].layout()[0][0])
                    resets += 1
                assert np.array_equal(ob[b], wo), (L, k, b, np.argwhere(ob[b] != wo)[:5].tolist())
            if k % every == every - 1 or dn.any():
                st = eng.export_state()
                max_en = max(max_en, int(st["hdr"]["n_en"].max()))
                max_tw = max(max_tw, int(st["hdr"]["n_tw"].max()))
                for b in range(B):
                    assert canon.state_digest(eng.board_state(b, st)) == canon.digest(orc[b].state_bytes()), (L, k, b)
        assert (eng.flags() == 0).all()
        assert resets >= B  # every board finished its 1,200-step episode and auto-reset
        # the tails beyond the 16 prefetched slots were exercised
        assert (max_en > 48) if p_build == 0.0 else (max_tw > 16), (max_en, max_tw)
    finally:
        eng.close()
        for o in orc:
            o.close()
