"""A refill claim held past the 1-s waits: the ring guard gives up on the
board and says so (TD_FLAG_CLAIM_TIMEOUT, td_guard_timeouts), and the board's episode
end -- its ring empty, the claim still held -- is flagged no_layout: the board keeps its
finished episode instead of being stepped on a stale layout.  Once the claim is given
back the next ring guard draws its layout and the board starts a new episode (reference:
TDGymBasic.reset at every episode end, gym_TD/envs/TDGymBasic.py:37-55)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

FLAG_NO_LAYOUT, FLAG_CLAIM_TIMEOUT = 8, 32


def test_claim_held_past_the_wait_is_flagged_not_stepped():
    from test_gpu_parity import reference_settings
    L, B, HELD = 10, 64, 5
    ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.02)  # episodes end within ~100 steps
    seeds = np.arange(B, dtype=np.int64) + 31000
    with reference_settings(ov, False):
        eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    try:
        eng.set_refill_interval(0)  # every layout from the ring guard on the step stream
        _lib.check(_lib.lib.td_debug_set_claim(eng._h, HELD, 1))  # a refill "holds" board HELD
        eng.reset_all()  # (the reset kernel draws the first layouts now, without claims)
        g = torch.Generator(device="cuda").manual_seed(3)
        ended = None
        for k in range(400):
            eng.step(def_act=torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64))
            if bool(eng.done[HELD].item()):
                ended = k
                break
        assert ended is not None, "board %d never finished an episode" % HELD
        flags = eng.flags()
        assert flags[HELD] & FLAG_CLAIM_TIMEOUT and flags[HELD] & FLAG_NO_LAYOUT, flags[HELD]
        assert eng.guard_timeouts() >= 1  # the first guard already gave up on the board
        others = np.delete(flags, HELD)
        assert (others == 0).all(), others[others != 0]
        st = eng.board_state(HELD)
        assert st["steps"] == ended + 1 and st["base_LP"] == 0  # the finished episode, not a new one
        # the claim still held: neither the step (take_dry_ring) nor the guard waits for the
        # flagged board again -- 30 more steps (two guard launches) take far less than one 1-s wait
        import time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(30):
            eng.step(def_act=torch.full((B,), 6 * L * L, device="cuda", dtype=torch.int64))
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 0.5, time.perf_counter() - t0
        st = eng.board_state(HELD)  # still its finished episode (stepped on, done at every step)
        assert st["base_LP"] == 0 and st["steps"] == ended + 31, st
        assert eng.guard_timeouts() == 1  # counted once, not at every guard launch
        # give the claim back: the next ring guard draws the layout, the board starts over
        _lib.check(_lib.lib.td_debug_set_claim(eng._h, HELD, 0))
        for k in range(16):
            eng.step(def_act=torch.full((B,), 6 * L * L, device="cuda", dtype=torch.int64))
        st = eng.board_state(HELD)
        assert st["steps"] < 16 and st["base_LP"] == 1, st
        assert eng.guard_timeouts(clear=True) >= 1 and eng.guard_timeouts() == 0
    finally:
        eng.close()
