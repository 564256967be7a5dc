"""Store policies of the observation lines a board shares with its neighbours (GPU).

18,000 B (10x10) / 72,000 B (20x20) of observation per board is not a multiple of the
128-B line, so each board shares its first and last line with the boards beside it.
The product stores those halves with plain write-back stores (td_set_store_policy edge_wt
= 2): with the XCD-contiguous board map both halves meet in one XCD's L2; where a pair is
split across two XCDs (the ends of the XCD blocks, or every pair with xcd_map = 0) both L2s
write their dirty bytes back.  Every policy and map must give the same bytes as the
write-through form (edge_wt = 1) on the same seeds and actions.  The batch is large
enough that the observation is not stored write-through as a whole (it exceeds the
256-MiB Infinity Cache), so the shared-line path is the one taken."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

# (xcd_map, edge_wt): the product first, then the reference form and the split pairs
POLICIES = [(1, 2), (1, 1), (0, 2), (0, 1)]


def _engine(L, B, seeds, xcd, edge):
    e = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    e.set_store_policy(xcd, edge)
    return e


@pytest.mark.parametrize("L,B,steps", [(20, 4096, 40), (10, 16384, 60)])
def test_shared_line_policies_agree(L, B, steps):
    assert B * 45 * L * L * 4 > 256 * 2**20  # beyond the write-through-everything batches
    seeds = np.arange(B) + 7100
    engs = [_engine(L, B, seeds, x, e) for x, e in POLICIES]
    try:
        for e in engs:
            e.reset_all()
        g = torch.Generator(device="cuda").manual_seed(17)
        for k in range(steps):
            act = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            for e in engs:
                e.step(def_act=act)
            ref = engs[1]  # write-through, XCD map on
            for i, e in enumerate(engs):
                if e is ref:
                    continue
                assert torch.equal(e.obs, ref.obs), (POLICIES[i], k)
                assert torch.equal(e.reward, ref.reward) and torch.equal(e.done, ref.done), (POLICIES[i], k)
    finally:
        for e in engs:
            e.close()


def test_engine_observation_block():
    """The engine's observation lives in a td_alloc_device block adopted by torch
    (contiguous device memory), is freed with its last tensor, and steps give the same
    bytes as into a torch-allocated buffer."""
    L, B = 10, 512
    seeds = np.arange(B) + 900
    a = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    b = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    try:
        assert getattr(a.obs, "_td_block", False), "torch did not adopt the td_alloc_device block"
        b.obs = torch.zeros_like(b.obs)
        b._io.obs = b.obs.data_ptr()
        a.reset_all()
        b.reset_all()
        g = torch.Generator(device="cuda").manual_seed(3)
        for k in range(60):
            d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            a.step(def_act=d)
            b.step(def_act=d)
            assert torch.equal(a.obs, b.obs), k
        view = a.obs[3]
        keep = view.clone()
    finally:
        a.close()
        b.close()
    torch.cuda.synchronize()
    assert torch.equal(view, keep)  # a view keeps the block alive after the engine closed


def test_alloc_reports_the_granted_placement():
    """td_alloc_is_contiguous answers how a td_alloc_device block was placed (a
    refused contiguous request falls back to a plain allocation, and TDEngine.obs_alloc --
    the key bench.py quotes PMC traffic records by -- must say so), -1 once it is freed."""
    from gym_TD.engine import device_zeros
    for want in (True, False):
        t = device_zeros((1 << 20,), torch.float32, "cuda", contiguous=want)
        assert getattr(t, "_td_block", False)
        got = _lib.lib.td_alloc_is_contiguous(t.data_ptr())
        assert got in (0, 1) and t._td_contig == (got == 1)
        if not want:
            assert got == 0  # a plain request is never contiguous
        ptr = t.data_ptr()
        del t
        import gc
        gc.collect()
        torch.cuda.synchronize()
        assert _lib.lib.td_alloc_is_contiguous(ptr) == -1
    eng = TDEngine(10, 64, "def", False, 1, np_seeds=np.arange(64), py_seeds=np.arange(64))
    try:
        got = _lib.lib.td_alloc_is_contiguous(eng.obs.data_ptr())
        assert eng.obs_alloc == {1: "contiguous", 0: "plain"}[got]
    finally:
        eng.close()
