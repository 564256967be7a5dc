"""The device road generator (td_layout.h run by td_reset_kernel / td_refill_kernel)
against the reference's own 1,200-seed road table (tests/golden/roadgen.json.gz,
TDRoadGen.py:4-199 driven by TDGymBasic.reset :42-51), on the GPU through the C-ABI.

* Explicit reset (td_reset, the reset kernel's draw): for every table seed the layout
  digest and num_roads, the failure of each seed the reference raises on, and the
  stream position after the draw (the table's next 31-bit draw).
* Auto-reset (the refill kernel's resumable draws, cut at kRefillWalks walks per
  launch): every layout a board's episodes run on equals the host restatement's
  sequence of draws on the same stream, failing draws skipped -- the host
  restatement is itself pinned to the same table (test_host_native.py)."""
import copy
import types

import numpy as np
import pytest
import torch

import goldens as G
from oracle import canon

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import _lib  # noqa: E402
from gym_TD import params as P  # noqa: E402
from gym_TD.engine import TDEngine, generate_layout, layout_planes  # noqa: E402

ROAD_ATTEMPTS = 1000  # td_kernels.h kRoadAttempts: the device's bound of each create_road_v2 loop
LAYOUT_RETRIES = 64   # td_kernels.h kLayoutRetries: auto-reset skips up to this many failing draws


def _next31(w):
    w = w.copy()
    return int(_lib.lib.td_np_randint(_lib.ptr(w, _lib.ctypes.c_uint32), 0, 2 ** 31 - 1))


@pytest.mark.parametrize("L", [10, 20, 30])
def test_reset_kernel_matches_reference_table(L):
    rows = G.load_roadgen()[str(L)]
    seeds = sorted(int(s) for s in rows)
    eng = TDEngine(L, len(seeds), "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        _, failed = eng.reset()
        want_fail = [b for b, s in enumerate(seeds) if "err" in rows[str(s)]]
        assert sorted(failed) == want_fail, (L, failed, want_fail)
        st = eng.export_state()
        for b, s in enumerate(seeds):
            row = rows[str(s)]
            w = eng.get_np_state(b)
            if "err" in row:
                # the reference raises; the device leaves the stream where the host
                # restatement (pinned to the oracle's failure kinds) leaves it
                h = np.zeros(625, np.uint32)
                _lib.lib.td_np_seed(_lib.ptr(h, _lib.ctypes.c_uint32), s)
                hst, _ = generate_layout(h, L, ROAD_ATTEMPTS)
                assert hst != 0, (L, s)
                assert w.tolist() == h.tolist(), (L, s)
                assert eng.board_state(b, st)["num_roads"] == 0  # never reset: unchanged
                continue
            m, start, end = eng.map_planes(b, st)
            assert int(st["hdr"][b]["num_roads"]) == row["nr"], (L, s)
            assert canon.layout_digest(m, start, end) == row["lay"], (L, s)
            assert _next31(w) == row["next"], (L, s)
    finally:
        eng.close()


def _host_sequence(seed, L, n):
    """The first n layouts an auto-reset board plays on (failing draws skipped),
    with the number of failing draws skipped on the way."""
    w = np.zeros(625, np.uint32)
    _lib.lib.td_np_seed(_lib.ptr(w, _lib.ctypes.c_uint32), seed)
    out, skipped = [], 0
    while len(out) < n:
        for _ in range(LAYOUT_RETRIES + 1):
            st, rec = generate_layout(w, L, ROAD_ATTEMPTS)
            if st == 0:
                break
            skipped += 1
        assert st == 0
        m, start, end, nr = layout_planes(rec, L)
        out.append((canon.layout_digest(m, start, end), nr))
    return out, skipped


def test_refill_kernel_layouts_match_host_sequence():
    """400 boards (the table's L = 10 seeds whose first draw succeeds), episodes of 64
    steps, 640 steps with auto-reset: the layouts the refill kernel drew -- resumable
    draws cut at 48 walks per launch, the failing ones skipped -- are the host
    restatement's, layout for layout."""
    L, ep, steps = 10, 64, 640
    rows = G.load_roadgen()[str(L)]
    seeds = sorted(int(s) for s in rows if "err" not in rows[str(s)])[:400]
    B = len(seeds)
    n_eps = steps // ep + 1
    want, skipped = zip(*[_host_sequence(s, L, n_eps) for s in seeds])
    # failing draws take ~1,000 walks per retry loop: cut at 48 walks a launch, every one of
    # them ran through the resumable path (RoadGen::draw resumed across refill launches)
    assert sum(skipped) > 0
    hp = types.SimpleNamespace(max_episode_steps=ep, max_cluster_length=8, max_num_of_roads=3,
                               allow_multiple_actions=False)
    cfg = copy.deepcopy(P.config)
    cfg.base_LP = 10 ** 6  # no leak ends an episode early: every board's episodes end together
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, cfg=cfg, hp=hp)
    try:
        _, failed = eng.reset()
        assert not failed
        played = [[] for _ in range(B)]

        def record():
            st = eng.export_state()
            for b in range(B):
                m, start, end = eng.map_planes(b, st)
                played[b].append((canon.layout_digest(m, start, end), int(st["hdr"][b]["num_roads"])))

        record()
        g = torch.Generator(device="cuda").manual_seed(11)
        for k in range(steps):
            d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            eng.step(def_act=d)
            if (k + 1) % ep == 0:
                assert bool(eng.done.all()), k
                record()
        assert (eng.flags() == 0).all()
        for b in range(B):
            assert played[b] == list(want[b][:len(played[b])]), (b, seeds[b])
    finally:
        eng.close()



@pytest.mark.parametrize("L,B,resets", [(10, 512, 10), (20, 128, 4)])
def test_reset_sequence_matches_host(L, B, resets):
    """Explicit resets one after another (each draws the board's next layout, failing
    draws leaving the board as it was): the reset kernel's draws -- including the
    hopeless branch loops failed at once (td_layout.h branch_hopeless; ~1 % of L = 10
    draws) -- equal the host restatement's, failure for failure, with the stream left
    at the same position after every draw."""
    seeds = list(range(50000, 50000 + B))
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    host = []
    for s in seeds:
        w = np.zeros(625, np.uint32)
        _lib.lib.td_np_seed(_lib.ptr(w, _lib.ctypes.c_uint32), s)
        host.append(w)
    try:
        bound = 0
        for r in range(resets):
            _, failed = eng.reset()
            st = eng.export_state()
            for b in range(B):
                hst, rec = generate_layout(host[b], L, ROAD_ATTEMPTS)
                bound += hst == 3
                assert (b in failed) == (hst != 0), (r, b, hst)
                assert eng.get_np_state(b).tolist() == host[b].tolist(), (r, b)
                if hst == 0:
                    m, start, end, nr = layout_planes(rec, L)
                    m2, s2, e2 = eng.map_planes(b, st)
                    assert canon.layout_digest(m, start, end) == canon.layout_digest(m2, s2, e2), (r, b)
        if L == 10:
            assert bound >= 10, bound  # hopeless draws were among them
    finally:
        eng.close()
