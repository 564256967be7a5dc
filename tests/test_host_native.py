"""CPU tests of libtdstep.so's host side (no GPU): exported symbols, the two
MT19937 streams, native road generation and layout records, pinned against
CPython ``random``, numpy ``RandomState`` and the reference's golden road table."""
import random
import re

import numpy as np
import pytest

import goldens as G
from oracle import canon
from oracle import td_oracle as O

from gym_TD import _lib
from gym_TD.engine import generate_layout, layout_planes

lib = _lib.lib
U32 = _lib.ctypes.c_uint32


def _p(a):
    return _lib.ptr(a, U32)


DIAG = {"td_set_step_kernel", "td_board_map", "td_set_store_policy", "td_debug_set_claim"}


@pytest.mark.parametrize("header", ["tdstep.h", "td_diag.h"])
def test_header_symbols_exported(header):
    """Every function include/*.h declares is exported by libtdstep.so; the test hooks are
    declared only in td_diag.h, never in the drop-in header."""
    hdr = open(G.GOLDEN + "/../../include/" + header).read()
    names = set(re.findall(r"\b(td_[a-z_0-9]+)\s*\(", hdr))
    assert len(names) >= (25 if header == "tdstep.h" else 4)
    for n in sorted(names):
        assert hasattr(lib, n), n
    if header == "tdstep.h":
        assert not (names & DIAG), names & DIAG
    else:
        assert names == DIAG, names


def test_alloc_placement_of_unknown_block():
    """td_alloc_is_contiguous answers -1 for memory td_alloc_device did not hand out."""
    buf = np.zeros(16, np.uint8)
    assert lib.td_alloc_is_contiguous(buf.ctypes.data) == -1
    assert lib.td_alloc_is_contiguous(None) == -1


def test_config_default_matches_reference_defaults():
    c = _lib.TdConfig()
    lib.td_config_default(c)
    ref = O.Config()
    for name in ("enemy_LP", "enemy_speed", "enemy_defense", "enemy_cost", "tower_attack", "tower_range",
                 "tower_splash_range", "tower_cost", "tower_attack_interval"):
        assert [[getattr(c, name)[t][l] for l in range(2)] for t in range(4)] == getattr(ref, name)
    for name in ("tower_destruct_return", "frozen_time", "frozen_ratio", "attacker_init_cost",
                 "defender_init_cost", "base_LP", "max_cost", "reward_kill", "penalty_leak", "reward_time",
                 "attacker_cost_init_rate", "attacker_cost_final_rate", "defender_cost_rate", "tower_distance",
                 "enemy_upgrade_at"):
        assert getattr(c, name) == getattr(ref, name), name
    assert c.max_episode_steps == 1200 and c.max_cluster_length == 8 and c.max_num_of_roads == 3


@pytest.mark.parametrize("seed", [0, 1, 42, 2 ** 31 + 7, 2 ** 32 - 1])
def test_cpython_random_stream(seed):
    w = np.zeros(625, np.uint32)
    lib.td_py_seed(_p(w), seed)
    r = random.Random(seed)
    st = r.getstate()[1]
    assert list(w[:624]) == list(st[:624]) and int(w[624]) == st[624]
    for n in (1, 2, 3, 4, 5, 8, 25, 100, 1000):
        for _ in range(50):
            assert lib.td_py_randint(_p(w), 0, n - 1) == r.randint(0, n - 1)
    for _ in range(2000):
        assert lib.td_mt_next(_p(w)) == r.getrandbits(32)


@pytest.mark.parametrize("seed", [0, 3, 1024, 2 ** 32 - 1])
def test_numpy_legacy_stream(seed):
    w = np.zeros(625, np.uint32)
    lib.td_np_seed(_p(w), seed)
    rs = np.random.RandomState(seed)
    st = rs.get_state()
    assert list(w[:624]) == list(st[1]) and int(w[624]) == st[2]
    for lo, hi in ((0, 1), (0, 2), (0, 4), (1, 4), (3, 7), (1, 2), (0, 3), (5, 17), (0, 1000)):
        for _ in range(40):
            assert lib.td_np_randint(_p(w), lo, hi) == rs.randint(lo, hi)


def test_roadgen_matches_reference_table():
    """Native create_road_v2 vs the reference's reset outcome, 1200 env seeds."""
    table = G.load_roadgen()
    for Ls, rows in table.items():
        L = int(Ls)
        for s, row in rows.items():
            w = np.zeros(625, np.uint32)
            lib.td_np_seed(_p(w), int(s))
            st, rec = generate_layout(w, L)
            if "err" in row:
                assert st != 0, (L, s)
                continue
            assert st == 0, (L, s, st)
            m, start, end, nr = layout_planes(rec, L)
            assert nr == row["nr"]
            assert canon.layout_digest(m, start, end) == row["lay"], (L, s)
            # the stream is left where the reference leaves it
            assert lib.td_np_randint(_p(w), 0, 2 ** 31 - 1) == row["next"], (L, s)


def test_roadgen_error_kinds_match_oracle():
    """Failing L=10 seeds: same failure, same stream position as the oracle restatement."""
    for s in (1, 45, 54, 55, 217):
        w = np.zeros(625, np.uint32)
        lib.td_np_seed(_p(w), s)
        st, _ = generate_layout(w, 10)
        rng = np.random.RandomState(s)
        nr = rng.randint(1, 4)
        with pytest.raises(O.RoadGenError):
            O.create_road(rng, 10, nr, max_attempts=20000)
        assert st in (1, 2)
        assert lib.td_np_randint(_p(w), 0, 2 ** 31 - 1) == rng.randint(0, 2 ** 31 - 1)


def test_layout_from_roads_matches_board_planes():
    rng = np.random.RandomState(7)
    for L in (10, 20, 30):
        for _ in range(5):
            nr = rng.randint(1, 4)
            try:
                roads = O.create_road(rng, L, nr, max_attempts=20000)
            except O.RoadGenError:
                continue
            m, start, end = O.layout_from_roads(roads, L)
            cells = np.asarray([p[0] * L + p[1] for r in roads for p in r], dtype=np.int32)
            off = np.cumsum([0] + [len(r) for r in roads]).astype(np.int32)
            rec = np.zeros(8 + L * L, np.uint32)
            assert lib.td_layout_from_roads(L, len(roads), _lib.ptr(cells, _lib.ctypes.c_int32),
                                            _lib.ptr(off, _lib.ctypes.c_int32), _p(rec)) == 0
            m2, s2, e2, nr2 = layout_planes(rec, L)
            assert np.array_equal(m, m2) and s2 == start and e2 == end and nr2 == len(roads)


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    c = _lib.TdConfig()
    lib.td_config_default(c)
    h = lib.td_create(c, 10, 4, 0, 0, 1, 0)
    assert not h
    assert lib.td_last_error()


def _digest_of_roads(roads, L):
    m, start, end = O.layout_from_roads(roads, L)
    return canon.layout_digest(m, start, end)


def test_hopeless_branch_rule_is_pinned():
    """The hopeless-branch rule (td_layout.h branch_hopeless) against the bounded loops it
    replaces, on auto-reset sequences of L = 10 draws: every draw the rule fails at once is
    one whose branch loop burns the whole 1,000-attempt bound (the reference never
    returns), and every other draw -- layout, error kind, stream position after it -- is
    the bounded loops' own.  The native host restatement follows the rule draw for draw."""
    L, hopeless, draws = 10, 0, 0
    for seed in range(200):
        rs = np.random.RandomState(seed)
        w = np.zeros(625, np.uint32)
        lib.td_np_seed(_p(w), seed)
        for _ in range(8):
            draws += 1
            old = np.random.RandomState()
            old.set_state(rs.get_state())
            nr = rs.randint(1, 4)
            assert old.randint(1, 4) == nr
            try:
                roads, err = O.create_road(rs, L, nr, max_attempts=1000), None
            except O.RoadGenError as ex:
                roads, err = None, str(ex)
            try:
                roads_old, err_old = O.create_road(old, L, nr, max_attempts=1000, prove_hopeless=False), None
            except O.RoadGenError as ex:
                roads_old, err_old = None, str(ex)
            st, rec = generate_layout(w, L, 1000)
            if err is not None and "loops forever" in err:
                hopeless += 1
                assert err_old == "retry bound exceeded", (seed, err_old)
                assert st == 3, (seed, st)  # ROAD_ERR_BOUND, at the loop's entry
            else:
                assert err == err_old and (roads == roads_old), (seed, err, err_old)
                assert old.get_state()[2] == rs.get_state()[2] and (old.get_state()[1] == rs.get_state()[1]).all()
                if err is None:
                    assert st == 0
                    m, start, end, nr2 = layout_planes(rec, L)
                    assert nr2 == nr and canon.layout_digest(m, start, end) == _digest_of_roads(roads, L)
                else:
                    assert st != 0
            # the native stream is where the Python restatement's is
            st_py = rs.get_state()
            assert list(w[:624]) == list(st_py[1]) and int(w[624]) == st_py[2], seed
    assert hopeless >= 3, (hopeless, draws)


def test_cpu_oracle_follows_the_hopeless_rule():
    """The C restatement's auto-reset sequence (failing draws skipped) equals the native
    host sequence under the same rule, over boards whose sequences hold hopeless draws."""
    from oracle import td_cpu as C
    L, checked = 10, 0
    for seed in range(60):
        try:
            env = C.Env(L, "def", 1, seed, seed, road_attempts=1000)
        except C.RoadGenError:
            continue
        w = np.zeros(625, np.uint32)
        lib.td_np_seed(_p(w), seed)
        st, rec = generate_layout(w, L, 1000)
        assert st == 0
        try:
            for _ in range(10):
                m, start, end, _ = layout_planes(rec, L)
                m2, s2, e2 = env.layout()
                assert canon.layout_digest(m, start, end) == canon.layout_digest(m2.astype(np.int32), s2, e2), seed
                while True:  # next layout of both, failing draws skipped
                    st, rec = generate_layout(w, L, 1000)
                    try:
                        env.reset()
                        assert st == 0, seed
                        break
                    except C.RoadGenError:
                        assert st != 0, seed
                        checked += st == 3
        finally:
            env.close()
    assert checked >= 1


@pytest.mark.parametrize("B", [1, 2, 7, 8, 9, 15, 16, 17, 100, 1000, 4095, 4096, 8192, 65536, 65537])
def test_board_map_is_an_xcd_contiguous_permutation(B):
    """td_board_map: every board stepped by exactly one block; the blocks of one XCD
    (i % 8) step one contiguous range of boards, in block order (neighbouring boards share
    an L2), and the ranges follow each other by XCD."""
    for kind in (0, 1):
        m = np.zeros(B, np.int32)
        assert lib.td_board_map(B, kind, 1, _lib.ptr(m, _lib.ctypes.c_int32)) == 0
        assert np.array_equal(np.sort(m), np.arange(B))
        start = 0
        for x in range(8):
            mine = m[x::8]
            assert np.array_equal(mine, np.arange(start, start + len(mine)))
            start += len(mine)
        ident = np.zeros(B, np.int32)
        assert lib.td_board_map(B, kind, 0, _lib.ptr(ident, _lib.ctypes.c_int32)) == 0
        assert np.array_equal(ident, np.arange(B))
