"""Pin the CPU oracle against golden vectors generated from the reference.

CPU-only.  Every trajectory fixture is replayed step by step; rewards must match
bit for bit, and the observation and canonical-state sha256 digests must be
equal (bit-exact obs and state).
"""
import numpy as np
import pytest

import goldens as G
from oracle import canon
from oracle import td_oracle as O


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, np.ndarray):
        return _jsonable(x.tolist())
    if isinstance(x, np.integer):
        return int(x)
    if isinstance(x, np.bool_):
        return bool(x)
    return x


def _info_view(info):
    ra = info["RealAction"]
    if isinstance(ra, dict):
        ra = {k: (canon.digest(np.asarray(v, np.int64).tobytes()) if np.ndim(v) else int(v)) for k, v in ra.items()}
    elif np.ndim(ra):
        ra = np.asarray(ra, np.int64).tolist()
    return _jsonable({"RealAction": ra, "Win": info["Win"], "AllowNextMove": info["AllowNextMove"],
                      "FailCode": info["FailCode"]})


@pytest.mark.parametrize("name", G.traj_names())
def test_oracle_replays_golden(name):
    tr = G.load_traj(name)
    L = tr["L"]
    for i, rec, got in G.replay_oracle(tr):
        if i == -1 or "reset" in rec:
            for key in ("o", "lay", "nr", "s"):
                assert got[key] == rec[key], (name, i, key)
            continue
        if "reset_error" in rec:
            assert got["reset_error"] == "error", (name, i)
            continue
        k = got["_k"]
        if "a" in rec:
            assert rec["a"] == got["_da"], (name, k, "action stream diverged")
        if got["s"] != rec["s"] or got["o"] != rec["o"] or got["r"] != rec["r"]:
            snap = tr["snaps"].get(str(k))
            msg = "%s step %d: reward %s/%s" % (name, k, got["r"], rec["r"])
            if snap is not None:
                want = G.snap_state(snap["state"])
                have = canon.oracle_state(got["_env"])
                msg += "\nwant %r\nhave %r" % (want, have)
                wo = G.unpack_obs(snap["obs"], L)
                bad = np.argwhere(wo != got["_obs"])
                msg += "\nobs diff at %r" % (bad[:10].tolist(),)
            pytest.fail(msg)
        assert got["d"] == rec["d"]
        if "info" in rec:
            assert _info_view(got["_info"]) == rec["info"], (name, k)
        snap = tr["snaps"].get(str(k))
        if snap is not None:
            assert np.array_equal(G.unpack_obs(snap["obs"], L), got["_obs"])


def test_roadgen_table():
    """create_road_v2 restatement vs the reference's reset outcomes, 400 seeds x 3 sizes."""
    table = G.load_roadgen()
    for L, rows in table.items():
        L = int(L)
        for s, row in rows.items():
            rng = np.random.RandomState(int(s))
            nr = rng.randint(low=1, high=4)
            try:
                roads = O.create_road(rng, L, nr, max_attempts=10000)
            except O.RoadGenError:
                assert "err" in row, (L, s)
                continue
            assert "err" not in row, (L, s, row)
            m, st, en = O.layout_from_roads(roads, L)
            assert nr == row["nr"]
            assert canon.layout_digest(m, st, en) == row["lay"], (L, s)
            assert int(rng.randint(0, 2 ** 31 - 1)) == row["next"], (L, s)


def test_reference_kat():
    """The reference's own known-answer test (TDBoard.py:674-751), seed 1024."""
    z = np.load(G.GOLDEN + "/kat_seed1024.npz")
    rng = np.random.RandomState()
    rng.seed(1024)
    cfg, hp = O.Config(), O.Hyper()
    b = O.Board(10, 2, rng, cfg, hp)
    assert np.array_equal(b.map, z["map"])
    assert np.array_equal(b.get_states(), z["obs"])
    assert [list(x) for x in b.start] == z["start"].tolist() and list(b.end) == z["end"].tolist()
    # the KAT's hand-written expectations (TDBoard.py:690-748)
    obs = b.get_states()
    assert obs[4, 4, 0] == 1 and obs[6, 4, 9] == 1 and obs[7, 9, 4] == 1
    assert np.all(obs[5] == 1) and np.all(obs[21] == 1) and np.all(obs[22:25] == 0)
    assert np.all(obs[9] == b.map[4].astype(np.float32) / np.float32(14))
    assert obs[11, 0, 0] == np.float32(0.1) and obs[12, 0, 0] == 0 and obs[13, 0, 0] == 0
    for i, c in enumerate((8, 15, 40, 30)):
        assert np.all(obs[41 + i] == np.float32(10 / c / 8))
    # summons fail at zero attacker cost (TDBoard.py:749-751)
    for i in range(4):
        for j in range(2):
            ok, _ = b.summon_cluster([i], j)
            assert not ok
    assert not any(z["summons"])


def test_doctests():
    """Doctest facts of TDBoard.py:151,160,170-180,374-382."""
    cfg, hp = O.Config(), O.Hyper()
    assert O.n_channels(cfg) == 45
    b = O.Board(10, 2, np.random.RandomState(3), cfg, hp)
    assert b.get_states().shape == (45, 10, 10)
    assert not b.is_valid_pos([10, 2]) and not b.is_valid_pos([-1, 3])
    assert not b.is_valid_pos([5, 10]) and not b.is_valid_pos([4, -1]) and b.is_valid_pos([2, 3])
    assert not b.done()
    b.base_LP = 0
    assert b.done()
    b.base_LP, b.steps = 5, 1200
    assert b.done()
