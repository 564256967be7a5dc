"""Pin the plain-C restatement (oracle/td_cpu.c, the native CPU baseline) against
the golden vectors generated from the reference, and against the Python oracle on
random batches.  CPU-only: rewards bit for bit, observation / state / layout
sha256 digests equal."""
import numpy as np
import pytest

import goldens as G
from oracle import canon, policies
from oracle import td_cpu as C
from oracle import td_oracle as O


def _cpu_env(tr):
    return C.Env(tr["L"], tr["mode"], tr["difficulty"], tr["seed"], tr["opp_seed"], O.Config(**tr["overrides"]),
                 multi=tr["multi"], road_attempts=10000)


@pytest.mark.parametrize("name", G.traj_names())
def test_cpu_replays_golden(name):
    tr = G.load_traj(name)
    env = _cpu_env(tr)
    try:
        m, start, end = env.layout()
        nxt = G.action_stream(tr, lambda: env.layout()[0][0])
        init = tr["init"]
        assert canon.layout_digest(m, start, end) == init["lay"]
        assert len(start) == init["nr"]
        assert canon.digest(env.state_bytes()) == init["s"]
        assert canon.obs_digest(env.obs()) == init["o"]
        k = 0
        for i, rec in enumerate(tr["records"]):
            if "reset_error" in rec:
                with pytest.raises(C.RoadGenError):
                    env.reset()
                break
            if "reset" in rec:
                o = env.reset()
                m, start, end = env.layout()
                assert canon.layout_digest(m, start, end) == rec["lay"], (name, i)
                assert canon.obs_digest(o) == rec["o"], (name, i)
                assert canon.digest(env.state_bytes()) == rec["s"], (name, i)
                continue
            k += 1
            da, aa = nxt()
            obs, r, d = env.step(da, aa)
            assert canon.fhex(r) == rec["r"], (name, k)
            assert canon.digest(env.state_bytes()) == rec["s"], (name, k)
            assert canon.obs_digest(obs) == rec["o"], (name, k)
            assert int(d) == rec["d"], (name, k)
        assert not env.overflow()
    finally:
        env.close()


@pytest.mark.parametrize("L,mode,multi,difficulty", [(10, "def", False, 1), (10, "atk", False, 2), (20, "2p", True, 1),
                                                     (10, "def", True, 0), (30, "def", False, 1)])
def test_cpu_matches_python_oracle(L, mode, multi, difficulty):
    """Random seeds and actions: the C and Python restatements agree step for step,
    resets included (failing layout draws skipped on both sides)."""
    rng = np.random.RandomState(L + difficulty)
    hp = O.Hyper(allow_multiple_actions=multi)
    cfg = O.Config(base_LP=2)
    n, steps = 0, 150
    for s in range(600, 700):
        try:
            po = O.Env(L, G.MODES[mode], difficulty, s, s + 1, cfg, hp, road_attempts=1000)
        except O.RoadGenError:
            with pytest.raises(C.RoadGenError):
                C.Env(L, mode, difficulty, s, s + 1, cfg, multi=multi, road_attempts=1000)
            continue
        co = C.Env(L, mode, difficulty, s, s + 1, cfg, multi=multi, road_attempts=1000)
        try:
            for k in range(steps):
                da = aa = None
                if mode != "atk":
                    da = policies.multi_def(rng, L) if multi else policies.discrete_def(rng, L, po._board.map[0], 0.5)
                if mode != "def":
                    aa = policies.atk(rng)
                wo, wr, wd, _ = po.step(da, aa)
                o, r, d = co.step(da, aa)
                assert canon.fhex(r) == canon.fhex(wr), (s, k)
                assert d == wd, (s, k)
                assert np.array_equal(o, wo), (s, k, np.argwhere(o != wo)[:5].tolist())
                assert canon.digest(co.state_bytes()) == canon.state_digest(canon.oracle_state(po)), (s, k)
                if wd:
                    while True:
                        try:
                            wo = po.reset()
                            break
                        except O.RoadGenError:
                            with pytest.raises(C.RoadGenError):
                                co.reset()
                    assert np.array_equal(co.reset(), wo), (s, k)
        finally:
            co.close()
        n += 1
        if n == 3:
            break
    assert n == 3


def test_cpu_bench_runs():
    steps, wall = C.bench(10, "def", False, n_envs=8, seconds=0.2, threads=2)
    assert steps > 0 and wall >= 0.2


def _skip_reset(env):
    """The next layout draw that succeeds (the device's staged layouts skip failing draws)."""
    for _ in range(65):
        try:
            return env.reset()
        except C.RoadGenError:
            pass
    raise AssertionError("no layout")


@pytest.mark.parametrize("L,mode,multi,n,steps,period", [(10, "def", False, 40, 260, 37), (20, "2p", True, 12, 150, 9),
                                                          (10, "atk", False, 16, 120, 25)])
def test_batch_matches_single_envs(L, mode, multi, n, steps, period):
    """tdc_batch_* (the every-board checker of tests/test_gpu_steady.py) against one C env
    per board stepped alone: bench.py's staggered explicit resets (bench.stagger_mask with a
    short period), auto-reset, 1-LP bases so episodes end within the run; reward bits, done
    and every observation byte of every board at every step, the state at the end."""
    import bench
    cfg = O.Config(base_LP=1)
    seeds, envs, s = [], [], 400 + 7 * L
    while len(envs) < n:  # boards whose first draw succeeds (C.Env raises on a failing one)
        try:
            envs.append(C.Env(L, mode, 1, s, s, cfg, multi=multi))
            seeds.append(s)
        except C.RoadGenError:
            pass
        s += 1
    bt = C.Batch(L, n, mode, 1, seeds, seeds, cfg, multi=multi, threads=4)
    assert bt.initial_failed == []
    rng = np.random.RandomState(3)
    obs = np.zeros((n, 45, L, L), np.float32)
    ends = 0
    assert np.array_equal(bt.obs(), np.stack([e.obs() for e in envs]))
    for k in range(steps):
        m = bench.stagger_mask(k, np.arange(n), period)
        if m is not None:
            assert bt.reset(m) == 0
            for b in np.flatnonzero(m):
                _skip_reset(envs[b])
        d = (rng.randint(0, 3, size=(n, 6, L, L)) if multi else rng.randint(0, 6 * L * L + 1, size=n)) \
            if mode != "atk" else None
        a = rng.randint(0, 5, size=(n, 3, 8)) if mode != "def" else None
        rw, dn = bt.step(d, a, obs)
        for b, e in enumerate(envs):
            wo, wr, wd = e.step(None if d is None else d[b], None if a is None else a[b])
            assert canon.fhex(rw[b]) == canon.fhex(wr) and bool(dn[b]) == wd, (k, b)
            if wd:
                wo = _skip_reset(e)
                ends += 1
            assert np.array_equal(obs[b], wo), (k, b)
    for b, e in enumerate(envs):
        assert bt.state_bytes(b) == e.state_bytes(), b
        e.close()
    assert not bt.no_layout().any()
    assert ends > 0
    bt.close()
