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
