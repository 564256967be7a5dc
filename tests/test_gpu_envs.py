"""GPU parity of the batched paths the golden replays do not reach: TD-atk and
TD-2p boards stepped together in one launch (every built-in opponent level,
discrete and multi-action, the info tensors), and the TDVecEnv rollout surface
(auto-reset with failing layout draws, sharding invariance of trajectories).
Everything is compared bit-exactly with the CPU oracle on the same seeds."""
import copy

import numpy as np
import pytest
import torch

import goldens as G
from oracle import canon, policies
from oracle import td_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import envs as E  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

from test_gpu_parity import reference_settings  # noqa: E402

ROAD_ATTEMPTS = 1000  # td_kernels.h kRoadAttempts: the device's bound of each create_road_v2 loop


def _first_ok_seeds(L, n, start, mode, multi, difficulty, cfg=None, random_agent=True):
    """Seeds whose first layout draw succeeds, with their oracle envs."""
    hp = O.Hyper(allow_multiple_actions=multi)
    seeds, envs = [], []
    s = start
    while len(seeds) < n:
        try:
            envs.append(O.Env(L, G.MODES[mode], difficulty, s, s, cfg or O.Config(), hp, random_agent=random_agent,
                              road_attempts=ROAD_ATTEMPTS))
            seeds.append(s)
        except O.RoadGenError:
            pass
        s += 1
    return seeds, envs


def _fc_list(row):
    return [int(v) for v in row if v >= 0]


_MODE_CASES = [
    (10, 24, "atk", False, 0, 150, True),
    (10, 24, "atk", False, 1, 150, True),
    (10, 24, "atk", False, 2, 150, True),
    (20, 12, "atk", False, 2, 100, True),
    (10, 24, "2p", False, 1, 150, True),
    (10, 16, "2p", True, 1, 120, True),
    (10, 16, "def", True, 1, 120, True),
    (10, 24, "def", False, 0, 150, True),
    # sizes off the specialised kernels (generic L <= 32 build; odd L*L: scalar observation path)
    (8, 16, "def", False, 1, 120, True),
    (12, 12, "atk", False, 1, 100, True),
    (15, 8, "2p", True, 1, 80, True),
    (16, 8, "def", False, 1, 100, True),
    # random_agent=False: the opponents on each board's numpy layout stream (OppRng<true>)
    (10, 16, "def", True, 1, 120, False),
    (10, 24, "def", False, 0, 150, False),
    (10, 24, "atk", False, 1, 150, False),
    (20, 12, "atk", False, 2, 100, False),
    (30, 6, "def", False, 1, 80, False),
]


@pytest.mark.parametrize("L,B,mode,multi,difficulty,steps,random_agent,kernel", [
    c + (k,) for c in _MODE_CASES for k in (("large", "small", "small2") if c[0] in (10, 20, 30) else ("large",))])
def test_batched_modes_vs_oracle(L, B, mode, multi, difficulty, steps, random_agent, kernel):
    """B boards of one mode in one launch vs B oracle envs: reward bits, done,
    state digest, observation bytes and the info tensors of every board, on every step
    kernel the map size has."""
    seeds, orc = _first_ok_seeds(L, B, 3000 + 97 * difficulty, mode, multi, difficulty, random_agent=random_agent)
    eng = TDEngine(L, B, mode, multi, difficulty, np_seeds=seeds, py_seeds=seeds, autoreset=False,
                   random_agent=random_agent, step_kernel=kernel)
    try:
        assert eng.step_kernel == kernel
        _, failed = eng.reset()
        assert not failed
        rng = np.random.RandomState(L * 31 + difficulty)
        for k in range(steps):
            da = aa = None
            if mode != "atk":
                if multi:
                    da = np.stack([policies.multi_def(rng, L) for _ in range(B)]).astype(np.int64)
                else:
                    da = np.array([policies.discrete_def(rng, L, o._board.map[0], 0.5) for o in orc], dtype=np.int64)
            if mode != "def":
                aa = np.stack([policies.atk(rng) for _ in range(B)]).astype(np.int64)
            eng.step(def_act=None if da is None else torch.from_numpy(da),
                     atk_act=None if aa is None else torch.from_numpy(aa))
            ob, rw, dn = eng.obs.cpu().numpy(), eng.reward.cpu().numpy(), eng.done.cpu().numpy()
            win, an = eng.win.cpu().numpy(), eng.allow_next.cpu().numpy()
            cdn = eng.cooldowns.cpu().numpy()
            assert ((an & 0xFC) == 0).all()  # AllowNextMove bits only (ABI 2: cool-downs have their own output)
            rd = eng.real_def.cpu().numpy() if eng.real_def is not None else None
            fd = eng.fail_def.cpu().numpy() if eng.fail_def is not None else None
            ra = eng.real_atk.cpu().numpy() if eng.real_atk is not None else None
            fa = eng.fail_atk.cpu().numpy() if eng.fail_atk is not None else None
            st = eng.export_state()
            for b, o in enumerate(orc):
                if o._board.done():
                    continue  # finished in an earlier step (no auto-reset here)
                d_b = None if da is None else (da[b] if multi else int(da[b]))
                wo, wr, wd, info = o.step(d_b, None if aa is None else aa[b])
                tag = (mode, multi, difficulty, k, b)
                assert canon.fhex(rw[b]) == canon.fhex(wr), tag
                assert bool(dn[b]) == wd, tag
                assert canon.state_digest(eng.board_state(b, st)) == canon.state_digest(canon.oracle_state(o)), tag
                assert np.array_equal(ob[b], wo), (tag, np.argwhere(ob[b] != wo)[:5].tolist())
                w = info["Win"]
                if isinstance(w, dict):
                    w = w["Defender"] if mode != "atk" else w["Attacker"]
                assert (int(win[b]) if win[b] >= 0 else None) == (None if w is None else int(w)), tag
                assert (int(cdn[b]) & 15, int(cdn[b]) >> 4) == (min(o.attacker_cd, 15), min(o.defender_cd, 15)), tag
                anm = info["AllowNextMove"]
                if mode == "2p":
                    assert bool(an[b] & 1) == anm["Attacker"] and bool(an[b] & 2) == anm["Defender"], tag
                elif mode == "atk":
                    assert bool(an[b] & 1) == anm, tag
                else:
                    assert bool(an[b] & 2) == anm, tag
                real, fc = info["RealAction"], info["FailCode"]
                if mode == "def":
                    if multi:
                        assert np.array_equal(rd[b], real), tag
                    else:
                        assert int(rd[b]) == int(real) and int(fd[b]) == int(fc), tag
                elif mode == "atk":
                    assert np.array_equal(ra[b], real), tag
                    assert _fc_list(fa[b]) == list(fc), tag
                else:
                    if multi:
                        assert np.array_equal(ra[b], real["Attacker"]) and np.array_equal(rd[b], real["Defender"]), tag
                    else:
                        if isinstance(real, dict):  # no defender success this step
                            assert np.array_equal(ra[b], real["Attacker"]), tag
                            assert int(rd[b]) == L * L * 6, tag
                        else:  # TDMulti.py:257: the defender action replaced the dict
                            assert int(rd[b]) == int(real), tag
                        assert _fc_list(fa[b]) == fc["Attacker"] and int(fd[b]) == fc["Defender"], tag
        assert (eng.flags() == 0).all()
    finally:
        eng.close()


def _oracle_reset_skipping(env):
    """Auto-reset of the device: a failing layout draw (the reference raises or
    hangs) is skipped and the next draw of the same stream is taken."""
    skipped = 0
    while True:
        try:
            return env.reset(), skipped
        except O.RoadGenError:
            skipped += 1


def test_vecenv_autoreset_vs_oracle():
    """TDVecEnv with auto-reset over many short episodes (1-LP bases): the obs
    returned for a finished board is its next episode's first obs, episode
    return / length describe the finished episode, and failing layout draws are
    skipped exactly as the oracle skips them."""
    L, B, steps = 10, 96, 400
    ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.02)  # weak defence: ~5 episodes per board
    cfg = O.Config(**ov)
    seeds, orc = _first_ok_seeds(L, B, 4000, "def", False, 1, cfg)
    with reference_settings(ov, False):
        ve = E.TDVecEnv(L, B, "def", seed=0)
    eng = ve.engine
    eng.seed(np_seeds=seeds, py_seeds=seeds)
    try:
        obs = ve.reset().cpu().numpy()
        for b, o in enumerate(orc):
            assert np.array_equal(obs[b], o._board.get_states())
        rets = np.zeros(B)
        last = (np.zeros(B), np.zeros(B, np.int32), np.full(B, -1, np.int32))  # td_episode_records
        rng = np.random.RandomState(9)
        resets = skipped = 0
        for k in range(steps):
            acts = np.array([policies.discrete_def(rng, L) for o in orc], dtype=np.int64)
            obs_t, rew_t, done_t, infos = ve.step(torch.from_numpy(acts).cuda())
            ob, rw, dn = obs_t.cpu().numpy(), rew_t.cpu().numpy(), done_t.cpu().numpy()
            er, el = infos["episode_return"].cpu().numpy(), infos["episode_length"].cpu().numpy()
            for b, o in enumerate(orc):
                wo, wr, wd, winfo = o.step(int(acts[b]))
                rets[b] += wr
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                assert bool(dn[b]) == wd, (k, b)
                if wd:
                    assert canon.fhex(er[b]) == canon.fhex(rets[b]) and int(el[b]) == o._board.steps, (k, b)
                    last[0][b], last[1][b], last[2][b] = rets[b], o._board.steps, int(winfo["Win"])
                    rets[b] = 0.0
                    wo, s = _oracle_reset_skipping(o)
                    skipped += s
                    resets += 1
                assert np.array_equal(ob[b], wo), (k, b, np.argwhere(ob[b] != wo)[:5].tolist())
        assert resets > 3 * B  # several episodes per board
        assert skipped > 0, "no failing layout draw was exercised; widen the run"
        r_ret, r_len, r_win = eng.episode_records()
        assert [canon.fhex(v) for v in r_ret.cpu().numpy()] == [canon.fhex(v) for v in last[0]]
        assert r_len.cpu().numpy().tolist() == last[1].tolist()
        assert r_win.cpu().numpy().tolist() == last[2].tolist()
        assert (eng.flags() == 0).all()
    finally:
        ve.close()


@pytest.mark.parametrize("L,B,mode,difficulty,steps", [
    (10, 64, "def", 1, 400), (10, 48, "def", 0, 300), (10, 48, "atk", 2, 300), (20, 24, "atk", 1, 400)])
def test_vecenv_random_agent_false_autoreset(L, B, mode, difficulty, steps):
    """random_agent=False under auto-reset (TDGymBasic.py:87-89,101-103 in gym 0.21's
    AsyncVectorEnv, train/main.py:329-347): the built-in opponent draws from each board's
    layout stream and every finished board's next layout is drawn from that stream right
    after the step that ended the episode (td_autoreset_kernel), failing draws skipped.
    Against the oracle's random_agent=False branch, bit for bit, over many short
    episodes; the streams end where the oracle's end."""
    ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.02) if mode == "def" else dict(base_LP=1)
    cfg = O.Config(**ov)
    seeds, orc = _first_ok_seeds(L, B, 6000 + 13 * difficulty, mode, False, difficulty, cfg, random_agent=False)
    with reference_settings(ov, False):
        ve = E.TDVecEnv(L, B, mode, difficulty=difficulty, seed=0, random_agent=False)
    eng = ve.engine
    eng.seed(np_seeds=seeds, py_seeds=seeds)
    try:
        obs = ve.reset().cpu().numpy()
        for b, o in enumerate(orc):
            assert np.array_equal(obs[b], o._board.get_states())
        rng = np.random.RandomState(17 + L)
        resets = skipped = 0
        for k in range(steps):
            if mode == "def":
                acts = np.array([policies.discrete_def(rng, L) for o in orc], dtype=np.int64)
            else:
                acts = np.stack([policies.atk(rng) for _ in orc]).astype(np.int64)
            obs_t, rew_t, done_t, _ = ve.step(torch.from_numpy(acts).cuda())
            ob, rw, dn = obs_t.cpu().numpy(), rew_t.cpu().numpy(), done_t.cpu().numpy()
            st = eng.export_state()
            for b, o in enumerate(orc):
                if mode == "def":
                    wo, wr, wd, _ = o.step(int(acts[b]))
                else:
                    wo, wr, wd, _ = o.step(None, acts[b])
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                assert bool(dn[b]) == wd, (k, b)
                if wd:
                    wo, s = _oracle_reset_skipping(o)
                    skipped += s
                    resets += 1
                assert np.array_equal(ob[b], wo), (k, b, np.argwhere(ob[b] != wo)[:5].tolist())
                assert canon.state_digest(eng.board_state(b, st)) == canon.state_digest(canon.oracle_state(o)), (k, b)
        assert resets >= B // 3  # episodes end and auto-reset throughout the run
        assert (eng.flags() == 0).all()
        for b in range(0, B, max(1, B // 8)):
            ns = orc[b].np_random.get_state()
            assert eng.get_np_state(b).tolist() == list(ns[1]) + [int(ns[2])], b
    finally:
        ve.close()


def test_random_agent_false_refused_with_staged_layouts():
    """Layouts an auto-reset refill drew ahead of play would put the numpy stream out of
    the reference's order once the opponent draws from it: switching random_agent off is
    refused then, and allowed again after re-seeding the layout streams."""
    from gym_TD import _lib
    eng = TDEngine(10, 8, "def", False, 1, np_seeds=range(8), py_seeds=range(8), autoreset=True)
    try:
        eng.reset_all()
        torch.cuda.synchronize()
        with pytest.raises(_lib.TDError):
            _lib.check(_lib.lib.td_set_random_agent(eng._h, 0))
        eng.seed(np_seeds=range(8))
        _lib.check(_lib.lib.td_set_random_agent(eng._h, 0))
    finally:
        eng.close()


@pytest.mark.parametrize("mode,multi,shards", [("def", False, 2), ("2p", True, 2), ("def", False, 8)])
def test_vecenv_sharding_invariance(mode, multi, shards):
    """Board i of the global batch follows the same trajectory whether it is
    stepped in one TDVecEnv of 64 boards or in its shard of 64 / shards boards, as
    rank r of a `shards`-GPU run owns it (trajectories at 1 and 8
    GPUs are bit-identical)."""
    L, B, steps = 10, 64, 200
    n = B // shards
    with reference_settings({"base_LP": 2}, multi):
        whole = E.TDVecEnv(L, B, mode, seed=777)
        parts = [E.TDVecEnv(L, n, mode, seed=777, global_offset=r * n) for r in range(shards)]
    try:
        ow = whole.reset()
        op = torch.cat([p.reset() for p in parts])
        assert torch.equal(ow, op)
        assert whole.roadgen_failures == sum(p.roadgen_failures for p in parts)
        g = torch.Generator(device="cuda").manual_seed(3)
        for k in range(steps):
            if multi:
                d = torch.randint(0, 3, (B, 6, L, L), device="cuda", generator=g, dtype=torch.int64)
            else:
                d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            a = torch.randint(0, 5, (B, 3, 8), device="cuda", generator=g, dtype=torch.int64)
            act = (lambda lo, hi: d[lo:hi]) if mode == "def" else (lambda lo, hi: (d[lo:hi], a[lo:hi]))
            ow, rw, dw, iw = whole.step(act(0, B))
            res = [p.step(act(r * n, (r + 1) * n)) for r, p in enumerate(parts)]
            assert torch.equal(ow, torch.cat([r[0] for r in res])), k
            assert torch.equal(rw, torch.cat([r[1] for r in res])), k
            assert torch.equal(dw, torch.cat([r[2] for r in res])), k
            for key in ("episode_return", "episode_length", "Win"):
                assert torch.equal(iw[key], torch.cat([r[3][key] for r in res])), (k, key)
        sw = whole.engine.episode_stats().cpu().numpy()
        sp = sum(p.engine.episode_stats().cpu().numpy() for p in parts)
        assert sw[0] == sp[0] > 0
        assert sw[1] == pytest.approx(sp[1], rel=1e-12, abs=1e-9)
    finally:
        whole.close()
        for p in parts:
            p.close()


def test_reset_layouts_uses_caller_records():
    """td_reset_layouts: boards restart from caller-supplied layout records (here the
    host restatement's first draw of each board's stream) without touching the
    streams or the staged rings; the result equals a plain reset() of the same seeds."""
    from gym_TD.engine import generate_layout
    L, B = 10, 16
    seeds, _ = _first_ok_seeds(L, B, 5000, "def", False, 1)
    ref = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    try:
        want, failed = ref.reset()
        assert not failed
        want = want.clone()
        before = [eng.get_np_state(b).copy() for b in range(B)]
        recs = []
        for s in seeds:
            st = np.random.RandomState(s).get_state()
            w = np.array(list(st[1]) + [int(st[2])], dtype=np.uint32)
            status, rec = generate_layout(w, L)
            assert status == 0
            recs.append(rec)
        obs = eng.reset_layouts(np.stack(recs), np.arange(B))
        assert torch.equal(obs, want)
        for b in range(B):
            assert eng.get_np_state(b).tolist() == before[b].tolist()
            assert canon.state_digest(eng.board_state(b)) == canon.state_digest(ref.board_state(b))
        # both keep stepping identically (the same opponent streams, auto-reset from the rings)
        g = torch.Generator(device="cuda").manual_seed(11)
        for k in range(50):
            a = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            ref.step(def_act=a)
            eng.step(def_act=a)
            assert torch.equal(ref.obs, eng.obs) and torch.equal(ref.reward, eng.reward), k
    finally:
        ref.close()
        eng.close()


def test_export_import_roundtrip():
    """td_export_state / td_import_state carry a board's whole step state (lists,
    costs, cool-downs, map[6], the opponent stream): an engine loaded from another's
    export continues bit-identically."""
    L, B = 10, 24
    seeds, _ = _first_ok_seeds(L, B, 6000, "def", False, 1)
    a_eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    b_eng = TDEngine(L, B, "def", False, 1, np_seeds=[s + 1 for s in seeds], py_seeds=[s + 7 for s in seeds],
                     autoreset=False)
    try:
        a_eng.reset()
        b_eng.reset()
        rng = np.random.RandomState(4)
        for k in range(120):
            a_eng.step(def_act=torch.from_numpy(rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64)))
        b_eng.import_state(a_eng.export_state())
        for b in range(B):
            assert canon.state_digest(b_eng.board_state(b)) == canon.state_digest(a_eng.board_state(b))
        for k in range(120):
            act = torch.from_numpy(rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64))
            a_eng.step(def_act=act)
            b_eng.step(def_act=act)
            assert torch.equal(a_eng.obs, b_eng.obs) and torch.equal(a_eng.reward, b_eng.reward), k
            assert torch.equal(a_eng.done, b_eng.done), k
    finally:
        a_eng.close()
        b_eng.close()


def test_step_kernel_selector():
    """td_set_step_kernel: every kind at L = 10 / 20 / 30, named as rocprofv3 names the
    kernel; a small kernel at an L without one is refused and changes nothing."""
    from gym_TD import _lib
    for L in (10, 20, 30):
        eng = TDEngine(L, 4, "def", False, 1, np_seeds=[1, 2, 3, 4], py_seeds=[1, 2, 3, 4])
        try:
            for k, name in (("large", "td_step_kernel<"), ("small", "td_step_kernel_small<"),
                            ("small2", "td_step_kernel_small2<")):
                eng.set_step_kernel(k)
                assert eng.step_kernel == k and eng.step_kernel_name == "%s%d, 0, false>" % (name, L)
            eng.set_step_kernel("auto")
            assert eng.step_kernel == "small2"  # 4 boards: half a round of waves or less
        finally:
            eng.close()
    eng = TDEngine(12, 4, "2p", True, 1, np_seeds=[1, 2, 3, 4], py_seeds=[1, 2, 3, 4])
    try:
        assert eng.step_kernel == "large" and eng.step_kernel_name == "td_step_kernel<0, 2, true>"
        with pytest.raises(_lib.TDError, match="no small-batch"):
            eng.set_step_kernel("small")
        assert eng.step_kernel == "large"
    finally:
        eng.close()


def test_import_refuses_records_without_captured_fields():
    """A state record whose max_cost / max_base_LP (TdHdr, captured at reset: TDBoard.py:66-72)
    are zero -- a record of an older header format, or a hand-built one -- would clamp every
    cost to 0 and divide the scalar observation channels by zero: td_import_state refuses
    it and changes nothing.  Boards never reset (no layout) carry no such fields."""
    from gym_TD import _lib
    L, B = 10, 8
    seeds, _ = _first_ok_seeds(L, B, 6100, "def", False, 1)
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        eng.reset()
        good = eng.export_state()
        before = [canon.state_digest(eng.board_state(b)) for b in range(B)]
        for field, value in (("max_cost", 0.0), ("max_base_LP", 0), ("format", 0), ("n_en", 129)):
            st = {k: np.array(v, copy=True) for k, v in good.items()}
            st["hdr"][3][field] = value
            with pytest.raises(_lib.TDError, match="board 3"):
                eng.import_state(st)
            assert [canon.state_digest(eng.board_state(b)) for b in range(B)] == before, field
        # a never-reset board (zero header, num_roads 0) imports as it is
        st = {k: np.array(v, copy=True) for k, v in good.items()}
        st["hdr"][5] = np.zeros(1, dtype=st["hdr"].dtype)[0]
        eng.import_state(st)
        assert eng.board_state(5)["num_roads"] == 0
        eng.import_state(good)
        assert [canon.state_digest(eng.board_state(b)) for b in range(B)] == before
    finally:
        eng.close()


def test_config_epochs_recycled_past_256():
    """paramConfig every step for 300 steps (a curriculum): the device has 256 constant
    blocks, so after 255 changes td_set_config recycles blocks no live enemy or tower
    refers to (td_cfg_usage_kernel).  Every entity must keep the values it captured
    (TDElements.py:4-43, 134-170) -- bit-exact against the oracle through the recycling.
    Then, with 256 epochs each held by a live tower, one more td_set_config fails cleanly
    and leaves the current config in place."""
    from gym_TD import _lib
    from gym_TD import params as P
    L, B = 10, 16
    # phase 1: a builder defender that stays under the 32-tower cap ((150 + 0.5 * 300) / 10 = 30 towers
    # at most); phase 2: explicit builds, one tower per board every 16 steps
    rich = dict(tower_distance=0, defender_init_cost=400, max_cost=400, defender_cost_rate=2)
    base = dict(rich, defender_init_cost=150, defender_cost_rate=0.5)

    def cfg_at(k, into):
        for key, v in base.items():
            setattr(into, key, copy.deepcopy(v))
        into.reward_time = 0.001 + k * 1e-6  # every step's config is distinct
        into.enemy_LP = [[820 + 10 * (k % 11), 1700], [2050, 3000 + 7 * (k % 5)], [6000, 8000], [8000 - 3 * (k % 9), 12000]]
        into.enemy_defense = [[k % 3, 0], [200 + k % 7, 250], [600, 800], [80, 100]]
        into.enemy_speed = [[.25, .25], [.13 + .01 * (k % 2), .13], [.1, .1], [.1, .1]]
        into.tower_attack = [[454 + k % 13, 540], [651, 771 + k % 4], [566 + k % 6, 691], [358, 424]]
        into.tower_range = [[3 + k % 2, 3], [2, 2], [4, 4], [3, 3]]
        return into

    cfg0 = cfg_at(0, O.Config())
    seeds, orc = _first_ok_seeds(L, B, 6200, "def", False, 1, cfg0)
    dcfg = cfg_at(0, copy.deepcopy(P.config))
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False, cfg=dcfg)
    try:
        eng.reset()
        rng = np.random.RandomState(31)
        seen = []
        for k in range(1, 301):
            eng.set_config(cfg_at(k, copy.deepcopy(P.config)))
            seen.append(_lib.lib.td_config_epoch(eng._h))
            for o in orc:
                cfg_at(k, o.cfg)
            acts = np.array([policies.discrete_def(rng, L, o._board.map[0], 0.7) for o in orc], dtype=np.int64)
            eng.step(def_act=torch.from_numpy(acts))
            ob, rw = eng.obs.cpu().numpy(), eng.reward.cpu().numpy()
            st = eng.export_state()
            for b, o in enumerate(orc):
                if o._board.done():
                    continue
                wo, wr, _, _ = o.step(int(acts[b]))
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                mine, want = eng.board_state(b, st), canon.oracle_state(o)
                assert canon.state_digest(mine) == canon.state_digest(want), (k, b, mine, want)
                assert np.array_equal(ob[b], wo), (k, b, np.argwhere(ob[b] != wo)[:5].tolist())
        assert len(set(seen)) == 256 and len(seen) == 300  # blocks were recycled
        assert (eng.flags() == 0).all()  # no board reached the tower / enemy caps
    finally:
        eng.close()
    base = rich
    # all 256 blocks held by live towers: one tower per config epoch, board k % 16 building at step k
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False, cfg=dcfg)
    try:
        eng.reset()
        st = eng.export_state()
        free = [[c for c in range(L * L) if (int(st["cells"][b][c]) >> 24) == 0] for b in range(B)]
        empty = 6 * L * L
        for k in range(256):
            eng.set_config(cfg_at(1000 + k, copy.deepcopy(P.config)))
            acts = np.full(B, empty, dtype=np.int64)
            acts[k % B] = free[k % B][k // B]  # op 0 (arrow) at a free cell
            eng.step(def_act=torch.from_numpy(acts))
            assert int(eng.fail_def[k % B]) == 0, k
        st = eng.export_state()
        held = {(int(u) >> 16) & 0xFF for b in range(B) for u in st["tw_inf"][b][:int(st["hdr"][b]["n_tw"])]}
        assert len(held) == 256
        ep = _lib.lib.td_config_epoch(eng._h)
        with pytest.raises(_lib.TDError, match="still referenced"):
            eng.set_config(cfg_at(5000, copy.deepcopy(P.config)))
        assert _lib.lib.td_config_epoch(eng._h) == ep
        eng.step(def_act=torch.full((B,), empty, dtype=torch.int64))  # the engine keeps stepping
        assert (eng.flags() == 0).all()
    finally:
        eng.close()


def test_export_import_roundtrip_random_agent_false():
    """With random_agent=False the built-in opponent draws from the board's numpy layout
    stream, which td_export_state does not carry (include/tdstep.h): a snapshot is the
    export plus get_np_state per board.  Restored into an engine with other seeds, the
    boards continue bit-identically -- opponent moves, rewards, and the layouts of the
    resets that follow."""
    L, B = 10, 16
    seeds, _ = _first_ok_seeds(L, B, 6100, "def", False, 1)
    mk = lambda s, off: TDEngine(L, B, "def", False, 1, np_seeds=[x + off for x in s], py_seeds=[x + off for x in s],
                                 autoreset=False, random_agent=False)
    a_eng, b_eng = mk(seeds, 0), mk(seeds, 3)
    try:
        a_eng.reset()
        b_eng.reset()
        rng = np.random.RandomState(5)
        for k in range(150):
            a_eng.step(def_act=torch.from_numpy(rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64)))
        b_eng.import_state(a_eng.export_state())
        for b in range(B):
            b_eng.set_np_state(b, a_eng.get_np_state(b))
            assert canon.state_digest(b_eng.board_state(b)) == canon.state_digest(a_eng.board_state(b))
        for k in range(150):
            act = torch.from_numpy(rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64))
            a_eng.step(def_act=act)
            b_eng.step(def_act=act)
            assert torch.equal(a_eng.obs, b_eng.obs) and torch.equal(a_eng.reward, b_eng.reward), k
            assert torch.equal(a_eng.done, b_eng.done), k
        # the next episodes' layouts come from the same restored streams
        oa, fa = a_eng.reset()
        ob, fb = b_eng.reset()
        assert list(fa) == list(fb) and torch.equal(oa, ob)
        for b in range(B):
            assert a_eng.get_np_state(b).tolist() == b_eng.get_np_state(b).tolist()
    finally:
        a_eng.close()
        b_eng.close()


@pytest.mark.parametrize("kernel", ("large", "small", "small2"))
def test_paramconfig_reaches_live_engines(kernel):
    """paramConfig (TDParam.py:98-100) in the middle of episodes, twice, on a live engine.
    The reference reads most values live from `config`, but an Enemy / Tower keeps the
    stats it was created or upgraded with (TDElements.py:4-69, 134-170: maxLP, speed,
    defense; atk, rge, dmgrge, intv, cost) and a TDBoard the max_cost / base_LP of its
    reset (TDBoard.py:66-72).  The device keeps one constant block per config epoch and
    tags entities with theirs: bit-exact against the oracle (whose Enemy / Tower objects
    capture like the reference's) through both changes and a reset of half the boards."""
    import gym_TD
    from gym_TD import params as P
    L, B = 10, 16
    ov1 = dict(reward_time=0.004, tower_range=[[4, 4], [3, 3], [5, 5], [4, 4]],
               enemy_speed=[[.2, .2], [.2, .2], [.15, .15], [.1, .1]], enemy_LP=[[600, 1500], [1500, 2500],
               [5000, 7000], [7000, 9000]], enemy_defense=[[10, 10], [150, 200], [500, 700], [60, 90]],
               tower_attack=[[500, 600], [700, 800], [600, 700], [400, 450]], max_cost=60, base_LP=7,
               tower_attack_interval=[[3, 3], [5, 5], [6, 6], [4.5, 4.5]], defender_cost_rate=0.5)
    ov2 = dict(tower_cost=[[8, 9], [15, 16], [20, 21], [11, 12]], tower_splash_range=[[0, 0], [0, 0], [2, 2], [1, 1]],
               frozen_ratio=0.3, tower_destruct_return=0.75, enemy_speed=[[.3, .3], [.15, .15], [.12, .12], [.1, .1]],
               max_cost=150, attacker_cost_final_rate=1.5)
    seeds, orc = _first_ok_seeds(L, B, 7000, "def", False, 1)
    saved = {k: copy.deepcopy(getattr(P.config, k)) for k in set(ov1) | set(ov2)}
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False, step_kernel=kernel)
    try:
        eng.reset()
        rng = np.random.RandomState(8)
        epochs = set()
        for k in range(160):
            if k in (30, 70):
                ov = ov1 if k == 30 else ov2
                gym_TD.paramConfig(**ov)  # re-uploads the live engine's config (a new epoch)
                for o in orc:
                    for key, v in ov.items():
                        setattr(o.cfg, key, copy.deepcopy(v))
            if k == 110:  # half the boards start a new episode: they capture the new max_cost / base_LP
                m = np.zeros(B, np.uint8)
                m[::2] = 1
                _, failed = eng.reset(m)
                while failed:  # the reference raises on these draws: both sides draw again
                    m[:] = 0
                    m[failed] = 1
                    _, failed = eng.reset(m)
                for b in range(0, B, 2):
                    _oracle_reset_skipping(orc[b])
            acts = np.array([policies.discrete_def(rng, L, o._board.map[0], 0.6) for o in orc], dtype=np.int64)
            eng.step(def_act=torch.from_numpy(acts))
            ob, rw = eng.obs.cpu().numpy(), eng.reward.cpu().numpy()
            st = eng.export_state()
            for b, o in enumerate(orc):
                if o._board.done():
                    continue
                wo, wr, _, _ = o.step(int(acts[b]))
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                assert canon.state_digest(eng.board_state(b, st)) == canon.state_digest(canon.oracle_state(o)), (k, b)
                assert np.array_equal(ob[b], wo), (k, b, np.argwhere(ob[b] != wo)[:5].tolist())
            for b in range(B):
                n, nt = int(st["hdr"][b]["n_en"]), int(st["hdr"][b]["n_tw"])
                epochs |= {int(u) >> 24 for u in st["en_inf"][b][:n]} | {int(u) >> 24 for u in st["tw_inf"][b][:nt]}
        assert len(epochs) >= 2  # entities of different config epochs lived side by side
        # the drop-in view shows each entity's captured values
        view = E.TDBoardView(eng, 1)
        for e in view.enemies:
            w = [x for x in orc[1]._board.enemies if x.loc == e.loc and x.type == e.type and x.LP == e.LP]
            assert w and w[0].maxLP == e.maxLP and w[0].speed == e.speed and w[0].defense == e.defense
        assert view.max_cost == orc[1]._board.max_cost and view.max_base_LP == orc[1]._board.max_base_LP
    finally:
        gym_TD.paramConfig(**saved)
        eng.close()


def test_capacity_overflow_is_flagged():
    """A config that summons past the 128-enemy cap (SURVEY a12 bounds the default
    config at 121) sets FLAG_EN_OVERFLOW and refuses the extra summons instead of
    corrupting the board."""
    from test_gpu_parity import reference_settings
    L, B = 10, 4
    ov = dict(attacker_init_cost=200, max_cost=200, enemy_cost=[[1, 1], [1, 1], [1, 1], [1, 1]],
              enemy_speed=[[.01, .01], [.01, .01], [.01, .01], [.01, .01]], defender_init_cost=0, defender_cost_rate=0)
    seeds, _ = _first_ok_seeds(L, B, 8000, "def", False, 1)
    with reference_settings(ov, False):
        eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        eng.reset()
        empty = torch.full((B,), 6 * L * L, dtype=torch.int64, device="cuda")
        for k in range(40):
            eng.step(def_act=empty)
        fl = eng.flags()
        assert (fl & 1).all(), fl
        for b in range(B):
            assert len(eng.board_state(b)["enemies"]) == 128
        assert bool(torch.isfinite(eng.obs).all())  # count/8 planes exceed 1 here, as in the reference
    finally:
        eng.close()


def _obs_checksum(obs):
    """Per-board checksum of the observation bits (two int64 sums), on the device."""
    w = obs.flatten(1).view(torch.int32).to(torch.int64)
    idx = torch.arange(1, w.shape[1] + 1, device=w.device, dtype=torch.int64)
    return torch.stack([w.sum(1), (w * idx).sum(1)], 1)


@pytest.mark.parametrize("B,steps,kernel,refill", [
    (16384, 200, "large", 16), (512, 1500, "small2", 16), (8192, 400, "small", 16), (4096, 300, "large", 16),
    (16384, 200, "large", 0), (8192, 400, "small", 0), (4096, 300, "small2", 0)])
def test_autoreset_under_load_matches_explicit_reset(B, steps, kernel, refill):
    """The staged-layout rings under load: 16,384 boards with 1-LP bases and a weak
    defence finish ~250 episodes per step; 512 boards step so fast that one draw
    the reference never finishes (2-5 ms of one lane) spans hundreds of steps.
    Phase 1 runs the auto-reset engine 200
    steps back to back with no host synchronisation, so the refill kernel publishes
    layouts while step grids consume them; per-step observation checksums, rewards
    and dones stay on the device.  Phase 2 replays the same actions on an engine
    reset explicitly (the reset kernel draws each layout on the spot, failing draws
    skipped as the refill skips them).  Every board must agree at every step, on each
    step kernel (8,192 boards: the N = 8 share's kernel).  refill = 0: no refill kernel at
    all -- every layout comes from the ring guard on the step stream (td_refill_kernel with
    guard = 15 = NSLOT - 1: before every 15th step it fills every ring below 15 layouts to
    15), so an episode end never depends on the refill cadence."""
    from test_gpu_parity import reference_settings
    L = 10
    ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.02)
    seeds = np.arange(B, dtype=np.int64) + 20000
    with reference_settings(ov, False):
        ea = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, step_kernel=kernel)
        eb = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        ea.set_refill_interval(refill)
        ea.reset_all()
        eb.reset_all()
        assert torch.equal(ea.obs, eb.obs)
        g = torch.Generator(device="cuda").manual_seed(21)
        acts = torch.randint(0, 6 * L * L + 1, (steps, B), device="cuda", generator=g, dtype=torch.int64)
        hist = []
        for k in range(steps):  # phase 1: asynchronous
            ea.step(def_act=acts[k])
            hist.append((_obs_checksum(ea.obs), ea.reward.clone(), ea.done.clone()))
        torch.cuda.synchronize()
        resets = 0
        for k in range(steps):  # phase 2: explicit resets
            eb.step(def_act=acts[k])
            cs, rw, dn = hist[k]
            assert torch.equal(rw, eb.reward) and torch.equal(dn, eb.done), k
            d = eb.done.cpu().numpy().astype(bool)
            if d.any():
                resets += int(d.sum())
                _, failed = eb.reset(d)
                while failed:
                    m = np.zeros(B, dtype=np.uint8)
                    m[failed] = 1
                    _, failed = eb.reset(m)
            bad = torch.nonzero((cs != _obs_checksum(eb.obs)).any(1)).flatten()
            assert bad.numel() == 0, (k, bad[:8].tolist())
        assert resets > steps * B // 100
        assert (ea.flags() == 0).all()
    finally:
        ea.close()
        eb.close()


@pytest.mark.parametrize("kernel", ("large", "small", "small2"))
def test_many_towers_vs_oracle(kernel):
    """Boards with more towers than the step prefetches up front (16): tower distance
    1, rich defender.  Same bit-exact comparison as the batched tests."""
    from test_gpu_parity import reference_settings
    L, B, steps = 10, 12, 120
    ov = dict(tower_distance=1, defender_init_cost=300, max_cost=400, defender_cost_rate=5)
    cfg = O.Config(**ov)
    seeds, orc = _first_ok_seeds(L, B, 9000, "def", False, 1, cfg)
    with reference_settings(ov, False):
        eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False, step_kernel=kernel)
    try:
        eng.reset()
        rng = np.random.RandomState(12)
        most = 0
        for k in range(steps):
            acts = np.array([policies.discrete_def(rng, L, o._board.map[0], 0.9) for o in orc], dtype=np.int64)
            eng.step(def_act=torch.from_numpy(acts))
            ob, rw = eng.obs.cpu().numpy(), eng.reward.cpu().numpy()
            st = eng.export_state()
            for b, o in enumerate(orc):
                if o._board.done():
                    continue
                wo, wr, _, _ = o.step(int(acts[b]))
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                assert canon.state_digest(eng.board_state(b, st)) == canon.state_digest(canon.oracle_state(o)), (k, b)
                assert np.array_equal(ob[b], wo), (k, b)
                most = max(most, len(o._board.towers))
        assert most > 16, most
        assert (eng.flags() == 0).all()
    finally:
        eng.close()


def _norm_info(info):
    def n(v):
        if isinstance(v, dict):
            return {k: n(x) for k, x in v.items()}
        if isinstance(v, (list, tuple)):
            return [n(x) for x in v]
        if isinstance(v, np.ndarray):
            return v.astype(np.int64).tolist()
        if isinstance(v, (np.integer,)):
            return int(v)
        if isinstance(v, np.bool_):
            return bool(v)
        return v
    return n({k: info[k] for k in ("RealAction", "Win", "AllowNextMove", "FailCode")})


@pytest.mark.parametrize("env_id,difficulty", [("TD-def-small-v0", 1), ("TD-atk-small-v0", 2), ("TD-2p-small-v0", 1)])
def test_async_vector_env_surface(env_id, difficulty):
    """gym_TD.vector.VectorEnv answers train/main.py's AsyncVectorEnv calls: numpy
    obs / rewards / dones and one info dict per env, equal to N oracle envs with
    auto-reset (failing layout draws skipped on both sides)."""
    from gym_TD.vector import VectorEnv
    kind = env_id.split("-")[1]
    L, N, steps = 10, 12, 150
    ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.05)
    S = None
    for s0 in range(2000, 2400, 16):
        try:
            orc = [O.Env(L, G.MODES[kind], difficulty, s0 + i, s0 + i, O.Config(**ov), O.Hyper(), road_attempts=1000)
                   for i in range(N)]
            S = s0
            break
        except O.RoadGenError:
            continue
    assert S is not None
    with reference_settings(ov, False):
        ve = VectorEnv(env_id, N, difficulty=difficulty, seed=S)
    try:
        assert len(ve.env_fns) == N
        obs = ve.reset()
        assert isinstance(obs, np.ndarray) and obs.shape == (N, 45, L, L)
        for i, o in enumerate(orc):
            assert np.array_equal(obs[i], o._board.get_states())
        rng = np.random.RandomState(5)
        for k in range(steps):
            da = [policies.discrete_def(rng, L, o._board.map[0], 0.3) for o in orc] if kind != "atk" else None
            aa = [policies.atk(rng) for _ in orc] if kind != "def" else None
            if kind == "def":
                act = np.array(da, dtype=np.int64)
            elif kind == "atk":
                act = np.stack(aa)
            else:
                act = {"Defender": np.array(da, dtype=np.int64), "Attacker": np.stack(aa)}
            obs, rew, done, infos = ve.step(act)
            assert isinstance(infos, tuple) and len(infos) == N
            for i, o in enumerate(orc):
                wo, wr, wd, winfo = o.step(None if da is None else da[i], None if aa is None else aa[i])
                assert canon.fhex(rew[i]) == canon.fhex(wr), (k, i)
                assert bool(done[i]) == wd, (k, i)
                assert _norm_info(infos[i]) == _norm_info(winfo), (k, i, infos[i], winfo)
                if wd:
                    wo, _ = _oracle_reset_skipping(o)
                assert np.array_equal(obs[i], wo), (k, i)
    finally:
        ve.close()


@pytest.mark.parametrize("env_cls,mode,calls", [
    ("TDMulti", "2p", ("random_tower_lv1", "random_enemy_lv1")),   # demo.py:72-80 play_2p
    ("TDMulti", "2p", ("random_tower_lv2", "random_enemy_lv0")),
    ("TDDefense", "def", ("random_tower_lv0",)),
    ("TDAttack", "atk", ("random_enemy_lv1",)),
])
def test_opponent_methods_called_directly(env_cls, mode, calls):
    """TDGymBasic's built-in opponents called by the caller between steps (demo.py:78-79),
    then step(empty_action()): bit-exact with the oracle env making the same calls."""
    L, seed, opp = 10, 31, 77
    cls = getattr(E, env_cls)
    kw = dict(seed=seed, opponent_seed=opp)
    if mode != "2p":
        kw["difficulty"] = 1
    env = cls(L, **kw)
    orc = O.Env(L, G.MODES[mode], 1, seed, opp, O.Config(), O.Hyper(), road_attempts=10000)
    try:
        for k in range(200):
            for name in calls:
                getattr(env, name)()
                getattr(orc, name)()
            obs, r, d, _ = env.step(env.empty_action())
            e = orc.empty_def() if mode != "atk" else None
            a = orc.empty_atk() if mode != "def" else None
            wo, wr, wd, _ = orc.step(e, a)
            assert canon.fhex(r) == canon.fhex(wr), (k, r, wr)
            assert canon.state_digest(env._engine.board_state(0)) == canon.state_digest(canon.oracle_state(orc)), k
            assert np.array_equal(obs, wo), (k, np.argwhere(obs != wo)[:5].tolist())
            assert d == wd, k
            if d:
                break
    finally:
        env.close()


def test_board_view_and_errors():
    """env._board mirrors TDBoard's attributes (TDBoard.py:25-79) after play, and the
    surface raises where the reference raises (invalid action: AssertionError,
    TDDefense.py:36) or where an option is not provided."""
    L, seed, opp = 10, 31, 77
    env = E.TDDefense(L, seed=seed, opponent_seed=opp)
    orc = O.Env(L, O.MODE_DEF, 1, seed, opp, O.Config(), O.Hyper(), road_attempts=10000)
    try:
        rng = np.random.RandomState(2)
        for k in range(120):
            a = policies.discrete_def(rng, L, orc._board.map[0], 0.6)
            env.step(a)
            orc.step(a)
        v, w = env._board, orc._board
        assert np.array_equal(v.map, w.map)
        assert v.start == [list(s) for s in w.start] and v.end == list(w.end)
        assert (v.cost_def, v.cost_atk, v.base_LP, v.steps) == (w.cost_def, w.cost_atk, w.base_LP, w.steps)
        assert v.progress == w.progress
        assert [(e.type, e.lv, e.loc, e.LP, e.margin, e.slowdown, e.dist) for e in v.enemies] == \
            [(e.type, e.lv, list(e.loc), e.LP, e.margin, e.slowdown, e.dist) for e in w.enemies]
        assert [(t.type, t.lv, t.loc, t.cd, t.intv, t.cost, t.atk, t.rge) for t in v.towers] == \
            [(t.type, t.lv, list(t.loc), t.cd, t.intv, t.cost, t.atk, t.rge) for t in w.towers]
        assert len(w.towers) > 0
        assert np.array_equal(v.get_states(), w.get_states())
        with pytest.raises(AssertionError):
            env.step(6 * L * L + 1)
        with pytest.raises(Exception):
            env._engine.opponent("tower", 3)
    finally:
        env.close()
    from gym_TD.vector import VectorEnv
    with pytest.raises(NotImplementedError):
        VectorEnv("TD-def-small-v0", 4, seed=0, fixed_seed=True)


@pytest.mark.parametrize("cls,mode,L,difficulty,steps", [
    ("TDDefense", "def", 10, 0, 1300), ("TDDefense", "def", 10, 1, 1300),
    ("TDAttack", "atk", 10, 0, 300), ("TDAttack", "atk", 10, 1, 400), ("TDAttack", "atk", 20, 2, 300)])
def test_random_agent_false_vs_oracle(cls, mode, L, difficulty, steps):
    """random_agent=False (TDGymBasic.py:87-289): the built-in opponents draw from the
    env's numpy layout stream, interleaved with reset()'s layout draws, except the
    destruct branch's tower index (CPython random, :191, :287).  Checked bit-exactly
    against the oracle's restatement of that branch over episodes and resets (the
    reference itself was not run for this mode: parity unpinned)."""
    rng = np.random.RandomState(L + difficulty)
    seed, opp = 300 + 17 * difficulty + L, 900 + difficulty
    while True:
        try:
            orc = O.Env(L, G.MODES[mode], difficulty, seed, opp, O.Config(), O.Hyper(), random_agent=False,
                        road_attempts=ROAD_ATTEMPTS)
            break
        except O.RoadGenError:
            seed += 1
    env = getattr(E, cls)(L, difficulty=difficulty, seed=seed, opponent_seed=opp, random_agent=False)
    try:
        assert np.array_equal(env._obs, orc._board.get_states())
        resets, ended, road_fail = 0, False, False
        for k in range(steps):
            if mode == "def":
                a = policies.discrete_def(rng, L, orc._board.map[0], 0.6)
                wo, wr, wd, wi = orc.step(a, None)
            else:
                a = policies.atk(rng)
                wo, wr, wd, wi = orc.step(None, a)
            o, r, d, info = env.step(a)
            assert canon.fhex(r) == canon.fhex(wr), k
            assert np.array_equal(o, wo), k
            assert d == bool(wd), k
            # the env's cool-down attributes (TDDefense.py:38-39,75; TDAttack.py:31-32,44)
            assert (env.attacker_cd, env.defender_cd) == (orc.attacker_cd, orc.defender_cd), k
            if d:
                ended = True
                try:
                    wo = orc.reset()
                except O.RoadGenError:
                    with pytest.raises(RuntimeError):
                        env.reset()
                    road_fail = True
                    break
                assert np.array_equal(env.reset(), wo), k
                resets += 1
        if not road_fail:
            assert env._engine.get_np_state(0)[:625].tolist() == list(orc.np_random.get_state()[1]) + \
                [orc.np_random.get_state()[2]]
        # TD-def episodes run to max_episode_steps (1200) against a random defender
        assert ended or mode == "atk"
    finally:
        env.close()
