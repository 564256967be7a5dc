"""GPU parity: the HIP step (through the C-ABI) against the reference's golden
vectors and the CPU oracle, bit-exact (rewards, state, observation bytes)."""
import contextlib

import numpy as np
import pytest
import torch

import goldens as G
from oracle import canon, policies
from oracle import td_oracle as O

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

import gym_TD  # noqa: E402
from gym_TD import envs as E  # noqa: E402
from gym_TD import params as P  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

from test_oracle_golden import _info_view  # noqa: E402

# The three step kernels (td_set_step_kernel): the large-batch kernel (20x20 / 30x30
# batches beyond a few rounds of waves), the one-round kernel of the N = 8 share (8,192
# boards), the two-wave kernel of the metric's 65,536 boards and configs[1] (4,096).  Every parity test below runs each of them.
KERNELS = ("large", "small", "small2")


@contextlib.contextmanager
def reference_settings(overrides, multi):
    saved = {k: (v if not isinstance(v, list) else [list(x) for x in v]) for k, v in P.config.__dict__.items()}
    saved_multi = P.hyper_parameters.allow_multiple_actions
    try:
        for k, v in overrides.items():
            setattr(P.config, k, v)
        object.__setattr__(P.hyper_parameters, "allow_multiple_actions", bool(multi))
        yield
    finally:
        for k, v in saved.items():
            setattr(P.config, k, v)
        object.__setattr__(P.hyper_parameters, "allow_multiple_actions", saved_multi)


def _make_env(tr):
    cls = {"def": E.TDDefense, "atk": E.TDAttack, "2p": E.TDMulti}[tr["mode"]]
    kw = dict(seed=tr["seed"], opponent_seed=tr["opp_seed"])
    if tr["mode"] != "2p":
        kw["difficulty"] = tr["difficulty"]
    return cls(tr["L"], **kw)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", G.traj_names())
def test_device_replays_golden(name, kernel):
    tr = G.load_traj(name)
    L = tr["L"]
    with reference_settings(tr["overrides"], tr["multi"]):
        env = _make_env(tr)
        try:
            env._engine.set_step_kernel(kernel)
            assert env._engine.step_kernel == kernel
            rep = G.replay_oracle(tr)
            _, init, _ = next(rep)
            st = env._engine.board_state(0)
            m, start, end = env._engine.map_planes(0)
            assert canon.layout_digest(m, start, end) == init["lay"]
            assert env.num_roads == init["nr"]
            # the cool-downs are env attributes in the reference; the device keeps them in the board header
            assert canon.state_digest(st) == init["s"]
            assert canon.obs_digest(env._obs) == init["o"]
            for i, rec, got in rep:
                if "reset_error" in rec:
                    with pytest.raises(RuntimeError):
                        env.reset()
                    break
                if "reset" in rec:
                    o = env.reset()
                    m, start, end = env._engine.map_planes(0)
                    assert canon.layout_digest(m, start, end) == rec["lay"], (name, i)
                    assert canon.obs_digest(o) == rec["o"], (name, i)
                    assert canon.state_digest(env._engine.board_state(0)) == rec["s"], (name, i)
                    continue
                k = got["_k"]
                if tr["mode"] == "def":
                    act = got["_da"]
                elif tr["mode"] == "atk":
                    act = got["_aa"]
                else:
                    act = {"Attacker": got["_aa"], "Defender": got["_da"]}
                obs, r, d, info = env.step(act)
                st = env._engine.board_state(0)
                if canon.state_digest(st) != rec["s"] or canon.obs_digest(obs) != rec["o"] or canon.fhex(r) != rec["r"]:
                    want = canon.oracle_state(got["_env"])
                    bad = np.argwhere(obs != got["_obs"])
                    pytest.fail("%s step %d: reward %s vs %s\nwant %r\nhave %r\nobs diff %r" % (
                        name, k, canon.fhex(r), rec["r"], want, st, bad[:10].tolist()))
                assert int(d) == rec["d"], (name, k)
                if "info" in rec:
                    assert _info_view(info) == rec["info"], (name, k, _info_view(info), rec["info"])
                assert st["flags"] == 0
        finally:
            env.close()


def _oracle_envs(L, seeds, mode="def", multi=False, difficulty=1):
    hp = O.Hyper(allow_multiple_actions=multi)
    return [O.Env(L, G.MODES[mode], difficulty, int(s), int(s), O.Config(), hp, road_attempts=20000) for s in seeds]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("L,B,steps", [(10, 95, 260), (20, 32, 160), (30, 16, 120)])
def test_batched_vs_oracle(L, B, steps, kernel):
    """B boards in one launch vs B oracle envs, random + smart defender actions (an odd
    batch at 10x10)."""
    seeds = [s for s in range(1000, 1000 + 3 * B) if L > 10 or s not in (1045,)]
    orc, ok = [], []
    for s in seeds:
        try:
            orc.append(_oracle_envs(L, [s])[0])
            ok.append(s)
        except O.RoadGenError:
            pass
        if len(ok) == B:
            break
    eng = TDEngine(L, B, "def", False, 1, np_seeds=ok, py_seeds=ok, autoreset=False, step_kernel=kernel)
    try:
        assert eng.step_kernel == kernel
        obs, failed = eng.reset()
        assert not failed
        rng = np.random.RandomState(L)
        for k in range(steps):
            acts = np.array([policies.discrete_def(rng, L, o._board.map[0], 0.5) for o in orc], dtype=np.int64)
            eng.step(def_act=torch.from_numpy(acts))
            want = [o.step(int(a)) for o, a in zip(orc, acts)]
            ob = eng.obs.cpu().numpy()
            rw = eng.reward.cpu().numpy()
            dn = eng.done.cpu().numpy()
            st = eng.export_state()
            for b in range(B):
                wo, wr, wd, _ = want[b]
                assert canon.fhex(rw[b]) == canon.fhex(wr), (L, k, b)
                assert canon.state_digest(eng.board_state(b, st)) == canon.state_digest(canon.oracle_state(orc[b])), (L, k, b)
                assert np.array_equal(ob[b], wo), (L, k, b, np.argwhere(ob[b] != wo)[:5].tolist())
                assert bool(dn[b]) == wd
        assert (eng.flags() == 0).all()
        # both RNG streams end where the reference's would (lazy twist completed on export)
        import random
        for b in range(0, B, max(1, B // 8)):
            # the device may have pre-drawn past CPython's block boundary: compare the streams
            mine, ref = random.Random(), random.Random()
            mine.setstate((3, tuple(int(v) for v in eng.get_py_state(b)), None))
            ref.setstate(orc[b].rnd.getstate())
            assert [mine.getrandbits(32) for _ in range(700)] == [ref.getrandbits(32) for _ in range(700)], (L, b)
            ns = orc[b].np_random.get_state()
            assert eng.get_np_state(b).tolist() == list(ns[1]) + [int(ns[2])], (L, b)
    finally:
        eng.close()


def test_autoreset_matches_explicit_reset():
    """Auto-reset obs == the obs of an explicit reset on the same streams, and
    episode stats equal the oracle's episode return/length."""
    L, B = 10, 8
    seeds = list(range(500, 500 + B))
    cfg = O.Config(base_LP=1)  # short episodes
    with reference_settings({"base_LP": 1}, False):
        ea = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
        eb = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        ea.reset()
        eb.reset()
        orc = [O.Env(L, O.MODE_DEF, 1, s, s, cfg, O.Hyper(), road_attempts=20000) for s in seeds]
        rets = [0.0] * B
        rng = np.random.RandomState(3)
        finished, finished_sum = 0, 0.0
        ea.episode_stats(clear=True)
        for k in range(400):
            acts = rng.randint(0, 6 * L * L + 1, size=B).astype(np.int64)
            ea.step(def_act=torch.from_numpy(acts))
            eb.step(def_act=torch.from_numpy(acts))
            da = ea.done.cpu().numpy().copy()
            assert np.array_equal(da, eb.done.cpu().numpy())
            assert np.array_equal(ea.reward.cpu().numpy(), eb.reward.cpu().numpy())
            for b in range(B):
                _, r, d, _ = orc[b].step(int(acts[b]))
                rets[b] += r
                assert bool(d) == bool(da[b])
                if d:
                    assert canon.fhex(ea.ep_return[b].item()) == canon.fhex(rets[b])
                    assert ea.ep_len[b].item() == orc[b]._board.steps
                    finished_sum += rets[b]
                    rets[b] = 0.0
                    orc[b].reset()
                    finished += 1
            if da.any():
                eb.reset(da)
                assert torch.equal(ea.obs, eb.obs)
            else:
                assert torch.equal(ea.obs, eb.obs)
        assert finished > 0
        # device-side episode accounting (td_episode_stats): count exact, f64 sum up to order
        st = ea.episode_stats().cpu().numpy()
        assert st[0] == finished
        assert st[1] == pytest.approx(finished_sum, rel=1e-12, abs=1e-9)
    finally:
        ea.close()
        eb.close()


# BASELINE.json configs[1]-[4] per GPU: 4,096 and 65,536 x 10x10 TD-def (configs[1], the
# metric at N = 1), 8,192 (the N = 8 share of configs[3]), 16,384 x 20x20 TD-2p multi-action
# (configs[2]) and 16,384 x 30x30 TD-def (one GPU's share of configs[4]), on the kernel
# td_create picks for each (and the 8,192 share also on the large kernel).  10x10 runs past a
# full episode (1,300 steps: every board reaches the 0.75 enemy upgrade and auto-resets at
# least once, on the staged-layout rings the refill kernel fills).
@pytest.mark.parametrize("L,B,mode,multi,steps,kernel", [
    (10, 4096, "def", False, 1300, "auto"), (10, 8192, "def", False, 1300, "auto"),
    (10, 8192, "def", False, 1300, "large"), (10, 16384, "def", False, 1300, "auto"),
    (10, 65536, "def", False, 1300, "auto"),
    (20, 16384, "2p", True, 300, "auto"), (30, 16384, "def", False, 300, "auto"),
    (30, 16384, "def", False, 300, "large")])
def test_full_size_properties(L, B, mode, multi, steps, kernel):
    """Invariants over every board every 50 steps, and 12 boards per batch bit-exact
    against the C restatement (oracle/td_cpu.c) at every step: reward bits, done, every
    observation byte (the next episode's first one after an auto-reset, failing layout
    draws skipped on both sides), the canonical state every 100 steps."""
    from oracle import td_cpu as C
    from test_gpu_deep import _reset_skipping, ROAD_ATTEMPTS
    seeds = np.arange(B, dtype=np.int64) + 7000 + 100000 * (B == 8192)
    eng = TDEngine(L, B, mode, multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, info=not multi,
                   step_kernel=kernel)
    orc = []
    try:
        if kernel == "auto" and torch.cuda.get_device_properties(0).multi_processor_count == 256:
            # td_create's rule on a 256-CU MI355X: two waves per board up to half a round of
            # waves, one round (8 per SIMD) -> small kernel, then two waves per board again
            # over more rounds (TD-def 10x10: every batch, other 10x10 modes: 3, 30x30: 10,
            # TD-2p 20x20 multi-action: 8; other multi-action boards: large)
            want = {(10, 4096): "small2", (10, 8192): "small", (10, 16384): "small2", (10, 65536): "small2",
                    (20, 16384): "small2" if mode == "2p" and multi else "large",
                    (30, 16384): "small2"}[(L, B)]
            assert eng.step_kernel == want, eng.step_kernel_name
        obs, failed = eng.reset()
        good = np.ones(B, bool)
        good[failed] = False
        picks = [int(b) for b in np.random.RandomState(1).choice(B, 24, replace=False) if good[b]][:12]
        orc = [C.Env(L, mode, 1, int(seeds[b]), int(seeds[b]), multi=multi, road_attempts=ROAD_ATTEMPTS) for b in picks]
        ob = obs[picks].cpu().numpy()
        for j, o in enumerate(orc):
            assert np.array_equal(ob[j], o.obs())
        # boards whose first draw failed (the reference raises) stay unstepped: flagged, zero obs
        assert len(failed) < B // 10
        g = torch.Generator(device="cuda").manual_seed(5)
        resets = 0
        for k in range(steps):
            if multi:
                d = torch.randint(0, 3, (B, 6, L, L), device="cuda", generator=g, dtype=torch.int64)
            else:
                d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            a = torch.randint(0, 5, (B, 3, 8), device="cuda", generator=g, dtype=torch.int64) if mode == "2p" else None
            eng.step(def_act=d, atk_act=a)
            ob = eng.obs
            if k % 50 == 0 or k == steps - 1:
                assert float(ob.min()) >= 0.0
                assert torch.equal(ob[:, 0], (ob[:, 1:4].sum(1) > 0).float())
                if failed:
                    assert float(ob[failed].abs().max()) == 0.0
            dh = d[picks].cpu().numpy()
            ah = a[picks].cpu().numpy() if a is not None else [None] * len(picks)
            obh = ob[picks].cpu().numpy()
            rwh = eng.reward[picks].cpu().numpy()
            dnh = eng.done[picks].cpu().numpy()
            st = eng.export_state() if k % 100 == 99 else None
            for j, o in enumerate(orc):
                wo, wr, wd = o.step(dh[j] if multi else int(dh[j]), ah[j])
                assert canon.fhex(rwh[j]) == canon.fhex(wr), (k, picks[j])
                assert bool(dnh[j]) == wd, (k, picks[j])
                if wd:
                    wo = _reset_skipping(o)
                    resets += 1
                assert np.array_equal(obh[j], wo), (k, picks[j], np.argwhere(obh[j] != wo)[:5].tolist())
                if st is not None:
                    assert canon.state_digest(eng.board_state(picks[j], st)) == canon.digest(o.state_bytes()), \
                        (k, picks[j])
        if steps > 1200:
            assert resets >= len(picks)  # every checked board finished an episode and auto-reset
        fl = eng.flags()
        assert (fl[good] == 0).all(), np.unique(fl[good], return_counts=True)
        assert (fl[~good] == 8).all()  # TD_FLAG_NO_LAYOUT
    finally:
        eng.close()
        for o in orc:
            o.close()


# Every board of the BASELINE-sized batches against the C restatement for the first
# steps (test_full_size_properties follows 12 boards per batch for 1,300 steps): the
# metric's 65,536 x 10x10 on the two-wave kernel, the N = 8 share (8,192, small kernel),
# configs[1] (4,096, two-wave kernel), configs[2] (16,384 x TD-2p 20x20 multi-action) and
# configs[4] per GPU (16,384 x 30x30).
@pytest.mark.parametrize("L,B,mode,multi,steps", [
    (10, 65536, "def", False, 8), (10, 8192, "def", False, 24), (10, 4096, "def", False, 24),
    (20, 16384, "2p", True, 3), (30, 16384, "def", False, 3)])
def test_every_board_of_full_size_batches(L, B, mode, multi, steps):
    """Reward bits, done and every observation byte of every board at every step (the
    boards whose first layout draw fails, where the reference raises, are flagged and
    stay unstepped on the device; the oracle skips them)."""
    from oracle import td_cpu as C
    from test_gpu_deep import _reset_skipping, ROAD_ATTEMPTS
    seeds = np.arange(B, dtype=np.int64) + 31000
    eng = TDEngine(L, B, mode, multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, info=not multi)
    orc = {}
    try:
        obs, failed = eng.reset()
        bad = set(int(b) for b in failed)
        for b in range(B):
            if b in bad:
                continue
            try:
                orc[b] = C.Env(L, mode, 1, int(seeds[b]), int(seeds[b]), multi=multi, road_attempts=ROAD_ATTEMPTS)
            except C.RoadGenError:  # the device flagged the same boards
                raise AssertionError("board %d: the oracle's draw failed, the device's did not" % b)
        assert len(orc) + len(bad) == B and len(bad) < B // 10
        ob = obs.cpu().numpy()
        for b, o in orc.items():
            assert np.array_equal(ob[b], o.obs()), b
        g = torch.Generator(device="cuda").manual_seed(11)
        for k in range(steps):
            if multi:
                d = torch.randint(0, 3, (B, 6, L, L), device="cuda", generator=g, dtype=torch.int64)
            else:
                d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
            a = torch.randint(0, 5, (B, 3, 8), device="cuda", generator=g, dtype=torch.int64) if mode == "2p" else None
            eng.step(def_act=d, atk_act=a)
            dh, ah = d.cpu().numpy(), (a.cpu().numpy() if a is not None else None)
            ob, rw, dn = eng.obs.cpu().numpy(), eng.reward.cpu().numpy(), eng.done.cpu().numpy()
            for b, o in orc.items():
                wo, wr, wd = o.step(dh[b] if multi else int(dh[b]), ah[b] if ah is not None else None)
                assert canon.fhex(rw[b]) == canon.fhex(wr), (k, b)
                assert bool(dn[b]) == wd, (k, b)
                if wd:
                    wo = _reset_skipping(o)
                assert np.array_equal(ob[b], wo), (k, b, np.argwhere(ob[b] != wo)[:5].tolist())
            del ob
        assert (eng.flags()[sorted(orc)] == 0).all()
    finally:
        eng.close()
        for o in orc.values():
            o.close()


def test_reference_kat_on_device():
    """The reference's own known-answer test (TDBoard.py:674-751) through the C-ABI:
    the seed-1024 two-road 10x10 layout (roads drawn by the restatement of
    create_road_v2, handed over with td_layout_from_roads) resets four TD-atk boards
    to the KAT's full initial observation, byte for byte; then every one-enemy
    cluster (types 0-3 on roads 0 and 1) fails at zero attacker cost
    (TDBoard.py:749-751): FailCode COST_SHORTAGE and no enemy on the board."""
    from gym_TD import fail_code
    from gym_TD import _lib
    z = np.load(G.GOLDEN + "/kat_seed1024.npz")
    L, B = 10, 4
    rng = np.random.RandomState()
    rng.seed(1024)
    roads = O.create_road(rng, L, 2)
    cells = np.asarray([p[0] * L + p[1] for r in roads for p in r], dtype=np.int32)
    off = np.cumsum([0] + [len(r) for r in roads]).astype(np.int32)
    rec = np.zeros(8 + L * L, np.uint32)
    assert _lib.lib.td_layout_from_roads(L, 2, _lib.ptr(cells, _lib.ctypes.c_int32),
                                         _lib.ptr(off, _lib.ctypes.c_int32), _lib.ptr(rec, _lib.ctypes.c_uint32)) == 0
    seeds = np.arange(B) + 1024
    eng = TDEngine(L, B, "atk", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=False)
    try:
        obs = eng.reset_layouts(np.stack([rec] * B), np.arange(B))
        for b in range(B):
            assert np.array_equal(obs[b].cpu().numpy(), z["obs"]), b
            m, start, end = eng.map_planes(b)
            assert np.array_equal(m, z["map"]) and start == z["start"].tolist() and end == z["end"].tolist()
        act = np.full((B, 3, 8), 4, dtype=np.int64)  # 4 = no enemy in that slot
        act[:, 0, 0] = np.arange(B)                    # board t: one enemy of type t on road 0 ...
        act[:, 1, 0] = np.arange(B)                    # ... and on road 1
        eng.step(atk_act=torch.from_numpy(act).cuda())
        fa = eng.fail_atk.cpu().numpy()
        assert (fa[:, :2] == fail_code.COST_SHORTAGE).all(), fa
        for b in range(B):
            assert eng.board_state(b)["enemies"] == []
    finally:
        eng.close()


@pytest.mark.parametrize("multi", [False, True])
def test_unaligned_caller_buffers(multi):
    """td_step takes caller-owned pointers: an observation buffer that is only 4-B
    aligned (a float view one element into a larger tensor) and multi-action flags
    only 8-B aligned give the same bytes as 16-B-aligned buffers (the kernels store
    16-B units and read 16-B flag pairs)."""
    L, B = 10, 48
    seeds = np.arange(B) + 3100
    a = TDEngine(L, B, "def", multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    b = TDEngine(L, B, "def", multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    try:
        a.reset_all()
        b.reset_all()
        n = B * 45 * L * L
        big = torch.full((n + 1,), -1.0, device="cuda")
        b.obs = big[1:].view(B, 45, L, L)
        assert b.obs.data_ptr() % 16 == 4
        b._io.obs = b.obs.data_ptr()
        g = torch.Generator(device="cuda").manual_seed(9)
        for k in range(120):
            if multi:
                d = torch.randint(0, 3, (B, 6, L, L), device="cuda", generator=g, dtype=torch.int64)
                dbig = torch.empty(d.numel() + 1, dtype=torch.int64, device="cuda")
                dbig[1:] = d.reshape(-1)
                du = dbig[1:].view(B, 6, L, L)
                assert du.data_ptr() % 16 == 8
            else:
                d = torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64)
                du = d
            a.step(def_act=d)
            b.step(def_act=du)
            assert torch.equal(a.obs, b.obs), k
            assert torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done), k
        assert float(big[0]) == -1.0  # nothing written before the buffer
    finally:
        a.close()
        b.close()
