"""ctypes binding of oracle/td_cpu.c -- TEST AND BENCH INFRASTRUCTURE ONLY.

The plain-C restatement of the env step: a second CPU checker (replayed against
the golden vectors in tests/test_cpu_oracle.py) and the native multi-core CPU
baseline bench.py reports beside the GPU number (SURVEY.md 8(d) ii).  Built by
``oracle/Makefile`` (``__graft_entry__.build()`` runs it) into oracle/lib/.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libtdcpu.so")

# td_cpu.c ``Cfg``: the [4][2] tables, then the scalars, all as doubles
TABLES = ("enemy_LP", "enemy_speed", "enemy_defense", "enemy_cost", "tower_attack", "tower_range",
          "tower_splash_range", "tower_cost", "tower_attack_interval")
SCALARS = ("tower_destruct_return", "frozen_time", "frozen_ratio", "attacker_init_cost", "defender_init_cost",
           "base_LP", "max_cost", "reward_kill", "penalty_leak", "reward_time", "attacker_cost_init_rate",
           "attacker_cost_final_rate", "defender_cost_rate", "tower_distance", "enemy_upgrade_at",
           "attacker_action_interval", "defender_action_interval", "max_tower_lv")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("%s is missing: run `make -C oracle`" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        vp, i64p, f32p, f64p = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p
        L.tdc_cfg_doubles.restype = ctypes.c_int
        L.tdc_new.restype = vp
        L.tdc_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                              ctypes.c_uint32, f64p, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.tdc_free.argtypes = [vp]
        L.tdc_reset.argtypes = [vp]
        L.tdc_reset.restype = ctypes.c_int
        L.tdc_step.argtypes = [vp, i64p, i64p, f32p, ctypes.POINTER(ctypes.c_int)]
        L.tdc_step.restype = ctypes.c_double
        L.tdc_obs.argtypes = [vp, f32p]
        L.tdc_state_bytes.argtypes = [vp, vp, ctypes.c_int]
        L.tdc_state_bytes.restype = ctypes.c_int
        L.tdc_layout.argtypes = [vp, i64p, i64p, i64p]
        L.tdc_layout.restype = ctypes.c_int
        L.tdc_overflow.argtypes = [vp]
        L.tdc_overflow.restype = ctypes.c_int
        L.tdc_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                ctypes.c_int, ctypes.c_uint32, f64p, ctypes.POINTER(ctypes.c_double)]
        L.tdc_bench.restype = ctypes.c_longlong
        L.tdc_batch_new.restype = vp
        L.tdc_batch_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp,
                                    f64p, ctypes.c_int, ctypes.c_int, vp]
        L.tdc_batch_free.argtypes = [vp]
        L.tdc_batch_reset.argtypes = [vp, vp]
        L.tdc_batch_reset.restype = ctypes.c_int
        L.tdc_batch_step.argtypes = [vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.tdc_batch_step.restype = ctypes.c_int
        L.tdc_batch_obs.argtypes = [vp, vp]
        L.tdc_batch_flags.argtypes = [vp, vp]
        L.tdc_batch_state_bytes.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int]
        L.tdc_batch_state_bytes.restype = ctypes.c_int
        _lib = L
    return _lib


def cfg_values(cfg):
    """``oracle.td_oracle.Config`` (or any object with TDParam's attribute names) -> float64 array."""
    vals = []
    for name in TABLES:
        vals.extend(float(v) for row in getattr(cfg, name) for v in row)
    vals.extend(float(getattr(cfg, name)) for name in SCALARS)
    a = np.ascontiguousarray(vals, dtype=np.float64)
    assert a.size == lib().tdc_cfg_doubles()
    return a


class RoadGenError(Exception):
    """create_road_v2 raised (or would not return) for this draw."""


MODES = {"def": 0, "atk": 1, "2p": 2}


class Env(object):
    """One env of the C restatement (the same draws and results as oracle.td_oracle.Env)."""

    def __init__(self, L, mode="def", difficulty=1, seed=0, opp_seed=None, cfg=None, multi=False,
                 road_attempts=1000):
        from oracle.td_oracle import Config
        self.L, self.mode, self.multi = int(L), mode, bool(multi)
        self._cfg = cfg_values(cfg or Config())
        st = ctypes.c_int(0)
        self._h = lib().tdc_new(self.L, MODES[mode], int(difficulty), int(self.multi), int(seed) & 0xFFFFFFFF,
                                int(seed if opp_seed is None else opp_seed) & 0xFFFFFFFF,
                                self._cfg.ctypes.data, int(road_attempts), ctypes.byref(st))
        if not self._h:
            raise ValueError("tdc_new failed")
        if st.value:
            self.close()
            raise RoadGenError("road generation status %d" % st.value)
        self._obs = np.zeros((45, self.L, self.L), dtype=np.float32)
        self._empty_def = np.array([6 * self.L * self.L], dtype=np.int64)
        self._empty_atk = np.full(24, 4, dtype=np.int64)

    def close(self):
        if getattr(self, "_h", None):
            lib().tdc_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reset(self):
        st = lib().tdc_reset(self._h)
        if st:
            raise RoadGenError("road generation status %d" % st)
        lib().tdc_obs(self._h, self._obs.ctypes.data)
        return self._obs.copy()

    def obs(self):
        lib().tdc_obs(self._h, self._obs.ctypes.data)
        return self._obs.copy()

    def step(self, def_act=None, atk_act=None):
        d = self._empty_def if def_act is None else np.ascontiguousarray(np.asarray(def_act, dtype=np.int64).reshape(-1))
        a = self._empty_atk if atk_act is None else np.ascontiguousarray(np.asarray(atk_act, dtype=np.int64).reshape(-1))
        done = ctypes.c_int(0)
        r = lib().tdc_step(self._h, d.ctypes.data, a.ctypes.data, self._obs.ctypes.data, ctypes.byref(done))
        return self._obs.copy(), float(r), bool(done.value)

    def state_bytes(self):
        """oracle.canon.state_bytes layout of the current state."""
        n = lib().tdc_state_bytes(self._h, None, 0)
        buf = np.zeros(n, dtype=np.uint8)
        lib().tdc_state_bytes(self._h, buf.ctypes.data, n)
        return buf.tobytes()

    def layout(self):
        """(map planes int64 (7, L, L), start list, end)."""
        m = np.zeros((7, self.L, self.L), dtype=np.int64)
        s = np.zeros(6, dtype=np.int64)
        e = np.zeros(2, dtype=np.int64)
        nr = lib().tdc_layout(self._h, m.ctypes.data, s.ctypes.data, e.ctypes.data)
        return m, [[int(s[2 * i]), int(s[2 * i + 1])] for i in range(nr)], [int(e[0]), int(e[1])]

    def overflow(self):
        return bool(lib().tdc_overflow(self._h))


def bench(L, mode, multi, n_envs, seconds, threads, seed=90001, cfg=None):
    """Env-steps per second of n_envs C envs on ``threads`` OpenMP threads."""
    from oracle.td_oracle import Config
    c = cfg_values(cfg or Config())
    wall = ctypes.c_double(0.0)
    n = lib().tdc_bench(int(L), MODES[mode], int(bool(multi)), int(n_envs), float(seconds), int(threads),
                        int(seed), c.ctypes.data, ctypes.byref(wall))
    return int(n), float(wall.value)


class Batch(object):
    """n envs of the C restatement stepped together on OpenMP threads (tdc_batch_*): the
    every-board checker of a device batch.  Every reset -- the initial one, explicit ones
    (``reset(mask)``) and auto-resets -- takes the board's next layout draw that succeeds
    (failing draws skipped, as the device's staged layouts are); a board with none keeps
    its state and is flagged (``no_layout``)."""

    def __init__(self, L, n, mode="def", difficulty=1, np_seeds=None, py_seeds=None, cfg=None, multi=False,
                 road_attempts=1000, threads=None):
        from oracle.td_oracle import Config
        self.L, self.n, self.mode, self.multi = int(L), int(n), mode, bool(multi)
        self._cfg = cfg_values(cfg or Config())
        nps = np.ascontiguousarray(np.asarray(np_seeds, dtype=np.int64) & 0xFFFFFFFF, dtype=np.uint32)
        pys = np.ascontiguousarray(np.asarray(py_seeds if py_seeds is not None else np_seeds, dtype=np.int64)
                                   & 0xFFFFFFFF, dtype=np.uint32)
        assert nps.size == self.n and pys.size == self.n
        self.threads = int(threads or min(16, os.cpu_count() or 1))
        st = np.zeros(self.n, dtype=np.int32)
        self._h = lib().tdc_batch_new(self.n, self.L, MODES[mode], int(difficulty), int(self.multi), nps.ctypes.data,
                                      pys.ctypes.data, self._cfg.ctypes.data, int(road_attempts), self.threads,
                                      st.ctypes.data)
        if not self._h:
            raise MemoryError("tdc_batch_new failed (%d envs)" % self.n)
        self.initial_failed = np.flatnonzero(st).tolist()
        self.reward = np.zeros(self.n, dtype=np.float64)
        self.done = np.zeros(self.n, dtype=np.uint8)

    def close(self):
        if getattr(self, "_h", None):
            lib().tdc_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def reset(self, mask=None):
        """Explicit reset of the masked boards (None = all); returns how many found no layout."""
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask).reshape(self.n), dtype=np.uint8)
        return lib().tdc_batch_reset(self._h, None if m is None else m.ctypes.data)

    def step(self, def_act=None, atk_act=None, obs=None, autoreset=True):
        """One step of every board; ``obs`` (float32 [n, 45, L, L]) is filled when given.
        Returns (reward, done) -- arrays owned by this object, overwritten by the next step."""
        d = None if def_act is None else np.ascontiguousarray(def_act, dtype=np.int64)
        a = None if atk_act is None else np.ascontiguousarray(atk_act, dtype=np.int64)
        if obs is not None:
            assert obs.dtype == np.float32 and obs.flags.c_contiguous and obs.size == self.n * 45 * self.L * self.L
        lib().tdc_batch_step(self._h, None if d is None else d.ctypes.data, None if a is None else a.ctypes.data,
                             self.reward.ctypes.data, self.done.ctypes.data,
                             None if obs is None else obs.ctypes.data, int(bool(autoreset)))
        return self.reward, self.done

    def obs(self, out=None):
        out = np.empty((self.n, 45, self.L, self.L), dtype=np.float32) if out is None else out
        lib().tdc_batch_obs(self._h, out.ctypes.data)
        return out

    def no_layout(self):
        f = np.zeros(self.n, dtype=np.int32)
        lib().tdc_batch_flags(self._h, f.ctypes.data)
        return f.astype(bool)

    def state_bytes(self, b):
        n = lib().tdc_batch_state_bytes(self._h, int(b), None, 0)
        buf = np.zeros(n, dtype=np.uint8)
        lib().tdc_batch_state_bytes(self._h, int(b), buf.ctypes.data, n)
        return buf.tobytes()
