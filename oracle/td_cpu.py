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
