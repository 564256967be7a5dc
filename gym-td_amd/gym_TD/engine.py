"""TDEngine: B independent gym-TD boards in HBM, stepped by libtdstep.so.

The batched counterpart of TDGymBasic + TDDefense / TDAttack / TDMulti
(gym_TD/envs/TDGymBasic.py, TDDefense.py, TDAttack.py, TDMulti.py).  Actions and
outputs are torch tensors on the engine's device; every step is one kernel
launch on torch's current stream.
"""
import copy
import os
import types

import numpy as np
import torch

from . import _lib
from . import params as P

MODES = {"def": 0, "atk": 1, "2p": 2}

HDR_DTYPE = np.dtype([
    ("cost_def", "<f8"), ("cost_atk", "<f8"), ("ep_return", "<f8"), ("steps", "<i4"), ("base_LP", "<i4"),
    ("atk_cd", "<i4"), ("def_cd", "<i4"), ("n_en", "<i4"), ("n_tw", "<i4"), ("num_roads", "<i4"),
    ("end_cell", "<i4"), ("start_cell", "<i4", (3,)), ("maxdist", "<i4"), ("flags", "<i4"), ("episodes", "<i4"),
    ("max_cost", "<f8"), ("max_base_LP", "<i4"), ("format", "<i4")])
assert HDR_DTYPE.itemsize == _lib.HDR_BYTES


class _DeviceBlock(object):
    """A td_alloc_device block seen by torch through __cuda_array_interface__.  The
    tensor keeps this object alive; the block is freed when the last tensor (or view)
    using it is gone."""

    def __init__(self, ptr, shape, typestr):
        self.ptr = ptr
        self.__cuda_array_interface__ = {"shape": tuple(int(n) for n in shape), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 2, "strides": None}

    def __del__(self):
        try:
            if self.ptr:
                _lib.lib.td_free_device(self.ptr)
                self.ptr = None
        except Exception:  # (interpreter shutdown)
            pass


_TYPESTR = {torch.float32: "<f4", torch.int64: "<i8"}


# The engine's observation in physically contiguous device memory or a plain allocation.
# auto (default): contiguous from CONTIG_OBS_MIN bytes on -- faster there (32,768 boards at
# 10x10, 590 MB: 112.5 vs 115.5 us; 30x30 / 16,384, 2.65 GB: 498.7 vs 517.6; 65,536 +-0),
# slower below (16,384 / 8,192 / 4,096 boards: +0.6-2.2 %), profiles/r04/s26.
# TD_CONTIG_OBS=1 / 0 (or true / false, yes / no, on / off) forces it; any other value
# warns once and keeps auto.
CONTIG_OBS_MIN = 512 << 20


def _parse_contig_obs(v):
    v = (v or "auto").strip().lower()
    if v in ("1", "true", "yes", "on"):
        return True
    if v in ("0", "false", "no", "off"):
        return False
    if v != "auto":
        import warnings
        warnings.warn("TD_CONTIG_OBS=%r is not auto / 0 / 1 / true / false: using auto" % v, RuntimeWarning)
    return "auto"


CONTIG_OBS = _parse_contig_obs(os.environ.get("TD_CONTIG_OBS"))


def _contig_obs(nbytes):
    if CONTIG_OBS == "auto":
        return nbytes >= CONTIG_OBS_MIN
    return CONTIG_OBS


def device_zeros(shape, dtype, device, contiguous=None):
    """A zeroed device tensor in td_alloc_device memory (contiguous: physically contiguous
    where the driver can give it); torch.zeros if torch cannot adopt the block."""
    dev = torch.device(device)
    n = int(np.prod(shape)) * torch.tensor([], dtype=dtype).element_size()
    p = _lib.ctypes.c_void_p()
    contig = _contig_obs(n) if contiguous is None else bool(contiguous)
    if _lib.lib.td_alloc_device(n, dev.index or 0, int(contig), _lib.ctypes.byref(p)) != 0 or not p.value:
        return torch.zeros(shape, dtype=dtype, device=dev)
    blk = _DeviceBlock(p.value, shape, _TYPESTR[dtype])
    try:
        t = torch.as_tensor(blk, device=dev)
    except Exception:
        t = None
    if t is None or t.data_ptr() != p.value or t.dtype != dtype or tuple(t.shape) != tuple(shape):
        del blk  # (frees the block)
        return torch.zeros(shape, dtype=dtype, device=dev)
    t._td_block = True  # (tests: the block was adopted)
    # how the block was placed (a refused contiguous request is a plain allocation):
    # TDEngine.obs_alloc, by which bench.py keys its PMC traffic records
    t._td_contig = _lib.lib.td_alloc_is_contiguous(p.value) == 1
    return t


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


class TDEngine(object):
    """B boards of one map size and mode.

    mode: 'def' (TD-def: defender acts, built-in random_enemy_lv{difficulty}),
          'atk' (TD-atk: attacker acts, built-in random_tower_lv{difficulty}),
          '2p'  (TD-2p: both act).
    multi_action: HyperParameters.allow_multiple_actions (defender flags (6, L, L)).
    np_seeds / py_seeds: per-board seeds of the layout stream (numpy RandomState)
          and of the built-in opponent's CPython ``random`` stream.
    autoreset: a board that finishes starts its next episode inside the same
          step and the returned obs is the new episode's first obs (gym 0.21
          AsyncVectorEnv semantics); reward/done/info describe the finished step.
    host_io: step inputs and outputs live in pinned host memory that the kernels
          read and write directly (zero-copy).  For the single-env classes: one
          launch and one stream synchronisation per step, no per-tensor copies.
          A host_io step() is synchronous: it returns once the kernel has read the
          staged actions and written the outputs.
    random_agent: TDGymBasic's random_agent (False: the built-in opponent draws from
          each board's layout stream; with auto-reset the next layout is then drawn
          right after the step that ends the episode, in stream order).
    step_kernel: 'auto' (td_create's rule by batch size), 'large', 'small' or 'small2'
          (td_set_step_kernel; the three give the same results).
    """

    def __init__(self, map_size, n_boards, mode="def", multi_action=None, difficulty=1, device=None,
                 np_seeds=None, py_seeds=None, autoreset=True, info=True, cfg=None, hp=None, host_io=False,
                 random_agent=True, step_kernel="auto"):
        hp = hp or P.hyper_parameters
        if multi_action is None:
            multi_action = bool(hp.allow_multiple_actions)
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.L, self.B, self.mode = int(map_size), int(n_boards), mode
        self.multi = bool(multi_action)
        self.difficulty = int(difficulty)
        self._cfg_c = P.to_c(cfg or P.config, hp)
        self._cfg_hist = {0: copy.deepcopy(cfg or P.config)}  # paramConfig epoch -> config (td_config_epoch)
        h = _lib.lib.td_create(self._cfg_c, self.L, self.B, MODES[mode], int(self.multi), self.difficulty,
                               self.device.index or 0)
        if not h:
            raise _lib.TDError(_lib.lib.td_last_error().decode())
        self._h = h
        self.lw = _lib.lib.td_layout_words(self.L)
        self.autoreset = bool(autoreset)
        _lib.check(_lib.lib.td_set_autoreset(h, int(self.autoreset)))
        self.random_agent = bool(random_agent)
        if not self.random_agent:  # opponents on the layout stream (needs auto-reset off)
            _lib.check(_lib.lib.td_set_random_agent(h, 0))
        B, L = self.B, self.L
        self.host_io = bool(host_io)
        dev = torch.device("cpu") if self.host_io else self.device
        zeros = (lambda shape, dtype: torch.zeros(shape, dtype=dtype).pin_memory()) if self.host_io else \
            (lambda shape, dtype: torch.zeros(shape, dtype=dtype, device=dev))
        # the observation, the step's write stream: contiguous device memory (td_alloc_device)
        self.obs = zeros((B, _lib.NCH, L, L), torch.float32) if self.host_io else \
            device_zeros((B, _lib.NCH, L, L), torch.float32, self.device)
        # how the observation was allocated (bench.py keys PMC traffic records by it)
        self.obs_alloc = "host" if self.host_io else "contiguous" if getattr(self.obs, "_td_contig", False) else "plain"
        self.reward = zeros(B, torch.float64)
        self.done = zeros(B, torch.uint8)
        self.info_enabled = bool(info)
        self.win = self.allow_next = self.cooldowns = self.ep_return = self.ep_len = None
        self.real_def = self.fail_def = self.real_atk = self.fail_atk = None
        if info:
            self.win = zeros(B, torch.int8)
            self.allow_next = zeros(B, torch.uint8)
            self.cooldowns = zeros(B, torch.uint8)
            self.ep_return = zeros(B, torch.float64)
            self.ep_len = zeros(B, torch.int32)
            if mode != "atk":
                shape = (B, 6, L, L) if self.multi else (B,)
                self.real_def = zeros(shape, torch.int64) if self.host_io or not self.multi else \
                    device_zeros(shape, torch.int64, self.device)
                self.fail_def = zeros(B, torch.int32)
            if mode != "def":
                self.real_atk = zeros((B, 3, 8), torch.int64)
                self.fail_atk = zeros((B, 3), torch.int32)
        if self.host_io:  # action staging, read by the kernel from pinned host memory
            self._def_in = zeros((B, 6, L, L) if self.multi else (B,), torch.int64) if mode != "atk" else None
            self._atk_in = zeros((B, 3, 8), torch.int64) if mode != "def" else None
        self._io = _lib.TdStepIO()
        # host_io: numpy views of the pinned buffers, made once (a torch -> numpy
        # conversion or a scalar read through torch costs microseconds per step)
        self.np = types.SimpleNamespace()
        for name in ("obs", "reward", "done", "real_def", "real_atk", "fail_def", "fail_atk", "win",
                     "allow_next", "cooldowns", "ep_return", "ep_len"):
            t = getattr(self, name)
            setattr(self._io, name, t.data_ptr() if t is not None else None)
            if self.host_io:
                setattr(self.np, name, t.numpy() if t is not None else None)
        if self.host_io:
            self._def_np = self._def_in.numpy() if self._def_in is not None else None
            self._atk_np = self._atk_in.numpy() if self._atk_in is not None else None
        if np_seeds is not None or py_seeds is not None:
            self.seed(np_seeds, py_seeds)
        if step_kernel != "auto":
            self.set_step_kernel(step_kernel)
        P._live.add(self)

    # ------------------------------------------------------------------ setup
    def close(self):
        if getattr(self, "_h", None):
            _lib.lib.td_destroy(self._h)
            self._h = None
        P._live.discard(self)  # paramConfig reaches live engines only

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_config(self, cfg=None, hp=None):
        """paramConfig on this engine: the new values apply from the next step; live
        enemies and towers keep the values they were created / upgraded with, and each
        board the max_cost / base_LP of its last reset (TDElements.py:4-69, TDBoard.py:66-72)."""
        self._cfg_c = P.to_c(cfg or P.config, hp)
        _lib.check(_lib.lib.td_set_config(self._h, self._cfg_c))
        self._cfg_hist[_lib.lib.td_config_epoch(self._h)] = copy.deepcopy(cfg or P.config)

    def config_of_epoch(self, ep):
        """The game config of paramConfig epoch ``ep`` (entity words carry their epoch)."""
        return self._cfg_hist.get(ep, P.config)

    def seed(self, np_seeds=None, py_seeds=None):
        """Per-board seeds (int or array of B)."""
        def arr(s):
            if s is None:
                return None
            a = np.asarray(s, dtype=np.int64)
            if a.ndim == 0:
                a = np.full(self.B, int(a), dtype=np.int64)
            if a.shape != (self.B,) or (a < 0).any() or (a > 0xFFFFFFFF).any():
                raise ValueError("seeds must be B ints in [0, 2**32)")
            return _u32(a)
        npa, pya = arr(np_seeds), arr(py_seeds)
        _lib.check(_lib.lib.td_seed(self._h, _lib.ptr(npa, _lib.ctypes.c_uint32) if npa is not None else None,
                                    _lib.ptr(pya, _lib.ctypes.c_uint32) if pya is not None else None))

    def set_py_state(self, b, state):
        """Import a CPython ``random.getstate()`` (or 625 words) as board b's opponent stream."""
        w = _mt_words(state)
        _lib.check(_lib.lib.td_set_py_state(self._h, int(b), _lib.ptr(w, _lib.ctypes.c_uint32)))

    def get_py_state(self, b):
        w = np.zeros(_lib.MT_WORDS, dtype=np.uint32)
        _lib.check(_lib.lib.td_get_py_state(self._h, int(b), _lib.ptr(w, _lib.ctypes.c_uint32)))
        return w

    def set_np_state(self, b, state):
        """Import a ``RandomState.get_state()`` (or 625 words) as board b's layout stream."""
        w = _mt_words(state)
        _lib.check(_lib.lib.td_set_np_state(self._h, int(b), _lib.ptr(w, _lib.ctypes.c_uint32)))

    def get_np_state(self, b):
        w = np.zeros(_lib.MT_WORDS, dtype=np.uint32)
        _lib.check(_lib.lib.td_get_np_state(self._h, int(b), _lib.ptr(w, _lib.ctypes.c_uint32)))
        return w

    # ------------------------------------------------------------------- run
    def _stream(self):
        return torch.cuda.current_stream(self.device).cuda_stream

    def reset(self, mask=None):
        """TDGymBasic.reset for the boards in ``mask`` (None = all).  Returns the
        obs tensor (B, 45, L, L) and the list of boards whose road generation
        failed (the reference raises or hangs there; those boards are unchanged)."""
        m = None
        if mask is not None:
            m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(self.B))
        torch.cuda.synchronize(self.device)
        rc = _lib.lib.td_reset(self._h, _lib.ptr(m, _lib.ctypes.c_uint8) if m is not None else None,
                               self.obs.data_ptr(), self._stream())
        _lib.check(rc)
        failed = []
        if rc > 0:
            ids = np.zeros(rc, dtype=np.int32)
            _lib.lib.td_last_reset_failures(self._h, _lib.ptr(ids, _lib.ctypes.c_int32), rc)
            failed = ids.tolist()
        return self.obs, failed

    def reset_all(self, max_retries=64):
        """reset() every board, redrawing (from the same streams) the layouts whose
        road generation failed -- the reference would raise or hang on those draws
        (TDRoadGen.py:177-189).  Returns (obs, number of failed draws skipped)."""
        obs, failed = self.reset()
        skipped = 0
        while failed and max_retries > 0:
            skipped += len(failed)
            m = np.zeros(self.B, dtype=np.uint8)
            m[failed] = 1
            obs, failed = self.reset(m)
            max_retries -= 1
        if failed:
            raise RuntimeError("road generation kept failing for boards %r" % failed[:8])
        return obs, skipped

    def reset_layouts(self, recs, boards):
        recs = _u32(recs).reshape(-1, self.lw)
        ids = np.ascontiguousarray(boards, dtype=np.int32)
        torch.cuda.synchronize(self.device)
        _lib.check(_lib.lib.td_reset_layouts(self._h, _lib.ptr(recs, _lib.ctypes.c_uint32),
                                             _lib.ptr(ids, _lib.ctypes.c_int32), len(ids), self.obs.data_ptr(),
                                             self._stream()))
        return self.obs

    def step(self, def_act=None, atk_act=None):
        """One step of every board; returns (obs, reward, done) device tensors.

        The tensors are the engine's own buffers, overwritten by the next step
        (clone them to keep a history)."""
        io = self._io
        keep = []
        if self.host_io:
            if self.mode != "atk":
                self._def_np[...] = np.asarray(def_act, dtype=np.int64).reshape(self._def_np.shape)
                io.def_act = self._def_in.data_ptr()
            if self.mode != "def":
                self._atk_np[...] = np.asarray(atk_act, dtype=np.int64).reshape(self._atk_np.shape)
                io.atk_act = self._atk_in.data_ptr()
            _lib.check(_lib.lib.td_step(self._h, io, self._stream()))
            # the outputs are the caller's as soon as this returns, and the next call
            # rewrites the staged actions: wait for the kernel
            torch.cuda.current_stream(self.device).synchronize()
            return self.obs, self.reward, self.done
        if self.mode != "atk":
            d = _as_dev(def_act, torch.int64, self.device)
            exp = (self.B, 6, self.L, self.L) if self.multi else (self.B,)
            if tuple(d.shape) != exp:
                raise ValueError("defender action must have shape %r" % (exp,))
            keep.append(d)
            io.def_act = d.data_ptr()
        if self.mode != "def":
            a = _as_dev(atk_act, torch.int64, self.device)
            if tuple(a.shape) != (self.B, 3, 8):
                raise ValueError("attacker action must have shape (B, 3, 8)")
            keep.append(a)
            io.atk_act = a.data_ptr()
        _lib.check(_lib.lib.td_step(self._h, io, self._stream()))
        self._keep = keep  # actions stay alive until the next call
        return self.obs, self.reward, self.done

    # ----------------------------------------------------------------- state
    def state_bytes(self, count):
        return _lib.lib.td_state_bytes(self._h, count)

    def export_state(self, b0=0, count=None):
        """Raw SoA state of boards [b0, b0+count) as numpy arrays (td_export_state).  The
        numpy layout stream is not included: get_np_state / set_np_state carry it (with
        random_agent=False it is the built-in opponent's stream too)."""
        count = self.B - b0 if count is None else count
        buf = np.zeros(self.state_bytes(count), dtype=np.uint8)
        torch.cuda.synchronize(self.device)
        _lib.check(_lib.lib.td_export_state(self._h, b0, count, buf.ctypes.data))
        return _decode_state(buf, count, self.L)

    def import_state(self, st, b0=0):
        count = len(st["hdr"])
        buf = _encode_state(st, count, self.L)
        torch.cuda.synchronize(self.device)
        _lib.check(_lib.lib.td_import_state(self._h, b0, count, buf.ctypes.data))

    def episode_stats(self, clear=False):
        """Device f64 [2]: episodes finished since the last clear and the sum of their returns."""
        out = torch.empty(2, dtype=torch.float64, device=self.device)
        _lib.check(_lib.lib.td_episode_stats(self._h, _lib.ctypes.c_void_p(out.data_ptr()), int(bool(clear)),
                                             self._stream()))
        return out

    def episode_records(self):
        """Each board's last finished episode (td_episode_records): (return f64 [B],
        length int32 [B], win int32 [B], -1 before the board's first finished episode),
        device tensors -- the per-board payload gathered across ranks."""
        raw = torch.empty((self.B, 16), dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib.td_episode_records(self._h, _lib.ctypes.c_void_p(raw.data_ptr()), self._stream()))
        ints = raw[:, 8:].contiguous().view(torch.int32)
        return raw[:, :8].contiguous().view(torch.float64).reshape(self.B), ints[:, 0], ints[:, 1]

    def opponent(self, side, level, mask=None):
        """Run the built-in opponent on its own (TDGymBasic.py:81-292): side 'enemy'
        (random_enemy_lv<level>) or 'tower' (random_tower_lv<level>), boards in mask."""
        m = None
        if mask is not None:
            m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(self.B))
        _lib.check(_lib.lib.td_opponent(self._h, {"enemy": 0, "tower": 1}[side], int(level),
                                        _lib.ptr(m, _lib.ctypes.c_uint8) if m is not None else None, self._stream()))

    def set_step_kernel(self, kind):
        """Select the step kernel: 'auto', 'large', 'small' or 'small2' (td_set_step_kernel)."""
        if kind not in _lib.STEP_KERNELS:
            raise ValueError("step kernel must be one of %s" % sorted(_lib.STEP_KERNELS))
        _lib.check(_lib.lib.td_set_step_kernel(self._h, _lib.STEP_KERNELS[kind]))

    @property
    def step_kernel(self):
        """The step kernel td_step launches: 'large', 'small' or 'small2'."""
        k = _lib.check(_lib.lib.td_step_kernel(self._h))
        return {v: n for n, v in _lib.STEP_KERNELS.items()}[k]

    @property
    def step_kernel_name(self):
        """Its name as rocprofv3 reports it, e.g. 'td_step_kernel_small<10, 0, false>'."""
        return _lib.lib.td_step_kernel_name(self._h).decode()

    def set_store_policy(self, xcd_map=1, edge_wt=2):
        """Board map and shared-line store policy of the step kernels (td_set_store_policy):
        xcd_map 1 = XCD-contiguous boards, 0 = block i steps board i; edge_wt 2 = the lines a
        board shares with its neighbours as plain write-back stores, 1 = write-through.  Every
        policy gives the same bytes; the defaults are the fastest measured."""
        _lib.check(_lib.lib.td_set_store_policy(self._h, int(xcd_map), int(edge_wt)))

    def guard_timeouts(self, clear=False):
        """Ring-guard waits for a board's refill claim that gave up (td_guard_timeouts)."""
        return _lib.check(_lib.lib.td_guard_timeouts(self._h, int(bool(clear))))

    def set_refill_interval(self, steps):
        """Steps between layout-refill launches (auto-reset; 0 = none, rings only drain)."""
        _lib.check(_lib.lib.td_set_refill_interval(self._h, int(steps)))

    def kernel_timing(self, max_launches, every=1):
        """Time the step kernels of every ``every``-th step from now, ``max_launches`` of
        them, from their dispatch timestamps (events bound to the launch itself); read
        them with kernel_times()."""
        _lib.check(_lib.lib.td_kernel_timing(self._h, int(max_launches), int(every)))

    def kernel_times(self):
        """Durations (microseconds, numpy float32) of the step kernels timed since kernel_timing()."""
        cap = 1 << 20
        n = _lib.check(_lib.lib.td_kernel_times(self._h, None, 0))
        out = np.zeros(max(n, 1), dtype=np.float32)
        n = _lib.check(_lib.lib.td_kernel_times(self._h, _lib.ptr(out, _lib.ctypes.c_float), min(n, cap)))
        return out[:n]

    def flags(self):
        f = np.zeros(self.B, dtype=np.int32)
        _lib.check(_lib.lib.td_get_flags(self._h, _lib.ptr(f, _lib.ctypes.c_int32)))
        return f

    def board_state(self, b, st=None):
        """Canonical state of board b (same record as the reference's board attributes)."""
        if st is None:
            st = self.export_state(b, 1)
            i = 0
        else:
            i = b
        h = st["hdr"][i]
        n, nt, L = int(h["n_en"]), int(h["n_tw"]), self.L
        inf = st["en_inf"][i][:n]
        ens = [(int((u >> 12) & 3), int((u >> 14) & 1), int(u & 0xFFF) // L, int(u & 0xFFF) % L, int((u >> 16) & 0xFF),
                float(st["en_lp"][i][k]), float(st["en_mg"][i][k])) for k, u in enumerate(inf)]
        tinf = st["tw_inf"][i][:nt]
        tws = [(int((u >> 12) & 3), int((u >> 14) & 1), int(u & 0xFFF) // L, int(u & 0xFFF) % L,
                float(st["tw_cd"][i][k])) for k, u in enumerate(tinf)]
        return {"steps": int(h["steps"]), "base_LP": int(h["base_LP"]), "cost_def": float(h["cost_def"]),
                "cost_atk": float(h["cost_atk"]), "attacker_cd": int(h["atk_cd"]), "defender_cd": int(h["def_cd"]),
                "enemies": ens, "towers": tws, "map6": (st["cells"][i] >> 24).astype(np.int64).tolist(),
                "num_roads": int(h["num_roads"]), "flags": int(h["flags"])}

    def map_planes(self, b, st=None):
        """TDBoard.map planes 0-6 of board b (int32 (7, L, L)), start list, end."""
        if st is None:
            st = self.export_state(b, 1)
            b = 0
        cw = st["cells"][b].astype(np.int64)
        L = self.L
        m = np.zeros((7, L, L), dtype=np.int32)
        for p in range(4):
            m[p] = ((cw >> p) & 1).reshape(L, L)
        m[4] = ((cw >> 16) & 0xFF).reshape(L, L)
        m[5] = ((cw >> 8) & 3).reshape(L, L)
        m[6] = (cw >> 24).reshape(L, L)
        h = st["hdr"][b]
        nr = int(h["num_roads"])
        start = [[int(c) // L, int(c) % L] for c in h["start_cell"][:nr]]
        end = [int(h["end_cell"]) // L, int(h["end_cell"]) % L]
        return m, start, end


def _as_dev(x, dtype, device):
    if isinstance(x, torch.Tensor):
        if x.device != device or x.dtype != dtype or not x.is_contiguous():
            x = x.to(device=device, dtype=dtype).contiguous()
        return x
    return torch.as_tensor(np.asarray(x), dtype=dtype).to(device).contiguous()


def _mt_words(state):
    """random.getstate() / RandomState.get_state() / 625 words -> uint32[625]."""
    if isinstance(state, tuple) and len(state) == 3 and isinstance(state[1], tuple):  # CPython random
        return _u32(list(state[1]))
    if isinstance(state, tuple) and len(state) >= 3 and state[0] == "MT19937":  # numpy RandomState
        return _u32(list(state[1]) + [int(state[2])])
    w = _u32(state)
    if w.shape != (_lib.MT_WORDS,):
        raise ValueError("expected 625 words")
    return w


def _layout(count, L):
    return [("hdr", HDR_DTYPE, ()), ("en_lp", np.float64, (_lib.ECAP,)), ("en_mg", np.float64, (_lib.ECAP,)),
            ("en_inf", np.uint32, (_lib.ECAP,)), ("tw_cd", np.float64, (_lib.TCAP,)),
            ("tw_inf", np.uint32, (_lib.TCAP,)), ("cells", np.uint32, (L * L,)),
            ("opp_mt", np.uint32, (_lib.OPP_WORDS,))]


def _decode_state(buf, count, L):
    out, off = {}, 0
    for name, dt, shape in _layout(count, L):
        dt = np.dtype(dt)
        n = count * int(np.prod(shape, dtype=np.int64)) if shape else count
        a = np.frombuffer(buf, dtype=dt, count=n, offset=off)
        out[name] = a.reshape((count,) + shape) if shape else a
        off += n * dt.itemsize
    return out


def _encode_state(st, count, L):
    parts = []
    for name, dt, shape in _layout(count, L):
        parts.append(np.ascontiguousarray(st[name], dtype=dt).tobytes())
    return np.frombuffer(b"".join(parts), dtype=np.uint8).copy()


def layout_planes(rec, L):
    """Layout record (td_layout.h) -> (map planes int32 (7, L, L), start list, end, num_roads)."""
    rec = np.asarray(rec, dtype=np.uint32)
    cw = rec[8:8 + L * L].astype(np.int64)
    m = np.zeros((7, L, L), dtype=np.int32)
    for p in range(4):
        m[p] = ((cw >> p) & 1).reshape(L, L)
    m[4] = ((cw >> 16) & 0xFF).reshape(L, L)
    m[5] = ((cw >> 8) & 3).reshape(L, L)
    m[6] = (cw >> 24).reshape(L, L)
    nr = int(rec[1])
    start = [[int(c) // L, int(c) % L] for c in rec[4:4 + nr]]
    end = [int(rec[2]) // L, int(rec[2]) % L]
    return m, start, end, nr


def generate_layout(np_state, L, max_attempts=20000):
    """TDGymBasic.reset's draws (num_roads + create_road_v2) on a 625-word numpy
    stream, in place; returns (status, record)."""
    rec = np.zeros(8 + L * L, dtype=np.uint32)
    st = _lib.lib.td_layout_generate(_lib.ptr(np_state, _lib.ctypes.c_uint32), L, max_attempts,
                                     _lib.ptr(rec, _lib.ctypes.c_uint32))
    return st, rec
