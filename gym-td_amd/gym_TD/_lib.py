"""ctypes binding of libtdstep.so (include/tdstep.h).

The library is the only compute path: importing this module without the built
library raises, there is no CPU fallback.  ``torch`` is imported first so that
libtdstep.so binds to the same HIP runtime instance torch already loaded
(both carry SONAME libamdhip64.so.7).
"""
import ctypes
import os

import torch  # noqa: F401  (HIP runtime first; see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TDSTEP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libtdstep.so"))

ECAP, TCAP, NCH = 128, 32, 45
MT_WORDS = 625
OPP_WORDS = 626
HDR_BYTES = 96
ABI_VERSION = 3  # include/tdstep.h TD_ABI_VERSION
STEP_KERNELS = {"auto": 0, "large": 1, "small": 2, "small2": 3}  # enum td_step_kernel_kind

c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_vp = ctypes.c_void_p


class TdConfig(ctypes.Structure):
    """struct td_config (tdstep.h)."""
    _fields_ = [(n, (ctypes.c_double * 2) * 4) for n in (
        "enemy_LP", "enemy_speed", "enemy_defense", "enemy_cost", "tower_attack", "tower_range",
        "tower_splash_range", "tower_cost", "tower_attack_interval")] + [
        (n, ctypes.c_double) for n in (
            "tower_destruct_return", "frozen_time", "frozen_ratio", "attacker_init_cost", "defender_init_cost",
            "base_LP", "max_cost", "reward_kill", "penalty_leak", "reward_time", "attacker_cost_init_rate",
            "attacker_cost_final_rate", "defender_cost_rate", "tower_distance", "enemy_upgrade_at",
            "attacker_action_interval", "defender_action_interval")] + [
        (n, ctypes.c_int32) for n in (
            "max_enemy_lv", "max_tower_lv", "enemy_types", "tower_types", "max_episode_steps",
            "max_cluster_length", "max_num_of_roads", "reserved")]


class TdStepIO(ctypes.Structure):
    """struct td_step_io (tdstep.h): the size / ABI header td_step checks, then device pointers."""
    _fields_ = [("size", ctypes.c_uint32), ("abi", ctypes.c_uint32)] + [(n, c_vp) for n in (
        "def_act", "atk_act", "obs", "reward", "done", "real_def", "real_atk", "fail_def", "fail_atk",
        "win", "allow_next", "ep_return", "ep_len", "cooldowns")]

    def __init__(self, **kw):
        kw.setdefault("size", ctypes.sizeof(TdStepIO))
        kw.setdefault("abi", ABI_VERSION)
        super().__init__(**kw)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError("libtdstep.so not found at %s -- build it with `make -C gym-td_amd/csrc` "
                          "(or __graft_entry__.build()); there is no CPU fallback" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    sig = {
        "td_abi_version": (ctypes.c_int, []),
        "td_step_io_size": (ctypes.c_int, []),
        "td_step_io_init": (None, [ctypes.POINTER(TdStepIO)]),
        "td_alloc_device": (ctypes.c_int, [ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
        "td_free_device": (ctypes.c_int, [ctypes.c_void_p]),
        "td_alloc_is_contiguous": (ctypes.c_int, [ctypes.c_void_p]),
        "td_last_error": (ctypes.c_char_p, []),
        "td_config_default": (None, [ctypes.POINTER(TdConfig)]),
        "td_create": (c_vp, [ctypes.POINTER(TdConfig), ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, ctypes.c_int]),
        "td_destroy": (None, [c_vp]),
        "td_set_config": (ctypes.c_int, [c_vp, ctypes.POINTER(TdConfig)]),
        "td_set_autoreset": (ctypes.c_int, [c_vp, ctypes.c_int]),
        "td_set_random_agent": (ctypes.c_int, [c_vp, ctypes.c_int]),
        "td_seed": (ctypes.c_int, [c_vp, c_u32p, c_u32p]),
        "td_set_py_state": (ctypes.c_int, [c_vp, ctypes.c_int, c_u32p]),
        "td_get_py_state": (ctypes.c_int, [c_vp, ctypes.c_int, c_u32p]),
        "td_set_np_state": (ctypes.c_int, [c_vp, ctypes.c_int, c_u32p]),
        "td_get_np_state": (ctypes.c_int, [c_vp, ctypes.c_int, c_u32p]),
        "td_reset": (ctypes.c_int, [c_vp, c_u8p, c_vp, c_vp]),
        "td_last_reset_failures": (ctypes.c_int, [c_vp, c_i32p, ctypes.c_int]),
        "td_reset_layouts": (ctypes.c_int, [c_vp, c_u32p, c_i32p, ctypes.c_int, c_vp, c_vp]),
        "td_step": (ctypes.c_int, [c_vp, ctypes.POINTER(TdStepIO), c_vp]),
        "td_layout_words": (ctypes.c_int, [ctypes.c_int]),
        "td_layout_from_roads": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_i32p, c_i32p, c_u32p]),
        "td_layout_generate": (ctypes.c_int, [c_u32p, ctypes.c_int, ctypes.c_int, c_u32p]),
        "td_state_bytes": (ctypes.c_size_t, [c_vp, ctypes.c_int]),
        "td_export_state": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, c_vp]),
        "td_import_state": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, c_vp]),
        "td_get_flags": (ctypes.c_int, [c_vp, c_i32p]),
        "td_episode_stats": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, c_vp]),
        "td_episode_records": (ctypes.c_int, [c_vp, c_vp, c_vp]),
        "td_opponent": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int, c_u8p, c_vp]),
        "td_set_refill_interval": (ctypes.c_int, [c_vp, ctypes.c_int]),
        "td_step_kernel": (ctypes.c_int, [c_vp]),
        "td_step_kernel_name": (ctypes.c_char_p, [c_vp]),
        "td_config_epoch": (ctypes.c_int, [c_vp]),
        "td_kernel_timing": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int]),
        "td_kernel_times": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
        "td_guard_timeouts": (ctypes.c_int, [c_vp, ctypes.c_int]),
        # test / measurement hooks (include/td_diag.h): not the drop-in surface
        "td_set_step_kernel": (ctypes.c_int, [c_vp, ctypes.c_int]),
        "td_board_map": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, c_i32p]),
        "td_set_store_policy": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int]),
        "td_debug_set_claim": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int]),
        "td_py_seed": (None, [c_u32p, ctypes.c_uint32]),
        "td_np_seed": (None, [c_u32p, ctypes.c_uint32]),
        "td_mt_next": (ctypes.c_uint32, [c_u32p]),
        "td_py_randint": (ctypes.c_int64, [c_u32p, ctypes.c_int64, ctypes.c_int64]),
        "td_np_randint": (ctypes.c_int64, [c_u32p, ctypes.c_int64, ctypes.c_int64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.td_abi_version() != ABI_VERSION or lib.td_step_io_size() != ctypes.sizeof(TdStepIO):
        raise ImportError("libtdstep.so ABI mismatch: library ABI %d / td_step_io %d bytes, binding ABI %d / %d bytes"
                          % (lib.td_abi_version(), lib.td_step_io_size(), ABI_VERSION, ctypes.sizeof(TdStepIO)))
    return lib


lib = _load()


class TDError(RuntimeError):
    pass


def check(rc):
    if rc is None or rc < 0:
        raise TDError(lib.td_last_error().decode(errors="replace"))
    return rc


def ptr(a, ctype):
    """numpy array -> ctypes pointer."""
    return a.ctypes.data_as(ctypes.POINTER(ctype))
