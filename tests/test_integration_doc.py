"""CPU checks of the C-ABI boundary's self-description (no GPU).

* INTEGRATION.md's reference-side ctypes stub declares exactly the structs the library
  was built with (field names, order and size) -- the stub is what a gym-TD maintainer
  copies, so it must never fall behind include/tdstep.h (round 3 shipped a 13-pointer
  stub against a 14-pointer td_step_io);
* td_step reads td_step_io's size / abi header first and refuses, before it looks at the
  handle or launches anything, a struct of another size or ABI -- including an ABI-2
  struct (14 pointers, no header).
The GPU half (tests/test_gpu_integration.py) runs the stub verbatim on the device."""
import ast
import ctypes
import os
import re

import pytest

from gym_TD import _lib

HERE = os.path.dirname(os.path.abspath(__file__))
DOC = os.path.join(HERE, "..", "INTEGRATION.md")
lib = _lib.lib


def doc_stub():
    """The python code block of INTEGRATION.md §2 (the one that declares TdStepIO)."""
    blocks = re.findall(r"```python\n(.*?)```", open(DOC).read(), re.S)
    stubs = [b for b in blocks if "class TdStepIO" in b]
    assert len(stubs) == 1, "INTEGRATION.md must hold exactly one TdStepIO stub"
    return stubs[0]


def doc_structs():
    """Execute only the stub's imports and class definitions (no library call)."""
    tree = ast.parse(doc_stub())
    keep = [n for n in tree.body if isinstance(n, (ast.Import, ast.ClassDef))]
    ns = {}
    exec(compile(ast.Module(body=keep, type_ignores=[]), "INTEGRATION.md", "exec"), ns)
    return ns["TdStepIO"], ns["TdConfig"]


def _layout(cls):
    return [(n, ctypes.sizeof(t), getattr(cls, n).offset) for n, t in cls._fields_]


def test_doc_stub_structs_match_the_library():
    io, cfg = doc_structs()
    assert _layout(io) == _layout(_lib.TdStepIO)
    assert _layout(cfg) == _layout(_lib.TdConfig)
    assert ctypes.sizeof(io) == lib.td_step_io_size() == 120
    assert ctypes.sizeof(cfg) == 744


def test_doc_stub_checks_the_abi_version():
    src = doc_stub()
    assert "td_abi_version() == %d" % _lib.ABI_VERSION in src
    assert "abi=%d" % _lib.ABI_VERSION in src
    assert lib.td_abi_version() == _lib.ABI_VERSION == 3


def test_step_io_init_sets_the_header():
    io = _lib.TdStepIO(obs=1234)
    lib.td_step_io_init(io)
    assert io.size == ctypes.sizeof(_lib.TdStepIO) and io.abi == _lib.ABI_VERSION
    assert io.obs is None  # zeroed


class AbiV2StepIO(ctypes.Structure):
    """td_step_io as ABI 2 laid it out: 14 pointers, no size / abi header."""
    _fields_ = [(n, ctypes.c_void_p) for n in (
        "def_act", "atk_act", "obs", "reward", "done", "real_def", "real_atk", "fail_def", "fail_atk",
        "win", "allow_next", "ep_return", "ep_len", "cooldowns")]


def _step(io):
    rc = lib.td_step(None, ctypes.cast(ctypes.byref(io), ctypes.POINTER(_lib.TdStepIO)), None)
    return rc, lib.td_last_error().decode()


def test_abi2_struct_is_refused_before_the_handle_is_read():
    # the pointers of a real ABI-2 caller: device addresses, never 0 in the first slot
    io = AbiV2StepIO(def_act=0x7F3A00001000, obs=0x7F3A00200000, reward=0x7F3A00300000, done=0x7F3A00400000)
    rc, err = _step(io)
    assert rc < 0 and "abi" in err and "size" in err, err
    # a TD-atk ABI-2 caller passes def_act = NULL: header words 0 / 0
    rc, err = _step(AbiV2StepIO(atk_act=0x7F3A00001000))
    assert rc < 0 and "size 0 / abi 0" in err, err


@pytest.mark.parametrize("size, abi", [(112, 3), (120, 2), (120, 4), (0, 3), (128, 3)])
def test_wrong_size_or_abi_is_refused(size, abi):
    io = _lib.TdStepIO(size=size, abi=abi, obs=1, reward=1, done=1, def_act=1)
    rc, err = _step(io)
    assert rc < 0 and ("size %d / abi %d" % (size, abi)) in err, err


def test_current_struct_passes_the_header_check():
    # header accepted: the next check is the handle (NULL here, no GPU needed)
    rc, err = _step(_lib.TdStepIO())
    assert rc < 0 and "NULL handle" in err, err
