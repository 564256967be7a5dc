"""GPU: the C-ABI as a gym-TD maintainer binds it.

INTEGRATION.md §2's ctypes stub -- the reference-side binding of td_step
(TDDefense.step, /root/reference/gym_TD/envs/TDDefense.py:34-87) -- is executed
verbatim, and every output it produced is compared with TDEngine (the package's own
binding) on the same seeds and actions, bit for bit.  An ABI-2 struct handed to a live
handle is refused with no launch: the observation buffer is left untouched."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # collected on CPU too, so skip cleanly
    pytest.skip("needs a GPU", allow_module_level=True)

from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

from test_integration_doc import AbiV2StepIO, doc_stub  # noqa: E402


def test_integration_stub_runs_verbatim_and_matches_the_engine(monkeypatch):
    monkeypatch.setenv("TDSTEP_LIB", _lib.LIB_PATH)
    ns = {"__name__": "integration_stub"}
    exec(compile(doc_stub(), "INTEGRATION.md", "exec"), ns)
    B, L = ns["B"], ns["L"]
    eng = TDEngine(L, B, "def", False, 1, device=0, np_seeds=np.arange(B), py_seeds=np.arange(B), autoreset=True)
    try:
        obs0, failed = eng.reset()
        assert len(failed) == ns["failed"]
        eng.step(def_act=ns["act"])
        torch.cuda.synchronize()
        assert torch.equal(eng.obs.view(torch.int32), ns["obs"].view(torch.int32))
        for k in ("reward", "ep_return"):
            assert torch.equal(getattr(eng, k).view(torch.int64), ns["out"][k].view(torch.int64)), k
        for k in ("done", "real_def", "fail_def", "win", "allow_next", "ep_len", "cooldowns"):
            assert torch.equal(getattr(eng, k), ns["out"][k]), k
        assert int(ns["out"]["done"].sum()) < B  # a real step, not a field of finished boards
    finally:
        eng.close()


def test_abi2_struct_on_a_live_handle_is_refused_without_a_launch():
    B, L = 256, 10
    eng = TDEngine(L, B, "def", False, 1, device=0, np_seeds=np.arange(B), py_seeds=np.arange(B))
    try:
        eng.reset_all()
        torch.cuda.synchronize()
        before = eng.obs.clone()
        act = torch.zeros(B, dtype=torch.int64, device="cuda")
        sentinel = torch.full((B,), 7, dtype=torch.uint8, device="cuda")
        io = AbiV2StepIO(def_act=act.data_ptr(), obs=eng.obs.data_ptr(), reward=eng.reward.data_ptr(),
                         done=sentinel.data_ptr(), cooldowns=sentinel.data_ptr())
        rc = _lib.lib.td_step(eng._h, ctypes.cast(ctypes.byref(io), ctypes.POINTER(_lib.TdStepIO)),
                              torch.cuda.current_stream().cuda_stream)
        assert rc < 0 and "abi" in _lib.lib.td_last_error().decode()
        torch.cuda.synchronize()
        assert torch.equal(eng.obs, before)
        assert (sentinel == 7).all()
        assert eng.export_state(0, 1)["hdr"][0]["steps"] == 0  # the board did not step
        eng.step(def_act=act)  # the engine's own (ABI-3) struct still steps
        torch.cuda.synchronize()
        assert eng.export_state(0, 1)["hdr"][0]["steps"] == 1
    finally:
        eng.close()
