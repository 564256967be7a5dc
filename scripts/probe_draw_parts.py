"""Probe (GPU, diagnostic build): where the device road generator's time goes.

  TDSTEP_LIB=gym-td_amd/lib/variants/libtdstep_genstamps.so python scripts/probe_draw_parts.py [B] [L]

(make -C gym-td_amd/csrc variant NAME=genstamps VFLAGS=-DTD_GEN_STAMPS.)  A fresh engine
of B boards is reset (the reset kernel draws each board's first layout) and its rings
filled by one refill launch (15 more draws per board); the generator's s_memtime
counters, summed per board: walks, the branch-loop proof, stamping, erasing, stream
windows, and the whole wave_layout call."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "gym-td_amd"))
import torch  # noqa: E402
from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
L = int(sys.argv[2]) if len(sys.argv) > 2 else 10
seeds = list(range(5000, 5000 + B))
eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
st = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
fn = _lib.lib.td_debug_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
fn.restype = ctypes.c_int
assert fn(eng._h, st.data_ptr()) == 0
eng.reset()
act = torch.full((B,), 6 * L * L, dtype=torch.int64, device="cuda")
eng.step(def_act=act)
torch.cuda.synchronize()
s = st.cpu().numpy().astype(np.float64)
calls = s[:, 7].sum()
names = ["walk", "proof", "stamp", "erase", "window", "walks"]
tot = s[:, 6].sum()
print("B=%d L=%d wave_layout calls %d, cycles per call %.0f" % (B, L, calls, tot / max(calls, 1)))
for i, nme in enumerate(names):
    if nme == "walks":
        print("  walks per call %.2f, cycles per walk %.0f" % (s[:, 5].sum() / calls, s[:, 0].sum() / max(s[:, 5].sum(), 1)))
    else:
        print("  %-7s %10.0f cycles per call  %5.1f %%" % (nme, s[:, i].sum() / calls, 100 * s[:, i].sum() / tot))
eng.close()
