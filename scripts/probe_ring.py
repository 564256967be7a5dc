"""Diagnostic: long staggered rollout, then the ring state of boards flagged NO_LAYOUT."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD import _lib
from gym_TD.engine import TDEngine
B, L, steps = int(sys.argv[1]), 10, int(sys.argv[2])
seeds = np.arange(B)
eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
eng.reset_all()
for k in range(1, 1200):
    m = (np.arange(B) % 1200) == k
    if m.any():
        eng.reset(m)
g = torch.Generator(device="cuda").manual_seed(0)
fn = _lib.lib.td_debug_ring
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
NW = fn(None, 0, None, 0)  # 3 + NSLOT words
prev = np.zeros(B, dtype=np.int32)
t = time.time()
for k in range(steps):
    eng.step(def_act=torch.randint(0, 601, (B,), device="cuda", generator=g))
    if k == steps - 1:
        f = eng.flags()
        new = np.nonzero((f & 8) & ~(prev & 8))[0]
        print("flagged", len(new))
        for b in new[:12]:
            out = np.zeros(NW, dtype=np.uint32)
            fn(eng._h, int(b), out.ctypes.data, NW)
            st = eng.board_state(int(b))
            print("step %d board %d head %d tail %d claim %d tags %s ep_steps %d base_LP %d" % (
                k, b, out[0], out[1], out[2], [hex(v) for v in out[3:]], st["steps"], st["base_LP"]), flush=True)
        prev = f
print("done %.1fs, flagged %d" % (time.time() - t, int(((eng.flags() & 8) != 0).sum())))
