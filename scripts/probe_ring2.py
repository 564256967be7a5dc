"""Diagnostic: short-episode auto-reset run; ring state of boards flagged NO_LAYOUT."""
import ctypes, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np, torch
from gym_TD import _lib, params as P
from gym_TD.engine import TDEngine
ov = dict(base_LP=1, defender_init_cost=0, defender_cost_rate=0.02)
for k, v in ov.items():
    setattr(P.config, k, v)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 96
seeds = np.arange(B) + 4000
eng = TDEngine(10, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
eng.reset_all()
fn = _lib.lib.td_debug_ring
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
NW = fn(None, 0, None, 0)  # 3 + NSLOT words
def ring(b):
    out = np.zeros(NW, dtype=np.uint32)
    fn(eng._h, int(b), out.ctypes.data, NW)
    return out[:3].tolist(), [hex(v) for v in out[3:]]
print("after reset", [ring(b) for b in range(3)])
rng = np.random.RandomState(9)
for k in range(200):
    eng.step(def_act=torch.from_numpy(rng.randint(0, 601, size=B).astype(np.int64)))
    f = eng.flags()
    if (f & 8).any():
        bs = np.nonzero(f & 8)[0]
        print("step", k, "flagged", bs.tolist()[:10])
        for b in bs[:4]:
            print("  board", b, ring(b))
        break
print("done")
