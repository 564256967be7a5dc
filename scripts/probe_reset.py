"""Probe: time engine creation / reset / refill / steps at growing batch sizes."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD.engine import TDEngine

def log(*a):
    print(*a, flush=True)

for B in [int(x) for x in sys.argv[1:]] or [256, 4096]:
    t = time.time()
    seeds = np.arange(B) + 7000
    eng = TDEngine(10, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    torch.cuda.synchronize(); log(B, "create", time.time() - t)
    t = time.time()
    eng.set_autoreset = None
    from gym_TD import _lib
    _lib.lib.td_set_autoreset(eng._h, 0)
    obs, failed = eng.reset()
    torch.cuda.synchronize(); log(B, "reset(no stage)", time.time() - t, "failed", len(failed))
    _lib.lib.td_set_autoreset(eng._h, 1)
    t = time.time()
    obs, failed = eng.reset()
    torch.cuda.synchronize(); log(B, "reset(+stage)", time.time() - t, "failed", len(failed))
    a = torch.randint(0, 601, (B,), device="cuda")
    for k in range(3):
        t = time.time(); eng.step(def_act=a); torch.cuda.synchronize(); log(B, "step", time.time() - t)
    eng.close()
