"""Diagnostic: GPU time of single layout draws (explicit reset kernel, one board),
to size the staged-layout rings against draws the reference never finishes."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD.engine import TDEngine

L = int(sys.argv[1]) if len(sys.argv) > 1 else 10
res = []
for s in range(int(sys.argv[2]) if len(sys.argv) > 2 else 200):
    eng = TDEngine(L, 1, "def", False, 1, np_seeds=[s], py_seeds=[s], autoreset=False)
    for d in range(10):
        torch.cuda.synchronize()
        t = time.perf_counter()
        _, failed = eng.reset()
        torch.cuda.synchronize()
        res.append((time.perf_counter() - t, bool(failed)))
    eng.close()
t = np.array([r[0] for r in res]) * 1e3
f = np.array([r[1] for r in res])
print("draws %d failed %d  ms: median %.3f p99 %.3f max %.3f  failed-draw ms: %s" % (
    len(t), f.sum(), np.median(t), np.percentile(t, 99), t.max(), np.sort(t[f])[::-1][:12].round(2).tolist()))
