"""Diagnostic: host time per TDEngine.step (tiny batch, kernel time negligible)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD.engine import TDEngine
for B in (64, 8192):
    eng = TDEngine(10, B, "def", False, 1, np_seeds=np.arange(B), py_seeds=np.arange(B), autoreset=True)
    eng.reset_all()
    acts = torch.randint(0, 601, (2000, B), device="cuda")
    for k in range(200):
        eng.step(def_act=acts[k])
    torch.cuda.synchronize()
    t = time.perf_counter()
    for k in range(200, 2000):
        eng.step(def_act=acts[k])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("B=%d host %.1f us/step, wall %.1f us/step" % (B, (t1 - t) / 1800 * 1e6, (t2 - t) / 1800 * 1e6))
    s = torch.cuda.current_stream()
    t = time.perf_counter()
    for k in range(1000):
        s.cuda_stream
    print("  torch.cuda.current_stream().cuda_stream: %.2f us" % ((time.perf_counter() - t) / 1000 * 1e6))
    t = time.perf_counter()
    for k in range(1000):
        torch.cuda.current_stream(eng.device)
    print("  current_stream(dev): %.2f us" % ((time.perf_counter() - t) / 1000 * 1e6))
    eng.close()
