"""Diagnostic: host time per TDEngine.step (staggered steady state), percentiles."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD.engine import TDEngine
B = int(sys.argv[1])
eng = TDEngine(10, B, "def", False, 1, np_seeds=np.arange(B), py_seeds=np.arange(B), autoreset=True)
eng.reset_all()
for k in range(1, 1200):
    m = (np.arange(B) % 1200) == k
    if m.any():
        eng.reset(m)
acts = torch.randint(0, 601, (400, B), device="cuda")
off = int(sys.argv[2]) if len(sys.argv) > 2 else -1  # sampled timing events at k % 4 == off (-1: none)
stream = torch.cuda.current_stream()
ev = {k: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for k in range(400) if k % 4 == off}
torch.cuda.synchronize()
ts = []
t0 = time.perf_counter()
for k in range(400):
    t = time.perf_counter()
    if k in ev:
        ev[k][0].record(stream)
    eng.step(def_act=acts[k])
    if k in ev:
        ev[k][1].record(stream)
    ts.append(time.perf_counter() - t)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
ts = np.array(ts) * 1e6
print("events at k%%4==%d" % off)
print("B=%d host per step: median %.1f p90 %.1f max %.1f us; loop %.1f us/step; wall %.1f us/step" % (
    B, np.median(ts), np.percentile(ts, 90), ts.max(), (t1 - t0) / 400 * 1e6, (t2 - t0) / 400 * 1e6))
print("slow calls (>100us) at steps:", [int(i) for i in np.nonzero(ts > 100)[0][:20]])
