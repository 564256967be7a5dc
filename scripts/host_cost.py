"""Diagnostic: host-side cost of one env step at small batches (is the step loop
host-bound?).  For each variant: the host time to enqueue N steps (no sync inside;
N small enough that the launch queue never fills), and the wall time per step once the
GPU has drained them.  usage: python scripts/host_cost.py [B] [N]"""
import ctypes
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "gym-td_amd"))

import torch  # noqa: E402

from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
N = int(sys.argv[2]) if len(sys.argv) > 2 else 200
L = 10
eng = TDEngine(L, B, "def", False, 1, np_seeds=range(B), py_seeds=range(B), autoreset=True)
eng.reset_all()
g = torch.Generator(device="cuda").manual_seed(0)
acts = [torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64) for _ in range(N)]
for k in range(50):
    eng.step(def_act=acts[k % N])
torch.cuda.synchronize()
stream = torch.cuda.current_stream().cuda_stream
io = eng._io
fn = _lib.lib.td_step
h = eng._h
ioref = ctypes.byref(io)


def run(name, step, refill):
    eng.set_refill_interval(refill)
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(N):
            step(k)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print("%-34s refill %2d  host enqueue %6.2f us/step   wall %6.2f us/step" % (
        name, refill, (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6), flush=True)


def py_step(k):
    eng.step(def_act=acts[k])


def raw_step(k):
    io.def_act = acts[k].data_ptr()
    fn(h, ioref, stream)


for refill in (0, 4, 16, 64):
    run("TDEngine.step", py_step, refill)
    run("ctypes td_step (actions preset)", raw_step, refill)
eng.close()
