"""Probe (GPU): how long the device road generator takes per layout draw.

  python scripts/probe_draw.py [B] [L]

A fresh auto-reset engine of B boards is reset: the reset kernel draws each board's
first layout now, then one refill launch fills every ring (16 staged layouts per board,
the first urgent, the rest within the walk budget) with one wave per board.  Run under
`rocprofv3 --kernel-trace --stats`: the refill kernel's duration / 16 is the time of one
draw by a wave alone on its SIMD (B <= 1,024 on a 256-CU part).  The script also times
the reset and the fill with HIP events."""
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "gym-td_amd"))
import torch  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
L = int(sys.argv[2]) if len(sys.argv) > 2 else 10
seeds = list(range(5000, 5000 + B))
eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
eng.reset()
torch.cuda.synchronize()
t1 = time.perf_counter()
act = torch.full((B,), 6 * L * L, dtype=torch.int64, device="cuda")
eng.step(def_act=act)  # the ring guard runs first: it waits for the fill
torch.cuda.synchronize()
t2 = time.perf_counter()
print("B=%d L=%d reset %.3f ms, first step (guard after the fill) %.3f ms" % (B, L, (t1 - t0) * 1e3, (t2 - t1) * 1e3))
eng.close()
