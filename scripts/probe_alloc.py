"""Probe (GPU): does the 30x30 step time depend on where its buffers landed?

  python scripts/probe_alloc.py [L] [B] [engines] [buffers]

Round 4 saw the same 30x30 build step 16,384 boards in 517-520 us in most processes and
453-467 us in a few (r04/s2, r04/s21).  This times the step (a) over several observation
buffers in one process (fresh allocations and offsets of one large allocation), and
(b) over several engines created one after another (fresh state arrays), to tell
placement-dependent time from box-dependent time."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "gym-td_amd"))
import torch  # noqa: E402
from gym_TD.engine import TDEngine  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 30
B = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
NE = int(sys.argv[3]) if len(sys.argv) > 3 else 3
NB = int(sys.argv[4]) if len(sys.argv) > 4 else 6
STEPS = 40


def timed(eng, g, n=STEPS):
    act = [torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64) for _ in range(n)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in act:
        eng.step(def_act=a)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def obs_info(t):
    p = t.data_ptr()
    return "base %#x (mod 2M %#x)" % (p, p % (2 << 20))


MODE = os.environ.get("PROBE_MODE", "torch")
g = torch.Generator(device="cuda").manual_seed(5)
if MODE == "hip":  # raw allocations: hipExtMallocWithFlags default (0) vs contiguous (4)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    seeds = np.arange(B)
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    eng.reset_all()
    for _ in range(4):
        timed(eng, g, 50)
    print("engine (%s): own obs %s  %.1f us" % (eng.step_kernel_name, obs_info(eng.obs), timed(eng, g)), flush=True)
    own = eng._io.obs
    nbytes = B * 45 * L * L * 4
    held = []
    flag_set = [int(f) for f in os.environ.get("PROBE_FLAGS", "0,4").split(",")]
    for rep in range(int(os.environ.get("PROBE_REPS", "3"))):
        for flags in flag_set:
            ptr = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(nbytes), ctypes.c_uint(flags))
            if rc != 0:
                print("  flags %d: hipExtMallocWithFlags rc %d" % (flags, rc), flush=True)
                continue
            held.append(ptr)
            eng._io.obs = ptr.value
            timed(eng, g, 10)
            print("  flags %d: base %#x  %.1f us" % (flags, ptr.value, timed(eng, g)), flush=True)
    eng._io.obs = own
    torch.cuda.synchronize()
    for ptr in held:
        hip.hipFree(ptr)
    eng.close()
    sys.exit(0)
for ei in range(NE):
    seeds = np.arange(B) + 100 * ei
    eng = TDEngine(L, B, "def", False, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    eng.reset_all()
    for _ in range(4):  # burn-in towards the steady state
        timed(eng, g, 50)
    print("engine %d (%s): own obs %s  %.1f us" % (ei, eng.step_kernel_name, obs_info(eng.obs), timed(eng, g)), flush=True)
    keep = []
    n = B * 45 * L * L
    for bi in range(NB):
        if bi % 2 == 0:  # a fresh allocation
            o = torch.empty((B, 45, L, L), dtype=torch.float32, device="cuda")
        else:  # the next buffer at an offset inside one larger allocation
            off = [1024, 64 << 10, 1 << 20][(bi // 2) % 3] // 4
            big = torch.empty(n + off, dtype=torch.float32, device="cuda")
            o = big[off:].view(B, 45, L, L)
            keep.append(big)
        keep.append(o)
        eng.obs = o
        eng._io.obs = o.data_ptr()
        timed(eng, g, 10)
        print("  obs buffer %d: %s  %.1f us" % (bi, obs_info(o), timed(eng, g)), flush=True)
    eng.close()
    del keep
    torch.cuda.empty_cache()
