"""Does the observation's placement change the write-bound step?  (some
processes stepped 30x30 / 16,384 boards in 448-454 us instead of 496-520.)

    python scripts/probe_offset.py L B steps [offsets...]

One physically contiguous td_alloc_device block; the engine's observation is a view of it
at each byte offset in turn (16-B aligned), the same boards and actions stepped on every
offset; prints the wall time per step for each."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "gym-td_amd"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_TD import _lib  # noqa: E402
from gym_TD.engine import TDEngine, device_zeros  # noqa: E402


def main():
    L, B, steps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    offs = [int(v) for v in sys.argv[4:]] or [0, 256, 1024, 4096, 16384, 65536, 262144, 1 << 20, 2 << 20, 3 << 20]
    n = B * 45 * L * L
    pad = (max(offs) + 15) // 4 + 1024
    block = device_zeros((n + pad,), torch.float32, "cuda", contiguous=True)
    seeds = np.arange(B)
    eng = TDEngine(L, B, "def", False, 1, device=0, np_seeds=seeds, py_seeds=seeds, autoreset=True)
    eng.reset_all()
    g = torch.Generator(device="cuda").manual_seed(7)
    acts = [torch.randint(0, 6 * L * L + 1, (B,), device="cuda", generator=g, dtype=torch.int64) for _ in range(16)]
    for k in range(200):  # burn-in
        eng.step(def_act=acts[k % 16])
    res = []
    for rep in range(2):
        for off in offs:
            view = block[off // 4: off // 4 + n].view(B, 45, L, L)
            eng.obs = view
            eng._io.obs = view.data_ptr()
            for k in range(20):
                eng.step(def_act=acts[k % 16])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(steps):
                eng.step(def_act=acts[k % 16])
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / steps * 1e6
            res.append({"offset": off, "rep": rep, "us_per_step": round(us, 2),
                        "phys_hint": hex(view.data_ptr() & 0xFFFFFFF)})
            print(json.dumps(res[-1]), flush=True)
    print("kernel", eng.step_kernel_name, "B", B, "L", L)
    eng.close()


if __name__ == "__main__":
    main()
