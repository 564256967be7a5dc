"""How timing events perturb the step they time (verdict r04, item 1).

    python scripts/probe_timing.py [boards] [burnin]

After bench.py's staggered burn-in, passes of steps back to back: with no events, with
dispatch-bound events (td_kernel_timing) on every 32nd / 8th / every launch.  Prints per
pass the wall time per step and the sampled kernel durations (with each sample's step
number modulo the refill interval, 64: a refill launched behind step 64k runs beside the
next step kernel)."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(HERE, "gym-td_amd"), HERE]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gym_TD.engine import TDEngine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    burnin = int(sys.argv[2]) if len(sys.argv) > 2 else 1200
    L = 10
    seeds = np.arange(B)
    eng = TDEngine(L, B, "def", False, 1, device=0, np_seeds=seeds, py_seeds=seeds, autoreset=True, info=True)
    eng.reset_all()
    g = torch.Generator(device="cuda").manual_seed(1234)
    gidx = np.arange(B)
    for k in range(burnin):
        if 0 < k < 1200:
            m = (gidx % 1200) == k
            if m.any():
                eng.reset(m)
        eng.step(def_act=torch.randint(0, 601, (B,), device="cuda", generator=g, dtype=torch.int64))
    acts = [torch.randint(0, 601, (B,), device="cuda", generator=g, dtype=torch.int64) for _ in range(64)]
    step_no = [burnin]

    def run(n, every):
        if every:
            eng.kernel_timing((n + every - 1) // every, every)
        first = step_no[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(n):
            eng.step(def_act=acts[k % 64])
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n * 1e6
        step_no[0] += n
        out = {"steps": n, "every": every, "wall_us_per_step": wall}
        if every:
            ks = eng.kernel_times().astype(float).tolist()
            eng.kernel_timing(0)
            out.update(kernel_mean_us=float(np.mean(ks)), kernel_median_us=float(np.median(ks)),
                       samples=[[int((first + i * every) % 64), round(v, 2)] for i, v in enumerate(ks)])
        return out

    res = [run(256, 0), run(256, 32), run(256, 0), run(256, 8), run(256, 0), run(128, 1), run(256, 0)]
    print(json.dumps({"boards": B, "kernel": eng.step_kernel_name, "passes": res}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
