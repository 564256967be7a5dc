"""Diagnostic: per-phase wave cycles of the step kernel (TD_STAMPS build) and
timings, at a chosen batch.
Usage: TDSTEP_LIB=.../libtdstep_stamps.so python probe_phases.py B L burnin [mode multi]"""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gym-td_amd"))
import numpy as np, torch
from gym_TD import _lib
from gym_TD.engine import TDEngine

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
L = int(sys.argv[2]) if len(sys.argv) > 2 else 10
burn = int(sys.argv[3]) if len(sys.argv) > 3 else 600
mode = sys.argv[4] if len(sys.argv) > 4 else "def"
multi = len(sys.argv) > 5 and sys.argv[5] == "1"
seeds = np.arange(B) + 11
eng = TDEngine(L, B, mode, multi, 1, np_seeds=seeds, py_seeds=seeds, autoreset=True, info=not multi)
if os.environ.get("TD_PROBE_KERNEL"):  # force a step kernel (td_set_step_kernel)
    eng.set_step_kernel(os.environ["TD_PROBE_KERNEL"])
print("kernel", eng.step_kernel_name)
eng.reset_all()
g = torch.Generator(device="cuda").manual_seed(0)
if multi:  # a few pre-drawn flag batches, cycled (bench.py's 2p-middle-multi shape)
    pool = [(torch.randint(0, 3, (B, 6, L, L), device="cuda", generator=g),
             torch.randint(0, 5, (B, 3, 8), device="cuda", generator=g)) for _ in range(4)]
    act = lambda k: pool[k % 4]
else:
    acts = torch.randint(0, 6 * L * L + 1, (burn + 20, B), device="cuda", generator=g)
    act = lambda k: (acts[k], None)


def step(k):
    d, a = act(k)
    eng.step(def_act=d, atk_act=a if mode != "def" else None)


for k in range(burn):
    step(k)
torch.cuda.synchronize()
stamps = torch.zeros((B, 16), dtype=torch.int64, device="cuda")
fn = getattr(_lib.lib, "td_debug_stamps", None)
if fn is not None:
    fn.restype = _lib.ctypes.c_int
    fn.argtypes = [_lib.c_vp, _lib.c_vp]
    fn(eng._h, stamps.data_ptr())
# stamp slots in time order (td_step.hip STAMP(i)); 9 / 10 are the 100-MHz start / end
order = [0, 1, 11, 12, 2, 3, 4, 5, 13, 14, 6, 7, 8]
names = ["load", "defender", "attacker", "cells+pack", "sort", "towers", "march+costs+done", "enemy_stats",
         "channel_scalars", "state+out", "obs", "-"]
acc = np.zeros(len(names))
t0 = time.time()
for k in range(burn, burn + 20):
    step(k)
    torch.cuda.synchronize()
    if fn is not None:
        s = stamps.cpu().numpy().astype(np.float64)
        d = np.diff(s[:, order], axis=1)
        acc += d.mean(axis=0)
dt = (time.time() - t0) / 20
print("B=%d L=%d step %.1f us" % (B, L, dt * 1e6))
if fn is not None:
    tot = acc.sum()
    for n, v in zip(names, acc / 20):
        print("  %-14s %10.0f cycles/wave  %5.1f%%" % (n, v, 100 * v / (tot / 20)))
    s = stamps.cpu().numpy()
    print("  mean wave life %.0f cycles (s_memtime)" % (s[:, 8] - s[:, 0]).mean())
    # 100-MHz chip clock (slots 9 / 10): wave start / end offsets from the first wave's start, in us
    st0 = s[:, 9].min()
    start = (s[:, 9] - st0) / 100.0
    end = (s[:, 10] - st0) / 100.0
    life = end - start
    pct = lambda v: " ".join("p%d=%.2f" % (q, np.percentile(v, q)) for q in (0, 10, 50, 90, 99, 100))
    print("  rt start us: " + pct(start))
    print("  rt end   us: " + pct(end))
    print("  rt life  us: " + pct(life))
    print("  rt span us: %.2f (first wave start -> last wave end)" % end.max())
    # cycles per realtime tick (shader clock estimate)
    print("  shader clock ~ %.0f MHz" % (100.0 * (s[:, 8] - s[:, 0]).sum() / max(1, (s[:, 10] - s[:, 9]).sum())))
    st = eng.export_state(0, min(B, 4096))
    print("  mean enemies %.2f towers %.2f steps %.0f" % (st["hdr"]["n_en"].mean(), st["hdr"]["n_tw"].mean(), st["hdr"]["steps"].mean()))
    # which boards form the tail: wave life (the last step) by board features
    nb = min(B, 4096)
    lf = life[:nb]
    tw, en, dn = st["hdr"]["n_tw"], st["hdr"]["n_en"], eng.done[:nb].cpu().numpy().astype(bool)
    cyc = (s[:nb, order[1:]] - s[:nb, order[:-1]]).astype(np.float64)
    slow = lf >= np.percentile(lf, 90)
    print("  tail (p90+ life) vs rest: towers %.2f / %.2f, enemies %.2f / %.2f, done %.3f / %.3f" % (
        tw[slow].mean(), tw[~slow].mean(), en[slow].mean(), en[~slow].mean(), dn[slow].mean(), dn[~slow].mean()))
    print("  tail phase cycles: " + " ".join("%s=%.0f/%.0f" % (n, cyc[slow, j].mean(), cyc[~slow, j].mean())
                                           for j, n in enumerate(names[:-1])))
    print("  start us of tail / rest: %.2f / %.2f" % (start[:nb][slow].mean(), start[:nb][~slow].mean()))
