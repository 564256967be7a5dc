"""Per-launch means of the step kernel's counters from rocprofv3 --pmc / --kernel-trace dirs.

    python scripts/pmc_compare.py gpurun_out/r05_s4 small half noearly

reads <dir>/pmc1_<v>, <dir>/pmc2_<v> (counter_collection.csv) and <dir>/kt_<v>
(kernel_stats.csv) for each variant v and prints one line per counter."""
import collections
import csv
import glob
import os
import sys


def counters(d):
    out, ids = collections.defaultdict(float), set()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "td_step_kernel" in r["Kernel_Name"]:
                out[r["Counter_Name"]] += float(r["Counter_Value"])
                ids.add(r["Dispatch_Id"])
    return {k: v / max(1, len(ids)) for k, v in out.items()}, len(ids)


def kstats(d):
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "td_step_kernel" in r["Name"]:
                return float(r["AverageNs"]) / 1e3, int(r["Calls"])
    return None, 0


def main():
    root, names = sys.argv[1], sys.argv[2:]
    res = {}
    for v in names:
        c = {}
        for p in ("pmc1_", "pmc2_"):
            cc, n = counters(os.path.join(root, p + v))
            c.update(cc)
        c["kernel_us"], c["launches"] = kstats(os.path.join(root, "kt_" + v))
        res[v] = c
    keys = sorted({k for c in res.values() for k in c})
    print("%-22s" % "counter" + "".join("%16s" % v for v in names))
    for k in keys:
        row = []
        for v in names:
            x = res[v].get(k)
            row.append("%16s" % ("-" if x is None else ("%.4g" % x)))
        print("%-22s" % k + "".join(row))
    for v in names:
        c = res[v]
        if c.get("SQ_WAVES"):
            w = c["SQ_WAVES"]
            print("%s per wave: VALU %.0f SALU %.0f LDS %.0f VMEM_WR %.1f cycles %.0f; wait_inst/any %.2f" % (
                v, c.get("SQ_INSTS_VALU", 0) / w, c.get("SQ_INSTS_SALU", 0) / w, c.get("SQ_INSTS_LDS", 0) / w,
                c.get("SQ_INSTS_VMEM_WR", 0) / w, c.get("SQ_WAVE_CYCLES", 0) / w,
                c.get("SQ_WAIT_INST_ANY", 0) / max(1.0, c.get("SQ_WAIT_ANY", 1.0))))


if __name__ == "__main__":
    main()
