"""Summarise a profile_session.sh run (gpurun_out/prof) into profiles/.

  [PMC_PROF=dir] [PMC_OUT=dir] python scripts/pmc_summary.py ROUND [B] [WORKLOAD]

writes profiles/<ROUND>_kernel_stats.csv (rocprofv3 --kernel-trace --stats),
profiles/<ROUND>_pmc.json (per-launch counter means of the step kernel) and
updates profiles/pmc_traffic.json["<WORKLOAD>_B<B>"] (bench.py's key) with the HBM bytes per launch:
(2 x FETCH_SIZE + WRITE_SIZE) x 1024 -- FETCH_SIZE / WRITE_SIZE are in KiB and
FETCH_SIZE counts half the bytes of 16-B-per-lane reads on gfx950
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section).
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.environ.get("PMC_PROF", os.path.join(HERE, "gpurun_out", "prof"))


def kernel_label(name):
    """'void td::td_step_kernel_small<10, 0, false>(td::StepArgs)' -> the name bench.py
    reports (td_step_kernel_name): 'td_step_kernel_small<10, 0, false>'."""
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    if name.startswith("td::"):
        name = name[4:]
    return name.split("(")[0]


def step_counters(name):
    path = os.path.join(PROF, name, "pmc_counter_collection.csv")
    agg, ids, names = collections.defaultdict(float), set(), collections.Counter()
    for r in csv.DictReader(open(path)):
        if "td_step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            ids.add(r["Dispatch_Id"])
            names[kernel_label(r["Kernel_Name"])] += 1
    return {k: v / len(ids) for k, v in agg.items()}, len(ids), names.most_common(1)[0][0]


def main():
    rnd = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    wl = sys.argv[3] if len(sys.argv) > 3 else "def-small"
    out = os.environ.get("PMC_OUT", os.path.join(HERE, "profiles"))
    tag = (rnd if wl == "def-small" else "%s_%s" % (rnd, wl)) + ("" if B == 65536 or wl != "def-small" else "_b%d" % B)
    shutil.copy(os.path.join(PROF, "kt", "kt_kernel_stats.csv"), os.path.join(out, "%s_kernel_stats.csv" % tag))
    pmc, launches, kernels = {}, {}, set()
    for n in ("pmc_fetch", "pmc_write", "pmc_sq1", "pmc_sq2"):
        if os.path.exists(os.path.join(PROF, n)):
            c, k, kn = step_counters(n)
            pmc.update(c)
            launches[n] = k
            kernels.add(kn)
    assert len(kernels) == 1, kernels  # every pass profiled the same step kernel
    kernel = kernels.pop()
    fetch = pmc["FETCH_SIZE"] * 2 * 1024
    write = pmc["WRITE_SIZE"] * 1024
    summary = {
        "kernel": kernel, "boards": B, "launches_per_pass": launches,
        "counters_per_launch": pmc,
        "hbm_read_bytes_per_launch": fetch, "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "per_board": {"read_bytes": fetch / B, "write_bytes": write / B,
                      "valu_insts": pmc.get("SQ_INSTS_VALU", 0) / B, "salu_insts": pmc.get("SQ_INSTS_SALU", 0) / B},
    }
    json.dump(summary, open(os.path.join(out, "%s_pmc.json" % tag), "w"), indent=1)
    tp = os.path.join(out, "pmc_traffic.json")
    if not os.path.exists(tp) and os.path.exists(os.path.join(HERE, "profiles", "pmc_traffic.json")):
        shutil.copy(os.path.join(HERE, "profiles", "pmc_traffic.json"), tp)
    tj = json.load(open(tp)) if os.path.exists(tp) else {}
    sys.path.insert(0, HERE)
    import bench  # noqa: E402  (the kernel-source hash bench.py checks before quoting this record)
    tj["%s_B%d" % (wl, B)] = {"hbm_bytes_per_launch": fetch + write, "read": fetch, "write": write, "round": rnd,
                              "kernel": kernel, "kernel_src": bench.kernel_source_hash()}
    json.dump(tj, open(tp, "w"), indent=1)
    print(json.dumps({k: summary[k] for k in ("hbm_read_bytes_per_launch", "hbm_write_bytes_per_launch", "per_board")}))


if __name__ == "__main__":
    main()
