"""Step-kernel durations and the gaps between consecutive step kernels in a
rocprofv3 --kernel-trace csv (diagnostic).  usage: python scripts/kt_gaps.py TRACE.csv [N] [--detail]

--detail: the other kernels (refill / autoreset) by queue, their durations, and for the
largest gaps the kernels that overlap them."""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 100
st = [r for r in rows if "td_step_kernel" in r["Kernel_Name"]][-n:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in st]
gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(st, st[1:])]
span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3 / len(st)
print("steps %d  kernel mean %.1f us  gap mean %.1f us (median %.1f)  span per step %.1f us"
      % (len(st), statistics.mean(dur), statistics.mean(gap), statistics.median(gap), span))
if "--detail" in sys.argv:
    t0, t1 = int(st[0]["Start_Timestamp"]), int(st[-1]["End_Timestamp"])
    qkey = "Queue_Id" if "Queue_Id" in st[0] else None
    print("step kernel queues:", sorted({r.get(qkey) for r in st}) if qkey else "n/a")
    other = [r for r in rows if "td_step_kernel" not in r["Kernel_Name"]
             and int(r["End_Timestamp"]) >= t0 and int(r["Start_Timestamp"]) <= t1]
    byname = {}
    for r in other:
        nm = r["Kernel_Name"].split("(")[0][:48] + " q" + str(r.get(qkey, "?"))
        byname.setdefault(nm, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for nm, d in sorted(byname.items()):
        print("  %-60s n %5d  mean %8.1f us  median %8.1f  max %8.1f" % (nm, len(d), statistics.mean(d),
                                                                         statistics.median(d), max(d)))
    big = sorted(range(len(gap)), key=lambda i: -gap[i])[:12]
    hist = [0, 0, 0, 0, 0]
    for g in gap:
        hist[0 if g < 1 else 1 if g < 5 else 2 if g < 20 else 3 if g < 50 else 4] += 1
    print("gap histogram  <1us %d  1-5 %d  5-20 %d  20-50 %d  >=50 %d" % tuple(hist))
    for i in sorted(big):
        a, b = int(st[i]["End_Timestamp"]), int(st[i + 1]["Start_Timestamp"])
        ov = [r for r in other if int(r["Start_Timestamp"]) < b and int(r["End_Timestamp"]) > a - 60000]
        desc = "; ".join("%s q%s [%+.1f, %+.1f]" % (r["Kernel_Name"].split("(")[0][-22:], r.get(qkey, "?"),
                                                     (int(r["Start_Timestamp"]) - a) / 1e3,
                                                     (int(r["End_Timestamp"]) - a) / 1e3) for r in ov)
        print("  step %5d gap %7.1f us | %s" % (i, gap[i], desc))
