"""Step-kernel durations and the gaps between consecutive step kernels in a
rocprofv3 --kernel-trace csv (diagnostic).  usage: python scripts/kt_gaps.py TRACE.csv [N]"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
st = [r for r in rows if "td_step_kernel" in r["Kernel_Name"]][-n:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in st]
gap = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(st, st[1:])]
span = (int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1e3 / len(st)
print("steps %d  kernel mean %.1f us  gap mean %.1f us (median %.1f)  span per step %.1f us"
      % (len(st), statistics.mean(dur), statistics.mean(gap), statistics.median(gap), span))
