#!/bin/bash
# HBM bytes per step-kernel launch of one build / env variant: separate FETCH_SIZE and
# WRITE_SIZE passes (rocprofv3 --pmc) over a short bench run; prints one summary line.
#   OUT=dir NAME=tag B=boards [WL=workload] bash scripts/pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_ab}; WL=${WL:-def-small}; B=${B:-65536}; NAME=${NAME:-x}
D=$OUT/$NAME; mkdir -p $D
BENCH="python bench.py --workload $WL --steps 20 --warmup 2 --burnin ${BURNIN:-300} --no-cpu-baseline --boards $B"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c -d $D/$c -o pmc --output-format csv -- $BENCH > $D/$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $D/$c.log; exit 1; }
done
python3 - "$D" "$NAME" "$B" "$WL" <<'PY'
import csv, glob, json, sys, collections
d, name, B, wl = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(d + "/" + c + "/**/*counter_collection.csv", recursive=True)[0]
    agg, ids, kern = collections.defaultdict(float), set(), collections.Counter()
    for r in csv.DictReader(open(f)):
        if "td_step_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"]); ids.add(r["Dispatch_Id"]); kern[r["Kernel_Name"].split("(")[0]] += 1
    res[c] = agg[c] / len(ids) * 1024
    res["launches"] = len(ids); res["kernel"] = kern.most_common(1)[0][0]
L = {"def-small": 10, "def-large": 30, "2p-middle-multi": 20}[wl]
alg = B * (45 * L * L * 4 + (6 * L * L * 8 + 24 * 8 if wl == "2p-middle-multi" else 8) + 9)
tot = 2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]
res.update(name=name, B=B, wl=wl, read_2x_MB=2 * res["FETCH_SIZE"] / 1e6, write_MB=res["WRITE_SIZE"] / 1e6,
           total_MB=tot / 1e6, ratio=tot / alg, read_B_per_board=2 * res["FETCH_SIZE"] / B, write_B_per_board=res["WRITE_SIZE"] / B)
json.dump(res, open(d + "/summary.json", "w"))
print("   pmc %-22s B=%d read(2x) %.1f MB (%.0f B/board) write %.1f MB (%.0f B/board) total %.1f MB = %.4fx  [%s, %d launches]" % (
    name, B, res["read_2x_MB"], res["read_B_per_board"], res["write_MB"], res["write_B_per_board"], res["total_MB"], res["ratio"], res["kernel"], res["launches"]))
PY
