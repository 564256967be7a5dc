"""Turn a scripts/pmc_ab.sh summary into a profiles/pmc_traffic.json record.

    python scripts/pmc_record.py <pmc_ab dir> <round> [--out profiles/pmc_traffic.json]

The record is keyed "<workload>_B<boards per GPU>" and carries what bench.py matches before
it quotes the bytes (bench.measured_traffic): the kernel-source hash of THIS tree, the step
kernel's name and the observation allocation kind, both read from the bench line that ran
under the counters (<dir>/FETCH_SIZE.log), so a record is never quoted for another build,
kernel or placement."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def bench_line(path):
    for ln in open(path, errors="replace"):
        if ln.startswith('{"metric"'):
            return json.loads(ln)
    raise SystemExit("no bench line in %s" % path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("round")
    ap.add_argument("--out", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    import bench
    summ = json.load(open(os.path.join(a.dir, "summary.json")))
    line = bench_line(os.path.join(a.dir, "FETCH_SIZE.log"))
    kernel = line["roofline"]["kernel"]
    if summ["kernel"].split("<")[0].split("::")[-1].replace("void td::", "") not in kernel.replace("td::", ""):
        raise SystemExit("counter kernel %s is not the bench line's %s" % (summ["kernel"], kernel))
    rec = {"hbm_bytes_per_launch": 2 * summ["FETCH_SIZE"] + summ["WRITE_SIZE"], "read": 2 * summ["FETCH_SIZE"],
           "write": summ["WRITE_SIZE"], "round": a.round, "kernel": kernel,
           "kernel_src": bench.kernel_source_hash(), "obs_alloc": line["config"]["obs_alloc"],
           "launches": summ["launches"], "ratio_to_algorithmic": summ["ratio"]}
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    key = "%s_B%d" % (summ["wl"], summ["B"])
    db[key] = rec
    with open(a.out, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
        f.write("\n")
    print(key, json.dumps(rec))


if __name__ == "__main__":
    main()
