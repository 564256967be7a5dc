#!/bin/bash
# A/B throughput of several builds of libtdstep.so on one GPU box (diagnostic).
# usage: scripts/ab_bench.sh ROUNDS name1 name2 ...   (gym-td_amd/lib/variants/libtdstep_<name>.so)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
R=$1; shift
for r in $(seq 1 $R); do
  for n in "$@"; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$n.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --burnin 300 --no-cpu-baseline ${AB_ARGS} > gpurun_out/ab/$n.$r.json 2> gpurun_out/ab/$n.$r.err || exit $?
    python - "$n" "$r" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab/%s.%s.json" % (sys.argv[1], sys.argv[2])).read().strip().splitlines()[-1])
print("%-10s r%s %8.1fM env-steps/s  step %6.1f us  kernel %6.1f us" % (sys.argv[1], sys.argv[2], d["value"] / 1e6, d["ms_per_step"] * 1e3, d["roofline"]["avg_kernel_us"]), flush=True)
PY
  done
done
