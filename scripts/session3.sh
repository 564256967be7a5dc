#!/bin/bash
# Staggered-episode bench + kernel trace (refill vs step kernel durations).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > "gpurun_out/s3/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" >&2; tail -3 "gpurun_out/s3/$name.log" >&2; return $rc; }
run bench_stag 300 python bench.py --no-cpu-baseline || exit $?
run bench_nostag 300 python bench.py --no-cpu-baseline --stagger 0 --burnin 600 || exit $?
run kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3/kt -o kt --output-format csv -- python bench.py --no-cpu-baseline --steps 100 || exit $?
exit 0
