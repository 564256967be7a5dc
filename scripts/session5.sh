#!/bin/bash
# GPU tests + the three bench workloads (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/s5
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > "gpurun_out/s5/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" >&2; tail -2 "gpurun_out/s5/$name.log" | cut -c1-400 >&2; return $rc; }
run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
for w in ${WLS:-def-small 2p-middle-multi def-large}; do run bench_$w 300 python bench.py --workload $w --no-cpu-baseline || exit $?; done
exit 0
