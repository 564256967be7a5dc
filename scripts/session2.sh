#!/bin/bash
# New GPU tests + the extra bench workloads + a timed window across the episode boundary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" >&2; tail -4 "gpurun_out/$name.log" >&2; return $rc; }
run envtests 600 python -u -m pytest tests/test_gpu_envs.py -m gpu -v --timeout 300 --timeout-method thread || exit $?
run bench_2p 300 python bench.py --workload 2p-middle-multi --steps 50 --warmup 5 --cpu-seconds 10 || exit $?
run bench_large 300 python bench.py --workload def-large --steps 50 --warmup 5 --cpu-seconds 10 || exit $?
run bench_surge 300 python bench.py --burnin 1150 --steps 100 --no-cpu-baseline || exit $?
exit 0
