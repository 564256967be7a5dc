#!/bin/bash
# Full GPU test suite + steady-state (staggered) bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > "gpurun_out/s4/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" >&2; tail -3 "gpurun_out/s4/$name.log" >&2; return $rc; }
run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
run bench_stag 300 python bench.py --no-cpu-baseline || exit $?
run kt 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s4/kt -o kt --output-format csv -- python bench.py --no-cpu-baseline --steps 100 || exit $?
exit 0
