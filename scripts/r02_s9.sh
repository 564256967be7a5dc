#!/bin/bash
# Round-2 GPU session 9: host cost of a step; deep batched parity test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s9
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -12 "$O/$name.log"; return $rc; }
run host8192 120 python scripts/host_cost.py 8192 200 &&
run host4096 120 python scripts/host_cost.py 4096 200 &&
run deep 400 python -u -m pytest tests/test_gpu_deep.py -x -v --timeout 300 --timeout-method thread
echo "session rc=$?"
