#!/bin/bash
# Round-2 GPU session 34 (re-entry): GPU parity suite on the rebuilt tree, then the
# strong-scaling per-GPU shares (65,536 / N boards for N = 1, 2, 4, 8) and configs[1].
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s34
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -5 "$O/$name.log"; return $rc; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
tail -3 $O/pytest_gpu.log
for B in 65536 32768 16384 8192 4096; do
  run bench_$B 200 python bench.py --global-batch $B --no-cpu-baseline --steps 1000 || exit 1
  grep '^{' $O/bench_$B.log
done
echo "session rc=0"
