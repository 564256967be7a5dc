#!/bin/bash
# Round-2 GPU session 45: the round's final build (a refill every 16th step, each ordered behind the
# step stream):
# GPU parity suite, smoke, the default bench line, the strong-scaling shares,
# 2p-middle-multi / def-large, and a 20,000-step run at 8,192 boards for dry rings.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s45
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -5 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])"; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
tail -1 $O/pytest_gpu.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 $O/smoke.log
run bench_default 300 python bench.py || exit 1
grep '^{' $O/bench_default.log
for bb in 32768 16384 8192 4096; do
  run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 || exit 1
  line b$bb
done
run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 2000 || exit 1
line p2
run large 300 python bench.py --workload def-large --no-cpu-baseline --steps 500 || exit 1
line large
run b8192_long 300 python bench.py --global-batch 8192 --no-cpu-baseline --steps 20000 || exit 1
line b8192_long
echo "session rc=0"
