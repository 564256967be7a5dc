#!/bin/bash
# Round-2 GPU session 46: ordered refills at a longer interval (TD_REFILL_EVERY=32: every
# launch still behind the step stream's event, 96 walks per launch) -- the GPU suite
# under that setting (auto-reset under load included), then 5,000-step lines at 4,096 /
# 8,192 / 65,536 boards against the product's every-16th-step refills.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s46
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -5 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])"; }
run pytest_gpu_e32 600 env TD_REFILL_EVERY=32 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
tail -1 $O/pytest_gpu_e32.log
B="python bench.py --no-cpu-baseline --steps 5000"
for rep in 1 2; do
  for bb in 4096 8192 65536; do
    run b${bb}_e16_$rep 200 $B --global-batch $bb || exit 1; line b${bb}_e16_$rep
    run b${bb}_e32_$rep 200 env TD_REFILL_EVERY=32 $B --global-batch $bb || exit 1; line b${bb}_e32_$rep
    run b${bb}_e64_$rep 200 env TD_REFILL_EVERY=64 $B --global-batch $bb || exit 1; line b${bb}_e64_$rep
  done
done
echo "session rc=0"
