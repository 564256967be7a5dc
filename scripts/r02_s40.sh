#!/bin/bash
# Round-2 GPU session 40: refills without the step-stream event (TD_REFILL_NOWAIT=1) at
# several intervals, at 4,096 / 8,192 boards, over 5,000 timed steps (each board ends ~5
# episodes: dry rings show as board flags).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s40
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-26s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), 'flags', d.get('board_flags_nonzero'), d.get('board_flags'), 'eps', d['episodes']['finished'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 5000"
for bb in 4096 8192; do
  run b${bb}_product 150 $B --global-batch $bb || exit 1
  for ev in 1 4 16 64; do
    run b${bb}_nowait_every$ev 150 env TD_REFILL_NOWAIT=1 TD_REFILL_EVERY=$ev $B --global-batch $bb || exit 1
  done
  run b${bb}_every16 150 env TD_REFILL_EVERY=16 $B --global-batch $bb || exit 1
done
echo "session rc=0"
