#!/bin/bash
# Round-2 GPU session 13: refill launch A/B -- without the cross-stream event, one side stream,
# few waves; step rate with timing off, then kernel traces of the best.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s14/ab
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
for bb in 8192 4096; do
  run b${bb}_base 120 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_nowait 120 env TD_REFILL_NOWAIT=1 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_side1 120 env TD_SIDE_STREAMS=1 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_w64 120 env TD_REFILL_WAVES=64 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_w64r16 120 env TD_REFILL_WAVES=64 TD_REFILL_EVERY=16 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_w16r16 120 env TD_REFILL_WAVES=16 TD_REFILL_EVERY=16 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_nowait_w64 120 env TD_REFILL_NOWAIT=1 TD_REFILL_WAVES=64 $B --global-batch $bb --steps 3000 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_w64 -o kt --output-format csv -- env TD_REFILL_WAVES=64 $B --global-batch 8192 --steps 2000 > $O/kt_w64.log 2>&1
echo "session rc=$?"
