#!/bin/bash
# Round-2 GPU session 21: refill walk budget per launch (draw residency) vs the step rate.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s21
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
for rep in 1 2; do
  run b8192_w48_$rep 120 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_w12_$rep 120 env TD_REFILL_WALKS=12 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_w4_$rep 120 env TD_REFILL_WALKS=4 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_w1_$rep 120 env TD_REFILL_WALKS=1 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_off_$rep 120 $B --global-batch 8192 --steps 3000 --refill-interval 0 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt_on -o kt --output-format csv -- $B --global-batch 8192 --steps 1000 > $O/kt_on.log 2>&1
echo "session rc=$?"
