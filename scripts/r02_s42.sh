#!/bin/bash
# Round-2 GPU session 42: refill pacing with the step-stream event on every k-th refill
# launch only (TD_REFILL_WAIT_EVERY=k; between them refills are not ordered after a
# step), 5,000 timed steps: step time and dry rings (no_layout flags) at 4,096 / 8,192 /
# 65,536 boards and 2p-middle-multi.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s42
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-26s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 5000"
for rep in 1 2; do
  for bb in 4096 8192 65536; do
    run b${bb}_product_$rep 200 $B --global-batch $bb || exit 1
    run b${bb}_e16w4_$rep 200 env TD_REFILL_EVERY=16 TD_REFILL_WAIT_EVERY=4 $B --global-batch $bb || exit 1
    run b${bb}_e8w8_$rep 200 env TD_REFILL_EVERY=8 TD_REFILL_WAIT_EVERY=8 $B --global-batch $bb || exit 1
    run b${bb}_e4w16_$rep 200 env TD_REFILL_EVERY=4 TD_REFILL_WAIT_EVERY=16 $B --global-batch $bb || exit 1
  done
done
run p2_product 300 python bench.py --no-cpu-baseline --workload 2p-middle-multi --steps 3000 || exit 1
run p2_e16w4 300 env TD_REFILL_EVERY=16 TD_REFILL_WAIT_EVERY=4 python bench.py --no-cpu-baseline --workload 2p-middle-multi --steps 3000 || exit 1
echo "session rc=0"
