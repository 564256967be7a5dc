#!/bin/bash
# Round-2 GPU session 10: refill launch interval / grid A/B (per-step rate, timing off),
# and the dispatch-sampled kernel timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s10
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-16s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'us  frac', round(r['frac'],3), 'flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
for bb in 8192 4096; do
for rw in "4 1024" "16 1024" "16 256" "16 128" "32 256" "64 256" "0 256"; do
  set -- $rw
  run b${bb}_r$1_w$2 120 env TD_REFILL_EVERY=$1 TD_REFILL_WAVES=$2 $B --global-batch $bb --steps 3000 --timing none || exit 1
done
done
run b8192_disp 120 $B --global-batch 8192 --steps 3000 &&
run b8192_disp_r16 120 env TD_REFILL_EVERY=16 TD_REFILL_WAVES=256 $B --global-batch 8192 --steps 3000 &&
run b65536_r4 120 env TD_REFILL_EVERY=4 TD_REFILL_WAVES=1024 $B --timing none --steps 300 &&
run b65536_r16 120 env TD_REFILL_EVERY=16 TD_REFILL_WAVES=1024 $B --timing none --steps 300 &&
run b65536_r16w256 120 env TD_REFILL_EVERY=16 TD_REFILL_WAVES=256 $B --timing none --steps 300 &&
run b2p_r4 200 env TD_REFILL_EVERY=4 TD_REFILL_WAVES=1024 $B --workload 2p-middle-multi --timing none --steps 500 &&
run b2p_r16 200 env TD_REFILL_EVERY=16 TD_REFILL_WAVES=256 $B --workload 2p-middle-multi --timing none --steps 500 &&
run b2p_r16w1024 200 env TD_REFILL_EVERY=16 TD_REFILL_WAVES=1024 $B --workload 2p-middle-multi --timing none --steps 500
echo "session rc=$?"
