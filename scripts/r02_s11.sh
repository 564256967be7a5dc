#!/bin/bash
# Round-2 GPU session 11: refill interference A/B at small batches (side-stream priority,
# CU-masked side streams, step-wave issue priority), per-step rate with timing off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s11
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
V=$PWD/gym-td_amd/lib/variants
for rep in 1 2; do
for bb in 8192 4096; do
  run b${bb}_base_$rep 120 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_off_$rep 120 $B --global-batch $bb --steps 3000 --refill-interval 0 || exit 1
  run b${bb}_sideprio_$rep 120 env TD_SIDE_PRIO=1 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_cus8_$rep 120 env TD_SIDE_CUS=8 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_cus32_$rep 120 env TD_SIDE_CUS=32 $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_stepprio_$rep 120 env TDSTEP_LIB=$V/libtdstep_prio.so $B --global-batch $bb --steps 3000 || exit 1
  run b${bb}_both_$rep 120 env TDSTEP_LIB=$V/libtdstep_prio.so TD_SIDE_PRIO=1 $B --global-batch $bb --steps 3000 || exit 1
done
done
run b65536_base 120 $B --steps 300 &&
run b65536_cus32 120 env TD_SIDE_CUS=32 $B --steps 300 &&
run b65536_stepprio 120 env TDSTEP_LIB=$V/libtdstep_prio.so $B --steps 300 &&
run b2p_base 200 $B --workload 2p-middle-multi --steps 500 &&
run b2p_cus32 200 env TD_SIDE_CUS=32 $B --workload 2p-middle-multi --steps 500 &&
run b2p_stepprio 200 env TDSTEP_LIB=$V/libtdstep_prio.so $B --workload 2p-middle-multi --steps 500
echo "session rc=$?"
