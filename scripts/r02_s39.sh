#!/bin/bash
# Round-2 GPU session 39: kernel choice on the current build -- the small kernel
# (8 waves/SIMD) against the large one (7) at the N = 2 / 4 shares and 65,536 boards, and
# at 4,096 boards the one-wave small kernel (half the wave slots, room for refill waves)
# against the two-wave one, with refills on and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s39
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), 'flags', d.get('board_flags_nonzero'))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 2000"
for rep in 1 2; do
  for bb in 65536 32768 16384; do
    run b${bb}_large_$rep 150 env TD_SMALL=0 $B --global-batch $bb || exit 1
    run b${bb}_small_$rep 150 env TD_SMALL=1 $B --global-batch $bb || exit 1
  done
  for s in 1 2; do
    run b4096_small${s}_$rep 150 env TD_SMALL=$s $B --global-batch 4096 || exit 1
    run b4096_small${s}_norefill_$rep 150 env TD_SMALL=$s TD_REFILL_EVERY=0 $B --global-batch 4096 || exit 1
  done
  run b8192_small1_$rep 150 env TD_SMALL=1 $B --global-batch 8192 || exit 1
  run b8192_large_$rep 150 env TD_SMALL=0 $B --global-batch 8192 || exit 1
done
echo "session rc=0"
