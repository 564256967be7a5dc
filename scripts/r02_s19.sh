#!/bin/bash
# Round-2 GPU session 19: same-box A/B of wave-level sync (product) vs workgroup barriers
# in the step path, one-wave small kernel, 4,096 / 8,192 boards; and the large kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s19
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
V=$PWD/gym-td_amd/lib/variants
for rep in 1 2; do
  run b4096_wsync_$rep 120 env TD_SMALL=1 $B --global-batch 4096 --steps 3000 || exit 1
  run b4096_barrier_$rep 120 env TD_SMALL=1 TDSTEP_LIB=$V/libtdstep_barrier.so $B --global-batch 4096 --steps 3000 || exit 1
  run b4096_small2_$rep 120 $B --global-batch 4096 --steps 3000 || exit 1
  run b8192_wsync_$rep 120 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_barrier_$rep 120 env TDSTEP_LIB=$V/libtdstep_barrier.so $B --global-batch 8192 --steps 3000 || exit 1
  run b65536_wsync_$rep 120 $B --steps 300 || exit 1
  run b65536_barrier_$rep 120 env TDSTEP_LIB=$V/libtdstep_barrier.so $B --steps 300 || exit 1
done
echo "session rc=$?"
