#!/bin/bash
# Round-2 GPU session 35: kernel choice at the N = 2 / 4 shares (32,768 / 16,384 boards):
# the large kernel (7 waves/SIMD: 4.6 / 2.3 rounds) against the small one (8 waves/SIMD:
# 4 / 2 whole rounds), with and without write-through observation stores.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s35
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 2000"
for rep in 1 2; do
  for bb in 32768 16384; do
    run b${bb}_large_$rep 150 env TD_SMALL=0 $B --global-batch $bb || exit 1
    run b${bb}_small_$rep 150 env TD_SMALL=1 TD_OBS_WT=0 $B --global-batch $bb || exit 1
    run b${bb}_smallwt_$rep 150 env TD_SMALL=1 TD_OBS_WT=1 $B --global-batch $bb || exit 1
    run b${bb}_largewt_$rep 150 env TD_SMALL=0 TD_OBS_WT=1 $B --global-batch $bb || exit 1
  done
done
echo "session rc=0"
