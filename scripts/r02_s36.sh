#!/bin/bash
# Round-2 GPU session 36: (1) the GPU parity suite on the enemy-plane zero-row writer;
# (2) cost attribution of the observation writer at 8,192 / 4,096 boards -- diagnostic
# builds (lib/variants, wrong observations by design) that turn one window class into
# broadcast windows (cls0 binary, cls2 enemy, cls3 mixed), drop the enemy planes or the
# writer, against the previous commit's build (head) and the new one (base);
# (3) kernel choice at the N = 2 / 4 shares (32,768 / 16,384 boards): large kernel
# (7 waves/SIMD) vs small (8 waves/SIMD), with and without write-through observations.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s36
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; }
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 2000"
V=gym-td_amd/lib/variants
for rep in 1 2; do
  for bb in 8192 4096; do
    run b${bb}_base_$rep 150 $B --global-batch $bb || exit 1
    for v in head noobs noenemy cls0 cls2 cls3; do
      run b${bb}_${v}_$rep 150 env TDSTEP_LIB=$V/libtdstep_$v.so $B --global-batch $bb || exit 1
    done
  done
done
for bb in 32768 16384; do
  run b${bb}_large 150 env TD_SMALL=0 $B --global-batch $bb || exit 1
  run b${bb}_small 150 env TD_SMALL=1 TD_OBS_WT=0 $B --global-batch $bb || exit 1
  run b${bb}_smallwt 150 env TD_SMALL=1 TD_OBS_WT=1 $B --global-batch $bb || exit 1
  run b${bb}_largewt 150 env TD_SMALL=0 TD_OBS_WT=1 $B --global-batch $bb || exit 1
done
run b65536_base 150 $B || exit 1
echo "session rc=0"
