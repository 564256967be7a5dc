#!/bin/bash
# Round-2 GPU session 18: wave-level sync in the step path + the two-wave small-batch
# kernel (4,096 boards): parity suite, then small-batch A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s18
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1; rc=$?
tail -3 $O/pytest_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env TD_SMALL=2 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_small2.log 2>&1; rc=$?
tail -3 $O/pytest_small2.log
[ $rc -ne 0 ] && exit $rc
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
for rep in 1 2; do
  run b4096_s2_$rep 120 $B --global-batch 4096 --steps 3000 || exit 1
  run b4096_s1_$rep 120 env TD_SMALL=1 $B --global-batch 4096 --steps 3000 || exit 1
  run b2048_s2_$rep 120 $B --global-batch 2048 --steps 3000 || exit 1
  run b2048_s1_$rep 120 env TD_SMALL=1 $B --global-batch 2048 --steps 3000 || exit 1
  run b8192_$rep 120 $B --global-batch 8192 --steps 3000 || exit 1
done
run b65536 120 $B --steps 300
echo "session rc=$?"
