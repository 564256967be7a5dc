#!/bin/bash
# Round-2 GPU session 25: four boards per workgroup (fewer workgroups to dispatch) A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s25
mkdir -p $O
timeout -k 10 400 env TD_SMALL=3 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_m.log 2>&1; rc=$?
tail -2 $O/pytest_m.log
[ $rc -ne 0 ] && exit $rc
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
for rep in 1 2; do
  for bb in 8192 4096 2048; do
    run b${bb}_s1_$rep 120 env TD_SMALL=1 $B --global-batch $bb --steps 3000 || exit 1
    run b${bb}_s3_$rep 120 env TD_SMALL=3 $B --global-batch $bb --steps 3000 || exit 1
  done
done
echo "session rc=$?"
