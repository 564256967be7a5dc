#!/bin/bash
# Round-2 GPU session 22: wave-parallel road generator -- road-table / refill / golden /
# deep / random_agent tests, full suite, then refill cost A/B and explicit-reset time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s22
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_roadgen.py -x -v --timeout 200 --timeout-method thread > $O/pytest_roadgen.log 2>&1; rc=$?
tail -6 $O/pytest_roadgen.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1; rc=$?
tail -3 $O/pytest_all.log
[ $rc -ne 0 ] && exit $rc
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2) if r['avg_kernel_us']==r['avg_kernel_us'] else '-', 'flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
for rep in 1 2; do
  run b8192_on_$rep 120 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_off_$rep 120 $B --global-batch 8192 --steps 3000 --refill-interval 0 || exit 1
  run b4096_on_$rep 120 $B --global-batch 4096 --steps 3000 || exit 1
  run b4096_off_$rep 120 $B --global-batch 4096 --steps 3000 --refill-interval 0 || exit 1
done
run b65536_on 120 $B --steps 300 &&
run b65536_off 120 $B --steps 300 --refill-interval 0 &&
run b2p_on 200 $B --workload 2p-middle-multi --steps 500 &&
run b2p_off 200 $B --workload 2p-middle-multi --steps 500 --refill-interval 0 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt8192 -o kt --output-format csv -- python bench.py --no-cpu-baseline --global-batch 8192 --steps 1000 > $O/kt8192.log 2>&1
echo "session rc=$?"
