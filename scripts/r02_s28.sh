#!/bin/bash
# Round-2 GPU session 28: follow-mode refills (device-paced, no event on the step stream):
# GPU suite, then step rate A/B against event-anchored refills and refills off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s28
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "session rc=$rc"; exit $rc; }
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
for rep in 1 2; do
  run b8192_follow_$rep 120 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_f4_$rep 120 env TD_REFILL_EVERY=4 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_f64_$rep 120 env TD_REFILL_EVERY=64 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_fw32_$rep 120 env TD_REFILL_WAVES=32 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_event_$rep 120 env TD_REFILL_FOLLOW=0 $B --global-batch 8192 --steps 3000 || exit 1
  run b8192_off_$rep 120 $B --global-batch 8192 --steps 3000 --refill-interval 0 || exit 1
  run b4096_follow_$rep 120 $B --global-batch 4096 --steps 3000 || exit 1
  run b4096_off_$rep 120 $B --global-batch 4096 --steps 3000 --refill-interval 0 || exit 1
done
run b65536_follow 200 $B --steps 300 || exit 1
run b65536_event 200 env TD_REFILL_FOLLOW=0 $B --steps 300 || exit 1
run b65536_fw256 200 env TD_REFILL_WAVES=256 $B --steps 300 || exit 1
run b65536_off 200 $B --steps 300 --refill-interval 0 || exit 1
run b2p_follow 200 $B --workload 2p-middle-multi --steps 300 || exit 1
run b2p_event 200 env TD_REFILL_FOLLOW=0 $B --workload 2p-middle-multi --steps 300 || exit 1
run b2p_off 200 $B --workload 2p-middle-multi --steps 300 --refill-interval 0 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- $B --global-batch 8192 --steps 2000 > $O/kt.log 2>&1 &&
python scripts/kt_gaps.py $O/kt/kt_kernel_trace.csv 2000 --detail > $O/gaps.txt 2>&1
rc=$?
cat $O/gaps.txt
echo "session rc=$rc"
