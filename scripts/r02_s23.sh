#!/bin/bash
# Round-2 GPU session 23: few long-lived refill waves (grid-stride over 64-board groups).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s23
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  flags', d['board_flags'])" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --timing none"
for rep in 1 2; do
  for bb in 8192 4096; do
    run b${bb}_w1024_$rep 120 $B --global-batch $bb --steps 3000 || exit 1
    for w in 64 16 8 4; do
      run b${bb}_w${w}_$rep 120 env TD_REFILL_WAVES=$w $B --global-batch $bb --steps 3000 || exit 1
    done
  done
done
run b65536_w1024 120 $B --steps 300 &&
run b65536_w16 120 env TD_REFILL_WAVES=16 $B --steps 300 &&
run b2p_w1024 200 $B --workload 2p-middle-multi --steps 500 &&
run b2p_w16 200 env TD_REFILL_WAVES=16 $B --workload 2p-middle-multi --steps 500
echo "session rc=$?"
