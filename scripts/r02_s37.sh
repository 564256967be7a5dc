#!/bin/bash
# Round-2 GPU session 37: where the small-batch step's tail goes -- refills off
# (TD_REFILL_EVERY=0: the four staged layouts per board last the run), auto-reset off
# (diagnostic, not the metric), and a build that polls the next layout's tag early for
# boards ending by the step limit (variants/libtdstep_early.so), at 8,192 / 4,096 boards;
# and the small kernel stepping TD_BPW boards per wave one after another
# (variants/libtdstep_bpw.so: one round of waves at 8,192-65,536 boards).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s37
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), 'flags', d.get('board_flags_nonzero'))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 2000"
V=gym-td_amd/lib/variants
for rep in 1 2; do
  for bb in 8192 4096; do
    run b${bb}_base_$rep 150 $B --global-batch $bb || exit 1
    run b${bb}_early_$rep 150 env TDSTEP_LIB=$V/libtdstep_early.so $B --global-batch $bb || exit 1
    run b${bb}_norefill_$rep 150 env TD_REFILL_EVERY=0 $B --global-batch $bb || exit 1
    run b${bb}_noauto_$rep 150 $B --global-batch $bb --autoreset 0 || exit 1
  done
done
for bb in 8192 16384 32768 65536; do
  for bpw in 1 2 4 8; do
    [ $((bb / bpw)) -lt 4096 ] && continue
    [ $((bb / bpw)) -gt 8192 ] && continue
    run b${bb}_bpw$bpw 150 env TDSTEP_LIB=$V/libtdstep_bpw.so TD_BPW=$bpw $B --global-batch $bb || exit 1
  done
done
run b65536_base 150 $B || exit 1
run b65536_early 150 env TDSTEP_LIB=$V/libtdstep_early.so $B || exit 1
echo "session rc=0"
