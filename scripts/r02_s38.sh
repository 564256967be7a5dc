#!/bin/bash
# Round-2 GPU session 38: the small kernel stepping TD_BPW boards per wave one after
# another (variants/libtdstep_bpw.so, arguments read through the kernarg segment pointer
# inside the board loop): one round of waves at 8,192-65,536 boards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s38
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), 'flags', d.get('board_flags_nonzero'))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline --steps 2000"
V=gym-td_amd/lib/variants
run b8192_bpw1_probe 120 env TDSTEP_LIB=$V/libtdstep_bpw.so TD_BPW=1 python bench.py --no-cpu-baseline --steps 20 --burnin 20 --global-batch 8192 || exit 1
for bb in 8192 16384 32768 65536; do
  for bpw in 1 2 4 8; do
    [ $((bb / bpw)) -lt 4096 ] && continue
    [ $((bb / bpw)) -gt 8192 ] && continue
    run b${bb}_bpw$bpw 150 env TDSTEP_LIB=$V/libtdstep_bpw.so TD_BPW=$bpw $B --global-batch $bb || exit 1
  done
  run b${bb}_base 150 $B --global-batch $bb || exit 1
done
echo "session rc=0"
