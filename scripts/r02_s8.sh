#!/bin/bash
# Round-2 GPU session 8: launch-gap floor; dispatch-bound kernel timing vs marker events;
# refill A/B at 8,192 / 4,096; VALU mix and no-observation / write-through-state variants.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s8
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   ', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'us  frac', round(r['frac'],3))" ; tail -1 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
V=$PWD/gym-td_amd/lib/variants
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32"
run roadgen 300 python -u -m pytest tests/test_gpu_roadgen.py -x -v --timeout 200 --timeout-method thread &&
run gap 60 ./scripts/bin/launch_gap &&
run b8192 120 $B --global-batch 8192 --steps 2000 &&
run b8192_marker 120 $B --global-batch 8192 --steps 2000 --timing marker &&
run b8192_norefill 120 $B --global-batch 8192 --steps 2000 --refill-interval 0 &&
run b4096 120 $B --global-batch 4096 --steps 2000 &&
run b4096_norefill 120 $B --global-batch 4096 --steps 2000 --refill-interval 0 &&
run b65536 120 $B &&
run b8192_sst2 120 env TDSTEP_LIB=$V/libtdstep_sst2.so $B --global-batch 8192 --steps 2000 &&
run b8192_noobs 120 env TDSTEP_LIB=$V/libtdstep_noobs.so $B --global-batch 8192 --steps 2000 &&
run b65536_noobs 120 env TDSTEP_LIB=$V/libtdstep_noobs.so $B &&
run pmc1_8192 120 rocprofv3 --pmc $P1 -d $O/pmc1_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc2_8192 120 rocprofv3 --pmc $P2 -d $O/pmc2_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc1_8192_noobs 120 env TDSTEP_LIB=$V/libtdstep_noobs.so rocprofv3 --pmc $P1 -d $O/pmc1_8192_noobs -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc2_8192_noobs 120 env TDSTEP_LIB=$V/libtdstep_noobs.so rocprofv3 --pmc $P2 -d $O/pmc2_8192_noobs -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300
echo "session rc=$?"
