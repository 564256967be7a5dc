#!/bin/bash
# Round-2 GPU session 6: single-phase writer; wt A/B; instruction counts with / without the observation.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s6
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); print('   ', round(d['value']/1e6,1), 'M/s kernel', round(d['roofline']['avg_kernel_us'],1), 'us frac', round(d['roofline']['frac'],3))" ; tail -1 "$O/$name.log"; return $rc; }
NO=$PWD/gym-td_amd/lib/variants/libtdstep_noobs.so
B="python bench.py --no-cpu-baseline"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES"
run pytest_auto 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
run pytest_big 300 env TD_SMALL=0 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread &&
run b4096 120 $B --global-batch 4096 --steps 2000 &&
run b4096_nowt 120 env TD_OBS_WT=0 $B --global-batch 4096 --steps 2000 &&
run b8192 120 $B --global-batch 8192 --steps 2000 &&
run b8192_nowt 120 env TD_OBS_WT=0 $B --global-batch 8192 --steps 2000 &&
run b8192_noobs 120 env TDSTEP_LIB=$NO $B --global-batch 8192 --steps 2000 &&
run b65536 120 $B &&
run b65536_noobs 120 env TDSTEP_LIB=$NO $B &&
run pmc_8192 120 rocprofv3 --pmc $P1 -d $O/pmc_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc_8192_noobs 120 env TDSTEP_LIB=$NO rocprofv3 --pmc $P1 -d $O/pmc_8192_noobs -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc_65536 120 rocprofv3 --pmc $P1 -d $O/pmc_65536 -o pmc --output-format csv -- $B --steps 10 --burnin 300
echo "session rc=$?"
