#!/bin/bash
# Round-2 GPU session 16: HBM write/read ceiling sweep; large-kernel live-slot prefetch A/B
# (bench + HBM PMC) at 65,536 10x10, 16,384 20x20 multi-action and 16,384 30x30.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s16
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-22s' % '$name', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3))" ; [ $rc -ne 0 ] && tail -3 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
V=$PWD/gym-td_amd/lib/variants
timeout -k 10 120 ./scripts/bin/hbm_ceiling > $O/hbm_ceiling.log 2>&1; cat $O/hbm_ceiling.log
for rep in 1 2; do
  run b65536_pf0_$rep 120 $B --steps 300 || exit 1
  run b65536_pf16_$rep 120 env TDSTEP_LIB=$V/libtdstep_pf16.so $B --steps 300 || exit 1
done
run b2p_pf0 200 $B --workload 2p-middle-multi --steps 300 &&
run b2p_pf16 200 env TDSTEP_LIB=$V/libtdstep_pf16.so $B --workload 2p-middle-multi --steps 300 &&
run blarge_pf0 200 $B --workload def-large --global-batch 16384 --steps 200 &&
run blarge_pf16 200 env TDSTEP_LIB=$V/libtdstep_pf16.so $B --workload def-large --global-batch 16384 --steps 200 &&
run pmcf_pf0 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_pf0 -o pmc --output-format csv -- $B --steps 10 --burnin 1200 &&
run pmcw_pf0 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_pf0 -o pmc --output-format csv -- $B --steps 10 --burnin 1200 &&
run pmcf_pf16 120 env TDSTEP_LIB=$V/libtdstep_pf16.so rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_pf16 -o pmc --output-format csv -- $B --steps 10 --burnin 1200 &&
run pmcw_pf16 120 env TDSTEP_LIB=$V/libtdstep_pf16.so rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_pf16 -o pmc --output-format csv -- $B --steps 10 --burnin 1200
echo "session rc=$?"
