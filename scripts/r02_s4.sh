#!/bin/bash
# Round-2 GPU session 4: store ceilings at small batches, 8- vs 6-wave build A/B, PMC.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s4
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
W6=$PWD/gym-td_amd/lib/variants/libtdstep_w6.so
B="python bench.py --no-cpu-baseline"
run sp4096 120 ./scripts/storepol 4096 &&
run sp8192 120 ./scripts/storepol 8192 &&
run b4096 120 $B --global-batch 4096 --steps 2000 &&
run b4096_w6 120 env TDSTEP_LIB=$W6 $B --global-batch 4096 --steps 2000 &&
run b8192 120 $B --global-batch 8192 --steps 2000 &&
run b8192_w6 120 env TDSTEP_LIB=$W6 $B --global-batch 8192 --steps 2000 &&
run b65536 120 $B &&
run b65536_w6 120 env TDSTEP_LIB=$W6 $B &&
run pmc1_8192 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmc1_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc2_8192 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d $O/pmc2_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmcf_8192 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmcw_8192 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmc1_65536 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmc1_65536 -o pmc --output-format csv -- $B --steps 10 --burnin 300 &&
run pmc2_65536 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_LDS -d $O/pmc2_65536 -o pmc --output-format csv -- $B --steps 10 --burnin 300 &&
run pmcw_65536 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_65536 -o pmc --output-format csv -- $B --steps 10 --burnin 300 &&
run pmcf_65536 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf_65536 -o pmc --output-format csv -- $B --steps 10 --burnin 300
echo "session rc=$?"
