#!/bin/bash
# Profiling session on the GPU box: phase stamps, kernel trace stats, PMC passes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
P=${PROF_DIR:-gpurun_out/prof}
mkdir -p $P
export TMPDIR=/tmp
WL=${WL:-def-small}
B=${B:-65536}
run() { local name=$1 secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" > "$P/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc" >&2; tail -3 "$P/$name.log" >&2; return $rc; }
BENCH="python bench.py --workload $WL --steps 20 --warmup 2 --burnin 100 --no-cpu-baseline --boards $B"
# kernel trace of the bench line's run (default steps; the CPU baseline legs are left out: their
# pool workers are killed at exit under the profiler)
run kt 600 rocprofv3 --kernel-trace --stats -d $P/kt -o kt --output-format csv -- python bench.py --workload $WL --boards $B --no-cpu-baseline || exit $?
run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE -d $P/pmc_fetch -o pmc --output-format csv -- $BENCH || exit $?
run pmc_write 400 rocprofv3 --pmc WRITE_SIZE -d $P/pmc_write -o pmc --output-format csv -- $BENCH || exit $?
run pmc_sq1 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $P/pmc_sq1 -o pmc --output-format csv -- $BENCH || exit $?
run pmc_sq2 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $P/pmc_sq2 -o pmc --output-format csv -- $BENCH || exit $?
exit 0
