#!/bin/bash
# Round-2 GPU session 7: current build — parity suite, bench at 4,096 / 8,192 / 65,536 boards,
# kernel traces and HBM PMC at the small batches.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s7
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
B="python bench.py --no-cpu-baseline"
run pytest 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
run b4096 120 $B --global-batch 4096 --steps 2000 &&
run b8192 120 $B --global-batch 8192 --steps 2000 &&
run b65536 120 $B &&
run kt8192 200 rocprofv3 --kernel-trace --stats -d $O/kt8192 -o kt --output-format csv -- $B --global-batch 8192 --steps 1000 &&
run kt4096 200 rocprofv3 --kernel-trace --stats -d $O/kt4096 -o kt --output-format csv -- $B --global-batch 4096 --steps 1000 &&
run pmcf8192 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmcw8192 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmcs8192 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmcs8192 -o pmc --output-format csv -- $B --global-batch 8192 --steps 20 --burnin 300 &&
run pmcf4096 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf4096 -o pmc --output-format csv -- $B --global-batch 4096 --steps 20 --burnin 300 &&
run pmcw4096 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw4096 -o pmc --output-format csv -- $B --global-batch 4096 --steps 20 --burnin 300
echo "session rc=$?"
