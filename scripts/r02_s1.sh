#!/bin/bash
# Round-2 GPU session 1: small-batch evidence for the round-1 kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s1
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$O/$name.log"; return $rc; }
run ph4096 240 env TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so python scripts/probe_phases.py 4096 10 600 &&
run ph8192 240 env TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so python scripts/probe_phases.py 8192 10 600 &&
run b8192 240 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline &&
run b4096 240 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline &&
run b256 240 python bench.py --global-batch 256 --steps 2000 --no-cpu-baseline &&
run b65536 240 python bench.py --no-cpu-baseline &&
run kt8192 300 rocprofv3 --kernel-trace --stats -d $O/kt8192 -o kt --output-format csv -- python bench.py --global-batch 8192 --steps 500 --no-cpu-baseline &&
run pmcf8192 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmcf8192 -o pmc --output-format csv -- python bench.py --global-batch 8192 --steps 20 --burnin 300 --no-cpu-baseline &&
run pmcw8192 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw8192 -o pmc --output-format csv -- python bench.py --global-batch 8192 --steps 20 --burnin 300 --no-cpu-baseline &&
run pmcs8192 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $O/pmcs8192 -o pmc --output-format csv -- python bench.py --global-batch 8192 --steps 20 --burnin 300 --no-cpu-baseline
echo "session rc=$?"
