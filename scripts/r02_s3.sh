#!/bin/bash
# Round-2 GPU session 3: line-window observation writer, 8 waves/SIMD, early lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s3
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
S=$PWD/gym-td_amd/lib/libtdstep_stamps.so
run pytest_auto 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
run pytest_noearly 300 env TD_EARLY_OBS=0 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread &&
run b4096 120 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline &&
run b4096_ne 120 env TD_EARLY_OBS=0 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline &&
run b8192 120 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline &&
run b8192_ne 120 env TD_EARLY_OBS=0 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline &&
run b65536 120 python bench.py --no-cpu-baseline &&
run b65536_e 120 env TD_EARLY_OBS=1 python bench.py --no-cpu-baseline &&
run b256 120 python bench.py --global-batch 256 --steps 2000 --no-cpu-baseline &&
run ph256 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 256 10 600 &&
run ph4096 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 4096 10 600 &&
run ph8192 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 8192 10 600 &&
run ph8192_ne 120 env TD_EARLY_OBS=0 TDSTEP_LIB=$S python scripts/probe_phases.py 8192 10 600 &&
run b2p 180 python bench.py --workload 2p-middle-multi --no-cpu-baseline &&
run blarge 180 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline
echo "session rc=$?"
