#!/bin/bash
# Round-2 GPU session 5: small-batch kernel (8 waves, early lines, write-through obs) vs large-batch kernel.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s5
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -h '^{' "$O/$name.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); print('   ', round(d['value']/1e6,1), 'M/s kernel', round(d['roofline']['avg_kernel_us'],1), 'us frac', round(d['roofline']['frac'],3))" ; tail -1 "$O/$name.log"; return $rc; }
S=$PWD/gym-td_amd/lib/libtdstep_stamps.so
B="python bench.py --no-cpu-baseline"
run pytest_auto 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread &&
run pytest_big 300 env TD_SMALL=0 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread &&
run pytest_small_noearly 300 env TD_EARLY_OBS=0 TD_OBS_WT=0 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread &&
run b4096 120 $B --global-batch 4096 --steps 2000 &&
run b4096_nowt 120 env TD_OBS_WT=0 $B --global-batch 4096 --steps 2000 &&
run b4096_noearly 120 env TD_EARLY_OBS=0 $B --global-batch 4096 --steps 2000 &&
run b4096_big 120 env TD_SMALL=0 $B --global-batch 4096 --steps 2000 &&
run b8192 120 $B --global-batch 8192 --steps 2000 &&
run b8192_nowt 120 env TD_OBS_WT=0 $B --global-batch 8192 --steps 2000 &&
run b8192_noearly 120 env TD_EARLY_OBS=0 $B --global-batch 8192 --steps 2000 &&
run b8192_big 120 env TD_SMALL=0 $B --global-batch 8192 --steps 2000 &&
run b65536 120 $B &&
run b16384 120 $B --global-batch 16384 --steps 1000 &&
run b256 120 $B --global-batch 256 --steps 2000 &&
run ph4096 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 4096 10 600 &&
run ph8192 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 8192 10 600 &&
run b2p 180 $B --workload 2p-middle-multi &&
run blarge 180 $B --workload def-large --global-batch 16384
echo "session rc=$?"
