#!/bin/bash
# Round-2 GPU session 2: realtime wave timelines at small batches, refill A/B,
# and the N>1 bench control flow rehearsed on one GPU (gloo, same device).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s2
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$O/$name.log"; return $rc; }
S=$PWD/gym-td_amd/lib/libtdstep_stamps.so
run ph256 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 256 10 600 &&
run ph1024 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 1024 10 600 &&
run ph4096 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 4096 10 600 &&
run ph8192 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 8192 10 600 &&
run ph65536 180 env TDSTEP_LIB=$S python scripts/probe_phases.py 65536 10 600 &&
run b4096_noar 120 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline --autoreset 0 &&
run b8192_noar 120 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline --autoreset 0 &&
run b256_noar 120 python bench.py --global-batch 256 --steps 2000 --no-cpu-baseline --autoreset 0 &&
run n2 300 env TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 &&
run n8 400 env TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8
echo "session rc=$?"
