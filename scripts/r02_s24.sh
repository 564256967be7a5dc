#!/bin/bash
# Round-2 GPU session 24: two-rank product run (gloo, one GPU) vs one process; N=8 bench
# rehearsal (gloo, 8 ranks on one GPU) of the strong-scaling line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s24
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multiproc.py -x -v --timeout 280 --timeout-method thread > $O/pytest_mp.log 2>&1; rc=$?
tail -4 $O/pytest_mp.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 8 --steps 100 --warmup 10 > $O/bench_n8_rehearsal.log 2>&1; rc=$?
grep '^{' $O/bench_n8_rehearsal.log | cut -c1-600
echo "session rc=$rc"
