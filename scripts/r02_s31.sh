#!/bin/bash
# Round-2 GPU session 31: observation-window class table (obs writer) -- parity, then
# A/B against the previous writer at 8,192 / 4,096 / 65,536 boards; host enqueue cost
# with follow-mode vs event-anchored refills.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s31
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && { echo "session rc=$rc"; exit $rc; }
AB_ARGS="--global-batch 8192 --steps 2000 --burnin 1200" timeout -k 10 400 bash scripts/ab_bench.sh 3 new oldobs > $O/ab_8192.log 2>&1 || { cat $O/ab_8192.log; exit 1; }
cat $O/ab_8192.log
AB_ARGS="--global-batch 4096 --steps 2000 --burnin 1200" timeout -k 10 400 bash scripts/ab_bench.sh 2 new oldobs > $O/ab_4096.log 2>&1 || { cat $O/ab_4096.log; exit 1; }
cat $O/ab_4096.log
AB_ARGS="--steps 200" timeout -k 10 400 bash scripts/ab_bench.sh 2 new oldobs > $O/ab_65536.log 2>&1 || { cat $O/ab_65536.log; exit 1; }
cat $O/ab_65536.log
timeout -k 10 200 python scripts/host_cost.py 8192 200 > $O/host_follow.log 2>&1 &&
TD_REFILL_FOLLOW=0 timeout -k 10 200 python scripts/host_cost.py 8192 200 > $O/host_event.log 2>&1
rc=$?
for f in host_follow host_event; do echo "== $f"; grep -v amdgpu.ids $O/$f.log; done
echo "session rc=$rc"
