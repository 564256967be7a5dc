#!/bin/bash
# Round-2 GPU session 30: host enqueue cost per step, follow-mode vs event-anchored refills.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s30
mkdir -p $O
timeout -k 10 200 python scripts/host_cost.py 8192 200 > $O/follow_200.log 2>&1 &&
timeout -k 10 200 python scripts/host_cost.py 8192 2000 > $O/follow_2000.log 2>&1 &&
TD_REFILL_FOLLOW=0 timeout -k 10 200 python scripts/host_cost.py 8192 200 > $O/event_200.log 2>&1 &&
TD_REFILL_FOLLOW=0 timeout -k 10 200 python scripts/host_cost.py 8192 2000 > $O/event_2000.log 2>&1
rc=$?
for f in follow_200 follow_2000 event_200 event_2000; do echo "== $f"; grep -v amdgpu.ids $O/$f.log; done
echo "session rc=$rc"
