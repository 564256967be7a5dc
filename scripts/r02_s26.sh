#!/bin/bash
# Round-2 GPU session 26: rollout-worker hand-off test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s26
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 250 --timeout-method thread > $O/pytest_rollout.log 2>&1; rc=$?
tail -5 $O/pytest_rollout.log
echo "session rc=$rc"
