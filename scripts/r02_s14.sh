#!/bin/bash
# Round-2 GPU session 14: random_agent=False auto-reset tests + full GPU suite, then the
# refill launch A/B of session 13.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s14
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_envs.py -x -v --timeout 120 --timeout-method thread -k "random_agent" > $O/pytest_ra.log 2>&1; rc=$?
tail -15 $O/pytest_ra.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1; rc=$?
tail -3 $O/pytest_all.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r02_s13.sh
