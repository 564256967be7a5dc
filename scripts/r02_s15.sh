#!/bin/bash
# Round-2 GPU session 15: config-epoch capture -- paramConfig test, full GPU suite, smoke, bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s15
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_envs.py -x -v --timeout 120 --timeout-method thread -k "paramconfig or export_import or board_view" > $O/pytest_cfg.log 2>&1; rc=$?
tail -8 $O/pytest_cfg.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1; rc=$?
tail -3 $O/pytest_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log &&
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/b65536.log 2>&1 && tail -1 $O/b65536.log | cut -c1-400 &&
timeout -k 10 200 python bench.py --no-cpu-baseline --global-batch 8192 --steps 2000 > $O/b8192.log 2>&1 && tail -1 $O/b8192.log | cut -c1-400
echo "session rc=$?"
