#!/bin/bash
# One GPU session: smoke -> gpu tests -> bench.  Stops after any crash/timeout
# (exit >= 2 other than pytest's 1 = failures).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  tail -5 "gpurun_out/$name.log" >&2
  return $rc
}
STEPS=${STEPS:-smoke,tests,bench}
if [[ $STEPS == *smoke* ]]; then run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?; fi
if [[ $STEPS == *tests* ]]; then run pytest_gpu 1200 python -m pytest tests -m gpu -v -x --timeout 400 ${PYTEST_ARGS}; rc=$?; [ $rc -le 1 ] || exit $rc; fi
if [[ $STEPS == *bench* ]]; then run bench 400 python bench.py ${BENCH_ARGS} || exit $?; fi
exit 0
