#!/bin/bash
# Round-2 GPU session 17: HBM ceiling incl. per-wave contiguous chunks; phase stamps of the
# current small-batch kernel at 4,096 / 8,192 boards.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s17
mkdir -p $O
S=$PWD/gym-td_amd/lib/libtdstep_stamps.so
timeout -k 10 180 ./scripts/bin/hbm_ceiling > $O/hbm_ceiling.log 2>&1; cat $O/hbm_ceiling.log
timeout -k 10 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 4096 10 600 > $O/ph4096.log 2>&1; tail -16 $O/ph4096.log
timeout -k 10 120 env TDSTEP_LIB=$S python scripts/probe_phases.py 8192 10 600 > $O/ph8192.log 2>&1; tail -16 $O/ph8192.log
echo "session rc=$?"
