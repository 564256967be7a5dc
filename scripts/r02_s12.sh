#!/bin/bash
# Round-2 GPU session 12: kernel traces at 8,192 boards with refills on / off.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s12
mkdir -p $O
B="python bench.py --no-cpu-baseline --timing none --global-batch 8192 --steps 2000"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/on -o kt --output-format csv -- $B > $O/on.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/off -o kt --output-format csv -- $B --refill-interval 0 > $O/off.log 2>&1
echo "session rc=$?"
