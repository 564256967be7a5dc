#!/bin/bash
# Round-2 GPU session 27: where the refill cost at 8,192 boards goes (kernel trace, per-queue timeline).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s27
mkdir -p $O
B="python bench.py --no-cpu-baseline --timing none --global-batch 8192 --steps 2000"
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/on -o kt --output-format csv -- $B > $O/on.log 2>&1 &&
python scripts/kt_gaps.py $O/on/kt_kernel_trace.csv 2000 --detail > $O/gaps_on.txt 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/r16 -o kt --output-format csv -- $B --refill-interval 16 > $O/r16.log 2>&1 &&
python scripts/kt_gaps.py $O/r16/kt_kernel_trace.csv 2000 --detail > $O/gaps_r16.txt 2>&1
rc=$?
head -3 $O/on/kt_kernel_trace.csv > $O/trace_head.txt 2>/dev/null
cat $O/gaps_on.txt $O/gaps_r16.txt
echo "session rc=$rc"
