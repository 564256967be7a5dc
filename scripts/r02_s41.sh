#!/bin/bash
# Round-2 GPU session 41: final profiles of the round's build (refills ordered after
# reset kernels in every mode): GPU parity suite, smoke, the no-wait refill A/B again
# (corrupt layouts were the refill racing the bench's staggering resets), the default
# bench line under the kernel tracer, PMC passes at 65,536 and 8,192 boards, and the
# 8,192 / 4,096 lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s41
mkdir -p $O/p65536 $O/p8192
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -5 "$O/$name.log"; return $rc; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
tail -1 $O/pytest_gpu.log
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
tail -1 $O/smoke.log
for bb in 4096 8192; do
  run nowait16_$bb 150 env TD_REFILL_NOWAIT=1 TD_REFILL_EVERY=16 python bench.py --no-cpu-baseline --steps 5000 --global-batch $bb || exit 1
  grep '^{' $O/nowait16_$bb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('   nowait16 $bb', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us', d['board_flags'])"
done
run bench_default 300 python bench.py || exit 1
grep '^{' $O/bench_default.log
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_BRANCH"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
for B in 65536 8192; do
  P=$O/p$B
  BENCH="python bench.py --global-batch $B --steps 20 --warmup 2 --no-cpu-baseline"
  if [ $B = 65536 ]; then KT="python bench.py"; else KT="python bench.py --global-batch $B --no-cpu-baseline --steps 1000"; fi
  run kt_$B 400 rocprofv3 --kernel-trace --stats -d $P/kt -o kt --output-format csv -- $KT || exit 1
  run pmc_fetch_$B 300 rocprofv3 --pmc FETCH_SIZE -d $P/pmc_fetch -o pmc --output-format csv -- $BENCH || exit 1
  run pmc_write_$B 300 rocprofv3 --pmc WRITE_SIZE -d $P/pmc_write -o pmc --output-format csv -- $BENCH || exit 1
  run pmc_sq1_$B 300 rocprofv3 --pmc $SQ1 -d $P/pmc_sq1 -o pmc --output-format csv -- $BENCH || exit 1
  run pmc_sq2_$B 300 rocprofv3 --pmc $SQ2 -d $P/pmc_sq2 -o pmc --output-format csv -- $BENCH || exit 1
done
mkdir -p $O/profiles
for B in 65536 8192; do
  PMC_PROF=$O/p$B PMC_OUT=$O/profiles python scripts/pmc_summary.py r02 $B def-small > $O/pmc_summary_$B.log 2>&1 || { cat $O/pmc_summary_$B.log; exit 1; }
  cat $O/pmc_summary_$B.log
  cp $O/p$B/kt/kt_kernel_stats.csv $O/profiles/r02_kt_stats_$B.csv
  python scripts/kt_gaps.py $O/p$B/kt/kt_kernel_trace.csv 1000 > $O/profiles/r02_kt_gaps_$B.txt 2>&1
done
rm -rf $O/p65536 $O/p8192  # raw traces and counter dumps stay on the box (64-MiB copy-back limit)
cp $O/profiles/pmc_traffic.json profiles/pmc_traffic.json
run bench_after_pmc 300 python bench.py --no-cpu-baseline || exit 1
grep '^{' $O/bench_after_pmc.log
run bench_8192 200 python bench.py --global-batch 8192 --no-cpu-baseline --steps 2000 || exit 1
grep '^{' $O/bench_8192.log
run bench_4096 200 python bench.py --global-batch 4096 --no-cpu-baseline --steps 2000 || exit 1
grep '^{' $O/bench_4096.log
echo "session rc=0"
