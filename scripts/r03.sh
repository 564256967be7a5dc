#!/bin/bash
# Round-3 GPU sessions: bash scripts/r03.sh <session>.  Every GPU step runs under its own
# time limit; the session stops at the first crash / timeout (pytest's 1 = failures
# is reported and the session goes on only where noted).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=$1
O=gpurun_out/r03_$S
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -25 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', round(r['frac'],3), r['kernel'], 'n', d['n_gpus'], d.get('world_size_reported'), 'B/gpu', d['config']['boards_per_gpu'], 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])"; }
case $S in
s1)  # the kernel-parametrised parity suite, smoke, default line, N = 2 self-launch rehearsal
  run pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_default 300 python bench.py || exit 1
  grep '^{' $O/bench_default.log; line bench_default
  export TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1
  run bench_n2 300 python bench.py --gpus 2 --no-cpu-baseline --steps 200 || exit 1
  unset TD_BENCH_DIST_BACKEND TD_BENCH_SAME_DEVICE
  line bench_n2
  ;;
s2)  # the failures of s1 after the fixes, and the new reset-sequence test
  run pytest_gpu 700 python -u -m pytest tests/test_gpu_roadgen.py tests/test_gpu_envs.py tests/test_gpu_deep.py -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -40; tail -3 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  ;;
s3)  # full suite, then every workload line on this build, refills off as the bound
  run pytest_gpu 700 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -20; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for bb in 32768 16384 8192 4096; do
    run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 || exit 1; line b$bb
    run b${bb}_norefill 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --refill-interval 0 || exit 1; line b${bb}_norefill
  done
  run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 1000 || exit 1; line p2
  run large 300 python bench.py --workload def-large --no-cpu-baseline --steps 300 || exit 1; line large
  ;;
s4)  # dry-ring draws in the step (refill interval 0 tests on every kernel), GPU suite, A/B vs the no-draw build
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for v in nodraw dry; do for bb in 65536 8192 4096; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 2000)) || exit 1; line ab_${v}_${bb}_$r
  done; done; done
  for v in nodraw dry; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 500 || exit 1; line ab_${v}_p2
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_large 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 300 || exit 1; line ab_${v}_large
  done
  ;;
s5)  # write ceiling at the guide's shape and the step's shape; current-build profiles of configs[2] / configs[4]
  run write_ceiling 300 ./scripts/bin/write_ceiling || exit 1
  cat $O/write_ceiling.log
  NO_PHASES=1 PROF_DIR=$O/prof_2p WL=2p-middle-multi B=16384 run prof_2p 900 bash scripts/profile_session.sh || exit 1
  NO_PHASES=1 PROF_DIR=$O/prof_large WL=def-large B=16384 run prof_large 900 bash scripts/profile_session.sh || exit 1
  ;;
s6)  # step-kernel A/B per workload (two-wave kernel at large batches), timing-event overhead, PC sampling at 8,192
  for wl in "def-large 16384" "def-large 131072" "2p-middle-multi 16384" "def-small 65536" "def-small 16384"; do
    set -- $wl
    for k in large small2; do
      run ab_${1}_$2_$k 300 python bench.py --workload $1 --global-batch $2 --no-cpu-baseline --steps 200 --step-kernel $k || exit 1; line ab_${1}_$2_$k
    done
  done
  for bb in 65536 8192; do
    run ev_none_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 20 --warmup 5 --timing none || exit 1; line ev_none_$bb
    run ev_1_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 20 --warmup 5 || exit 1; line ev_1_$bb
    run ev_none200_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 200 --timing none || exit 1; line ev_none200_$bb
    run ev_1_200_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 200 --event-every 1 || exit 1; line ev_1_200_$bb
  done
  ;;
s7)  # step kernel by batch: every kernel at the strong-scaling shares and around the thresholds, two passes
  for r in 1 2; do
    for bb in 32768 16384 12288 8192 6144 4096; do for k in large small small2; do
      run k_${bb}_${k}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 400 --step-kernel $k || exit 1; line k_${bb}_${k}_$r
    done; done
    for bb in 16384 32768 65536; do for k in large small2; do
      run kl_${bb}_${k}_$r 300 python bench.py --workload def-large --global-batch $bb --no-cpu-baseline --steps 100 --step-kernel $k || exit 1; line kl_${bb}_${k}_$r
    done; done
  done
  ;;
s8)  # GPU suite on the new kernel rule + scalar lane reads; lines; issue / i-cache counters at 8,192 and 65,536
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for bb in 65536 32768 16384 8192 4096; do
    run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 1000 || exit 1; line b$bb
  done
  for bb in 8192 65536; do
    B="python bench.py --global-batch $bb --steps 20 --warmup 2 --burnin 300 --no-cpu-baseline"
    run pmcA_$bb 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $O/pmcA_$bb -o pmc --output-format csv -- $B || exit 1
    run pmcB_$bb 300 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVES -d $O/pmcB_$bb -o pmc --output-format csv -- $B || exit 1
    run pmcC_$bb 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ -d $O/pmcC_$bb -o pmc --output-format csv -- $B || exit 1
  done
  ;;
s9)  # per-phase wave cycles (stamps build): alone on its SIMD (256 boards), 4,096, 8,192, 65,536; the tail boards
  for bb in 256 4096 8192 65536; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_$bb 300 python scripts/probe_phases.py $bb 10 600 || exit 1
    cat $O/phases_$bb.log | grep -v amdgpu.ids
  done
  ;;
s10) # kernel arguments read through the kernarg segment (product) vs by value: A/B, then the GPU suite
  for r in 1 2; do for v in byval karg; do
    for bb in 65536 16384 8192 4096; do
      TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 400 : 2000)) || exit 1; line ab_${v}_${bb}_$r
    done
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 300 || exit 1; line ab_${v}_p2_$r
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run ab_${v}_large_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line ab_${v}_large_$r
  done; done
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  ;;
s11) # the round's build: GPU suite, every workload line, refill cost at the small shares (interleaved A/B)
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_default 300 python bench.py || exit 1
  grep '^{' $O/bench_default.log; line bench_default
  for bb in 32768 16384; do run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 1000 || exit 1; line b$bb; done
  for r in 1 2; do for bb in 8192 4096; do
    run b${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 || exit 1; line b${bb}_$r
    run b${bb}_norefill_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 --refill-interval 0 || exit 1; line b${bb}_norefill_$r
  done; done
  run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 500 || exit 1; line p2
  run large16k 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 300 || exit 1; line large16k
  run large 300 python bench.py --workload def-large --no-cpu-baseline --steps 100 || exit 1; line large
  ;;
s12) # the ring guard: auto-reset under load with refills off on every kernel, then its cost (guard off = A/B only)
  run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "under_load|FAIL|^E  " $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for g in 0 4; do for bb in 65536 8192 4096; do
    TD_GUARD_EVERY=$g run g${g}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line g${g}_${bb}_$r
  done; done; done
  ;;
s13) # the ring guard at G = 3 (rings below 3 only): under-load tests, then its cost against guard off
  run pytest_load 600 python -u -m pytest tests/test_gpu_envs.py -k autoreset_under_load -v --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "PASS|FAIL|^E  " $O/pytest_load.log | head -30; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for g in 0 3; do for bb in 65536 8192 4096; do
    TD_GUARD_EVERY=$g run g${g}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line g${g}_${bb}_$r
  done; done; done
  for g in 0 3; do
    TD_GUARD_EVERY=$g run g${g}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 300 || exit 1; line g${g}_p2
  done
  ;;
s14) # rings of 16, guard every 15th step: the GPU suite, then guard / serial-refill A/Bs
  run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "under_load|FAIL|^E  " $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for v in prod noguard serial serial12; do for bb in 65536 8192 4096; do
    case $v in prod) E="";; noguard) E="TD_GUARD_EVERY=0";; serial) E="TD_REFILL_SERIAL=1";; serial12) E="TD_REFILL_SERIAL=1 TD_REFILL_WALKS=12";; esac
    env $E true; export $E 2>/dev/null
    run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line ${v}_${bb}_$r
    unset TD_GUARD_EVERY TD_REFILL_SERIAL TD_REFILL_WALKS
  done; done; done
  ;;
s15) # state stores deferred to the end of the step, no flat loads: GPU suite, every workload line, refills off as the bound
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for bb in 65536 32768 16384 8192 4096; do
    run b${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line b${bb}_$r
  done; done
  for bb in 8192 4096; do
    run b${bb}_norefill 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 --refill-interval 0 || exit 1; line b${bb}_norefill
  done
  run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 500 || exit 1; line p2
  run large16k 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 300 || exit 1; line large16k
  ;;
s16) # A/B on one box: state stores at the step's end + no flat loads (product) vs stores where final + flat (early)
  for r in 1 2 3; do for v in prod early; do for bb in 65536 8192 4096; do
    L=$PWD/gym-td_amd/lib/libtdstep.so; [ $v = early ] && L=$PWD/gym-td_amd/lib/variants/libtdstep_early.so
    TDSTEP_LIB=$L run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line ${v}_${bb}_$r
  done; done; done
  for v in prod early; do
    L=$PWD/gym-td_amd/lib/libtdstep.so; [ $v = early ] && L=$PWD/gym-td_amd/lib/variants/libtdstep_early.so
    TDSTEP_LIB=$L run ${v}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 300 || exit 1; line ${v}_p2
    TDSTEP_LIB=$L run ${v}_large 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line ${v}_large
  done
  ;;
s17) # A/B on one box: no flat loads (product) vs merged flat loads; step-refill event fence scope
  P=$PWD/gym-td_amd/lib/libtdstep.so; F=$PWD/gym-td_amd/lib/variants/libtdstep_flat.so
  for r in 1 2 3; do for v in prod flat; do for bb in 65536 8192 4096; do
    L=$P; [ $v = flat ] && L=$F
    TDSTEP_LIB=$L run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 500 : 3000)) || exit 1; line ${v}_${bb}_$r
  done; done; done
  for r in 1 2; do for fe in 0 1 2; do for bb in 8192 4096; do
    TD_EVENT_FENCE=$fe run fence${fe}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 || exit 1; line fence${fe}_${bb}_$r
  done; done; done
  ;;
s18|s19) # the round's build: GPU suite, smoke, default line; kernel traces + PMC per workload (summaries on the box)
  if [ $S = s18 ]; then
    run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
    rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
    run bench_default 300 python bench.py || exit 1
    grep '^{' $O/bench_default.log; line bench_default
    WLS="def-small:65536 def-small:8192 def-small:4096"
  else
    export TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1
    run bench_n2 300 python bench.py --gpus 2 --no-cpu-baseline --steps 200 || exit 1
    unset TD_BENCH_DIST_BACKEND TD_BENCH_SAME_DEVICE
    grep '^{' $O/bench_n2.log; line bench_n2
    WLS="2p-middle-multi:16384 def-large:16384"
  fi
  for wb in $WLS; do
    wl=${wb%%:*}; bb=${wb##*:}
    NO_PHASES=1 PROF_DIR=$O/prof_${wl}_$bb WL=$wl B=$bb run prof_${wl}_$bb 900 bash scripts/profile_session.sh || exit 1
    PMC_PROF=$O/prof_${wl}_$bb PMC_OUT=$O run sum_${wl}_$bb 120 python scripts/pmc_summary.py r03 $bb $wl || exit 1
    cat $O/sum_${wl}_$bb.log | tail -2
    rm -rf $O/prof_${wl}_$bb/pmc_* $O/prof_${wl}_$bb/kt/*_trace.csv
  done
  ;;
s20) # two-wave kernel: binary-plane windows written early by the second wave; parity on small2, then A/B vs the previous build
  run pytest_s2 600 python -u -m pytest tests -m gpu -q -k "small2 or 4096 or rollout" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_s2.log | head -30; tail -1 $O/pytest_s2.log; [ $rc -le 1 ] || exit $rc
  P=$PWD/gym-td_amd/lib/libtdstep.so; B0=$PWD/gym-td_amd/lib/variants/libtdstep_base.so
  for r in 1 2 3; do for v in prod base; do for wb in def-small:4096 def-small:16384 def-large:16384; do
    wl=${wb%%:*}; bb=${wb##*:}; L=$P; [ $v = base ] && L=$B0
    st=3000; [ $bb -gt 10000 ] && st=1000; [ $wl = def-large ] && st=200
    TDSTEP_LIB=$L run ${v}_${wl}_${bb}_$r 300 python bench.py --workload $wl --global-batch $bb --no-cpu-baseline --steps $st || exit 1; line ${v}_${wl}_${bb}_$r
  done; done; done
  ;;
s21) # observation stores write-through (sc1) vs non-temporal by batch (scripts/write_ceiling: sc1 6.7-6.9 TB/s up to 302 MB)
  for r in 1 2; do for wt in 0 1; do for bb in 65536 32768 16384 8192 4096; do
    st=3000; [ $bb -gt 10000 ] && st=1000; [ $bb -gt 40000 ] && st=500
    TD_OBS_WT=$wt run wt${wt}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $st || exit 1; line wt${wt}_${bb}_$r
  done; done; done
  for wt in 0 1; do
    TD_OBS_WT=$wt run wt${wt}_large16k 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line wt${wt}_large16k
    TD_OBS_WT=$wt run wt${wt}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 300 || exit 1; line wt${wt}_p2
  done
  ;;
s22) # full GPU suite on the early-window build; one- vs two-wave kernel at 8,192; phase stamps at 4,096 / 8,192
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for k in auto small2; do for bb in 8192 6144; do
    run k${k}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 --step-kernel $k || exit 1; line k${k}_${bb}_$r
  done; done; done
  for bb in 4096 8192; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_$bb 300 python scripts/probe_phases.py $bb 10 600 || exit 1
    grep -v amdgpu.ids $O/phases_$bb.log | head -30
  done
  ;;
s23) # refill cost on the current build: refill interval 16 (product) / 32 / 64 vs no refills and no guard (rings drain: the bound)
  for r in 1 2; do for v in r16 r32 r64 bound; do for bb in 8192 4096 65536; do
    st=3000; [ $bb -gt 10000 ] && st=500
    case $v in r16) A="";; r32) A="--refill-interval 32";; r64) A="--refill-interval 64";; bound) A="--refill-interval 0";; esac
    G=15; [ $v = bound ] && G=0
    TD_GUARD_EVERY=$G run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $st $A || exit 1; line ${v}_${bb}_$r
  done; done; done
  ;;
s24) # one-pass channel divisions (prod, refills every 64th step) vs the previous build at the same interval; longer intervals
  P=$PWD/gym-td_amd/lib/libtdstep.so; B0=$PWD/gym-td_amd/lib/variants/libtdstep_base.so
  for r in 1 2 3; do for v in prod base; do for bb in 8192 4096 65536; do
    st=3000; [ $bb -gt 10000 ] && st=500
    L=$P; [ $v = base ] && L=$B0
    TDSTEP_LIB=$L run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $st --refill-interval 64 || exit 1; line ${v}_${bb}_$r
  done; done; done
  for r in 1 2; do for ri in 128 256; do for bb in 8192 4096; do
    run r${ri}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 --refill-interval $ri || exit 1; line r${ri}_${bb}_$r
  done; done; done
  run pytest_load 600 python -u -m pytest tests/test_gpu_envs.py -k "autoreset_under_load" -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -1 $O/pytest_load.log; [ $rc -le 1 ] || exit $rc
  ;;
s25) # serial refills (step stream, no concurrency) at long intervals vs side refills every 64th step
  for r in 1 2; do for v in side64 ser256 ser1024; do for bb in 4096 8192; do
    case $v in side64) E=""; A="";; ser256) E="TD_REFILL_SERIAL=1"; A="--refill-interval 256";; ser1024) E="TD_REFILL_SERIAL=1"; A="--refill-interval 1024";; esac
    env $E timeout -k 10 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 $A > $O/${v}_${bb}_$r.log 2>&1 || { tail $O/${v}_${bb}_$r.log; exit 1; }; line ${v}_${bb}_$r
  done; done; done
  ;;
s26) # the device road generator's time per draw (one wave per SIMD), kernel trace
  for bb in 256 1024; do
    run draw_$bb 200 python scripts/probe_draw.py $bb 10 || exit 1; grep "^B=" $O/draw_$bb.log
    run kt_draw_$bb 200 rocprofv3 --kernel-trace --stats -d $O/kt_draw_$bb -o kt --output-format csv -- python scripts/probe_draw.py $bb 10 || exit 1
    cut -c1-150 $O/kt_draw_$bb/kt_kernel_stats.csv | head -6
  done
  ;;
s27) # where the device road generator's time goes (diagnostic build)
  for bb in 256 1024; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_genstamps.so run parts_$bb 200 python scripts/probe_draw_parts.py $bb 10 || exit 1
    grep -v amdgpu.ids $O/parts_$bb.log
  done
  ;;
s29) # towers targeting in parallel on boards with few enemies: GPU suite, then A/B vs the previous build
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  P=$PWD/gym-td_amd/lib/libtdstep.so; B0=$PWD/gym-td_amd/lib/variants/libtdstep_base.so
  for r in 1 2 3; do for v in prod base; do for bb in 4096 8192 65536; do
    st=3000; [ $bb -gt 10000 ] && st=500
    L=$P; [ $v = base ] && L=$B0
    TDSTEP_LIB=$L run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $st || exit 1; line ${v}_${bb}_$r
  done; done; done
  for v in prod base; do
    L=$P; [ $v = base ] && L=$B0
    TDSTEP_LIB=$L run ${v}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 300 || exit 1; line ${v}_p2
  done
  ;;
s32) # the step's staged-record read: acquire + plain loads (product) vs sc1 loads without the acquire (noacq)
  P=$PWD/gym-td_amd/lib/libtdstep.so; V=$PWD/gym-td_amd/lib/variants/libtdstep_noacq.so
  TDSTEP_LIB=$V run pytest_load 600 python -u -m pytest tests/test_gpu_envs.py -k "autoreset_under_load" -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -1 $O/pytest_load.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2 3; do for v in prod noacq; do for bb in 4096 8192 65536; do
    st=3000; [ $bb -gt 10000 ] && st=500
    L=$P; [ $v = noacq ] && L=$V
    TDSTEP_LIB=$L run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $st || exit 1; line ${v}_${bb}_$r
  done; done; done
  ;;
s33) # long steady-state runs on the final build (board flags, episode counts)
  run long_8192 400 python bench.py --global-batch 8192 --no-cpu-baseline --steps 20000 || exit 1; line long_8192
  run long_4096 400 python bench.py --global-batch 4096 --no-cpu-baseline --steps 20000 || exit 1; line long_4096
  run long_65536 400 python bench.py --no-cpu-baseline --steps 3000 || exit 1; line long_65536
  ;;
s34) # refill walk budget per launch (TD_REFILL_WALKS; product: 3 per step of interval = 192) at the small shares
  for r in 1 2; do for w in 192 48 12 768; do for bb in 4096 8192; do
    TD_REFILL_WALKS=$w run w${w}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 3000 || exit 1; line w${w}_${bb}_$r
  done; done; done
  ;;
s35) # per-phase wave cycles on the final build (stamps build): 4,096 / 8,192 / 65,536 boards
  for bb in 4096 8192 65536; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_$bb 300 python scripts/probe_phases.py $bb 10 600 || exit 1
    grep -v amdgpu.ids $O/phases_$bb.log | head -30
  done
  ;;
s36) # the clean rebuild of the final sources: GPU suite, smoke, default line
  run pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_default 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  grep '^{' $O/bench_default.log; line bench_default
  ;;
*) echo "unknown session $S"; exit 2 ;;
esac
echo "session $S rc=0"
