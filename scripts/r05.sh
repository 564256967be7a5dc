#!/bin/bash
# Round-5 GPU sessions: bash scripts/r05.sh <session>.  Every GPU step runs under its own
# time limit; the session stops at the first crash / timeout (pytest's 1 = failures is
# reported and the session goes on only where noted).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=$1
O=gpurun_out/r05_$S
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -25 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', r['avg_kernel_us'] and round(r['avg_kernel_us'],2), 'frac', r['frac'] and round(r['frac'],3), r['kernel'], 'n', r['kernel_samples'], 'B/gpu', d['config']['boards_per_gpu'], 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])"; }
gpusuite() { run pytest_gpu ${1:-900} python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider; local rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; return $rc; }
case $S in
s1)  # the stripped build + the half-wave kernel: its parity first, the GPU suite, smoke, the driver's command, every share, timing-event probe
  run pytest_half 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "half and batched" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_half.log | head -30; tail -1 $O/pytest_half.log; [ $rc -le 1 ] || exit $rc
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  grep '^{' $O/bench_driver.log; line bench_driver
  run b65536 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line b65536
  for bb in 8192 4096; do
    run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line b$bb
  done
  for bb in 8192 4096 16384; do
    run h$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none --step-kernel half || exit 1; line h$bb
  done
  run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line p2
  run l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line l30
  run probe_timing_65536 300 python scripts/probe_timing.py 65536 || exit 1; cat $O/probe_timing_65536.log | tail -1 | cut -c1-3000
  run probe_timing_8192 300 python scripts/probe_timing.py 8192 || exit 1; cat $O/probe_timing_8192.log | tail -1 | cut -c1-3000
  ;;
s2)  # phase stamps of the half-wave kernel vs the one-wave kernels; the driver's command with the new kernel timing
  for k in small half; do for bb in 8192 4096; do
    TD_PROBE_KERNEL=$k TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_${k}_$bb 300 python scripts/probe_phases.py $bb 10 600 || exit 1
    cat $O/phases_${k}_$bb.log
  done; done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line bench_driver
  grep -o '"kernel_timing": "[^"]*"' $O/bench_driver.log
  ;;
s3)  # half-wave kernel with the early observation pass: its parity, phase stamps, lines beside the one-wave kernels
  run pytest_half 900 python -u -m pytest tests -m gpu -q -k "half" --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_half.log | head -30; tail -1 $O/pytest_half.log; [ $rc -le 1 ] || exit $rc
  for bb in 8192 4096; do
    TD_PROBE_KERNEL=half TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_half_$bb 300 python scripts/probe_phases.py $bb 10 600 || exit 1
    grep -E "obs|rt |attacker|march" $O/phases_half_$bb.log
  done
  for r in 1 2; do for bb in 8192 4096 16384 32768 65536; do for k in auto half; do
    run ${k}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 40000 ? 300 : bb > 20000 ? 500 : 2000)) --timing none --step-kernel $k || exit 1; line ${k}_${bb}_$r
  done; done; done
  ;;
s4)  # why the half-wave kernel is slow: SQ counters of small / half / half without the early pass at 8,192 boards
  V=$PWD/gym-td_amd/lib/variants
  for v in small half noearly; do
    lib=$PWD/gym-td_amd/lib/libtdstep.so; k=$v; [ $v = noearly ] && { lib=$V/libtdstep_noearly.so; k=half; }
    BENCH="python bench.py --global-batch 8192 --steps 20 --warmup 2 --burnin 300 --no-cpu-baseline --timing none --step-kernel $k"
    TDSTEP_LIB=$lib run pmc1_$v 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR -d $O/pmc1_$v -o pmc --output-format csv -- $BENCH || exit 1
    TDSTEP_LIB=$lib run pmc2_$v 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -d $O/pmc2_$v -o pmc --output-format csv -- $BENCH || exit 1
    TDSTEP_LIB=$lib run kt_$v 120 timeout -s KILL 100 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- $BENCH || exit 1
  done
  python3 scripts/pmc_compare.py $O small half noearly > $O/pmc_compare.txt 2>&1; cat $O/pmc_compare.txt
  for v in small half noearly; do for d in pmc1 pmc2 kt; do
    find $O/${d}_$v -name "*stats.csv" -exec cp {} $O/${d}_${v}_stats.csv \; 2>/dev/null; rm -rf $O/${d}_$v
  done; done
  TDSTEP_LIB=$V/libtdstep_noearly.so run nb_8192 200 python bench.py --global-batch 8192 --no-cpu-baseline --steps 2000 --timing none --step-kernel half; line nb_8192
  ;;
s5)  # placement of the observation: offsets into one contiguous block, 30x30 / 16,384 and 10x10 / 65,536
  run off30 400 python scripts/probe_offset.py 30 16384 100 || exit 1; grep -h offset $O/off30.log | tr '\n' ' '; echo
  run off10 400 python scripts/probe_offset.py 10 65536 200 || exit 1; grep -h offset $O/off10.log | tr '\n' ' '; echo
  ;;
s6)  # issue priority by dispatch order in one-round grids (variants p4: 4 levels, p2: first half high)
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do for v in prod p4 p2; do for bb in 8192 4096; do
    lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v != prod ] && lib=$V/libtdstep_$v.so
    TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
  done; done; done
  for v in p4 p2; do
    TDSTEP_LIB=$V/libtdstep_$v.so run pytest_$v 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "small and not full_size" --timeout 300 --timeout-method thread -p no:cacheprovider
    rc=$?; tail -1 $O/pytest_$v.log; [ $rc -le 1 ] || exit $rc
  done
  ;;
s7)  # compact group map (NC > 256): GPU suite, 30x30 / 2p lines, the driver's command
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    run l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line l30_$r
    run p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line p2_$r
  done
  run l30_large 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none --step-kernel large || exit 1; line l30_large
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver
  ;;
s8)  # compact group map vs none at 30x30 (same box), 2p; the driver's command with the pre-pass kernel timing
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2 3; do for v in prod nocompact; do
    lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v != prod ] && lib=$V/libtdstep_$v.so
    TDSTEP_LIB=$lib run l30_${v}_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line l30_${v}_$r
  done; done
  for v in prod nocompact; do
    lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v != prod ] && lib=$V/libtdstep_$v.so
    TDSTEP_LIB=$lib run p2_${v} 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line p2_${v}
  done
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line bench_driver_$r
    grep -o '"frac_withheld[^}]*' $O/bench_driver_$r.log || true
  done
  run pytest_30 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deep.py tests/test_gpu_envs.py -m gpu -q -x -k "30 or 20" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -1 $O/pytest_30.log; [ $rc -le 1 ] || exit $rc
  ;;
s9)  # the driver's command: where the kernel is sampled (pre / post pass), and the timed region alone
  for r in 1 2; do
    for m in pre post; do
      run drv_${m}_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --kernel-sampling $m || exit 1; line drv_${m}_$r
    done
    run drv_none_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --timing none || exit 1; line drv_none_$r
    run drv_256_$r 300 python bench.py --gpus 1 --steps 256 --warmup 5 --no-cpu-baseline --event-every 32 || exit 1; line drv_256_$r
  done
  ;;
s10)  # is the slow 20-step window after the pre-pass the pass or the step range?  timed-region sampling every 2nd/4th launch at K=20
  for bi in 1200 1456 1461 1520; do
    run none_b$bi 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --timing none --burnin $bi || exit 1; line none_b$bi
  done
  for r in 1 2; do
    for bb in 65536 8192 4096; do
      run none_${bb}_$r 300 python bench.py --global-batch $bb --steps 20 --warmup 5 --no-cpu-baseline --timing none || exit 1; line none_${bb}_$r
      for e in 2 4; do
        run e${e}_${bb}_$r 300 python bench.py --global-batch $bb --steps 20 --warmup 5 --no-cpu-baseline --event-every $e || exit 1; line e${e}_${bb}_$r
      done
    done
  done
  ;;
s11)  # kernel sampled inside the timed region (stride from the warm-up): the driver's command, its kernel trace, the other lines
  for r in 1 2 3; do
    run drv_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line drv_$r
  done
  run kt_drv 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_drv -o kt --output-format csv -- python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  line kt_drv; grep -h "td_step_kernel" $(find $O/kt_drv -name "*kernel_stats.csv") | cut -c1-200
  for bb in 8192 4096; do
    run k20_$bb 300 python bench.py --global-batch $bb --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line k20_$bb
    run k2000_$bb 300 python bench.py --global-batch $bb --steps 2000 --no-cpu-baseline || exit 1; line k2000_$bb
  done
  run p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line p2
  run l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line l30
  ;;
s12)  # 16-bit cell words at L = 10: the GPU suite, the driver's command, the L = 10 lines, the bytes at 65,536
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    run drv_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line drv_$r
    run b65536_$r 300 python bench.py --steps 300 --no-cpu-baseline || exit 1; line b65536_$r
  done
  for bb in 8192 4096 32768; do
    run b${bb} 300 python bench.py --global-batch $bb --steps 2000 --no-cpu-baseline || exit 1; line b$bb
  done
  OUT=$O NAME=c16_65536 B=65536 timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
  rm -rf $O/c16_65536/FETCH_SIZE $O/c16_65536/WRITE_SIZE
  ;;
s13)  # A/B on one box: this build (16-bit cell words, rolled flag fold + 8 waves/SIMD for the multi-action scan) vs libtdstep_prev.so
  for r in 1 2; do
    for v in prev new; do
      lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v = prev ] && lib=$PWD/gym-td_amd/lib/libtdstep_prev.so
      TDSTEP_LIB=$lib run ${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_p2_$r
    done
    for bb in 4096 8192 16384 65536; do
      st=2000; [ $bb -ge 65536 ] && st=300
      for v in prev new; do
        lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v = prev ] && lib=$PWD/gym-td_amd/lib/libtdstep_prev.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  for v in prev new; do
    lib=$PWD/gym-td_amd/lib/libtdstep.so; [ $v = prev ] && lib=$PWD/gym-td_amd/lib/libtdstep_prev.so
    TDSTEP_LIB=$lib run ${v}_p2_32768 300 python bench.py --workload 2p-middle-multi --global-batch 32768 --steps 100 --no-cpu-baseline --timing none || exit 1; line ${v}_p2_32768
  done
  ;;
s14)  # probes: c16 without the end / start compares (v1: wrong observation, timing only); the u32 build with vmcnt(0) after the opponent prefetch (v2)
  for r in 1 2; do
    for bb in 4096 16384 8192 65536; do
      st=2000; [ $bb -ge 65536 ] && st=300
      for v in prev new v1 v2; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = new ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s15)  # per-phase instruction attribution at 8,192 boards: builds without the observation (x1), channel_scalars (x2), enemy_stats (x3)
  BENCH="python bench.py --global-batch 8192 --steps 20 --warmup 2 --burnin 300 --no-cpu-baseline --timing none"
  for v in base x1 x2 x3; do
    lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run pmc1_$v 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_WR -d $O/pmc1_$v -o pmc --output-format csv -- $BENCH || exit 1
    TDSTEP_LIB=$lib run kt_$v 120 timeout -s KILL 100 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- $BENCH || exit 1
    TDSTEP_LIB=$lib run t_$v 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline --timing none || exit 1; line t_$v
  done
  python3 scripts/pmc_compare.py $O base x1 x2 x3 > $O/pmc_compare.txt; cat $O/pmc_compare.txt
  rm -rf $O/pmc1_* $O/kt_*
  ;;
s16)  # probes of the small kernel's shape: 4 waves per SIMD over 2 rounds (y1), two boards per wave in sequence (y3)
  for r in 1 2; do
    for v in base y1 y3; do
      lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_8192_$r 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline --timing none || exit 1; line ${v}_8192_$r
    done
  done
  for bb in 4096 16384; do
    for v in base y3; do
      lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_small_$bb 300 python bench.py --global-batch $bb --steps 2000 --no-cpu-baseline --timing none --step-kernel small || exit 1; line ${v}_small_$bb
    done
  done
  ;;
s17)  # 24-bit multiplies for the divisions by L and by L^2/4 (v_mul_hi_u32 / v_mul_lo_u32 are quarter rate): the GPU suite, then A/B vs libtdstep_base.so
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for bb in 4096 8192 16384 65536; do
      st=2000; [ $bb -ge 65536 ] && st=300
      for v in base new; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = new ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
    for v in base new; do
      lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = new ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_p2_$r
      TDSTEP_LIB=$lib run ${v}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_l30_$r
    done
  done
  ;;
s18)  # final-build validation and profiles: GPU suite, smoke, the driver's command, every line, kernel traces, PMC bytes
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r
  done
  run line_65536 300 python bench.py --steps 300 --no-cpu-baseline || exit 1; line line_65536
  run line_32768 300 python bench.py --global-batch 32768 --steps 600 --no-cpu-baseline || exit 1; line line_32768
  run line_16384 300 python bench.py --global-batch 16384 --steps 1000 --no-cpu-baseline || exit 1; line line_16384
  run line_8192 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline || exit 1; line line_8192
  run line_4096 300 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline || exit 1; line line_4096
  run line_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline || exit 1; line line_l30
  kt() { local name=$1; shift; run kt_$name 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- "$@" || return 1; cp $(find $O/kt_$name -name "*kernel_stats.csv") $O/kt_${name}_kernel_stats.csv; rm -rf $O/kt_$name; grep -h td_step_kernel $O/kt_${name}_kernel_stats.csv | cut -c1-160; }
  kt drv python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  kt b8192 python bench.py --global-batch 8192 --steps 300 --no-cpu-baseline || exit 1
  kt b4096 python bench.py --global-batch 4096 --steps 300 --no-cpu-baseline || exit 1
  kt p2 python bench.py --workload 2p-middle-multi --steps 100 --no-cpu-baseline || exit 1
  kt l30 python bench.py --workload def-large --global-batch 16384 --steps 100 --no-cpu-baseline || exit 1
  for spec in def-small:65536 def-small:8192 def-small:4096 2p-middle-multi:16384 def-large:16384; do
    wl=${spec%%:*}; bb=${spec##*:}
    OUT=$O/pmc NAME=${wl}_$bb WL=$wl B=$bb timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
    rm -rf $O/pmc/${wl}_$bb/FETCH_SIZE $O/pmc/${wl}_$bb/WRITE_SIZE
  done
  ;;
s19)  # one-wave kernels: binary-plane windows early (z1); observation windows per batch 2 (z2) / 8 (z3) instead of 4
  for r in 1 2; do
    for spec in 8192:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base z1 z2 z3; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s20)  # every board of the BASELINE-sized batches against the C restatement (new parity test)
  run pytest_every 1000 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k every_board --timeout 900 --timeout-method thread -p no:cacheprovider --durations=0
  rc=$?; grep -E "PASSED|FAILED|^E  |passed|failed|s call" $O/pytest_every.log | head -40; exit $rc
  ;;
s21)  # s19 then s20 in one call
  bash scripts/r05.sh s19 || exit 1
  bash scripts/r05.sh s20
  ;;
s22)  # the observation stream alone (scripts/obs_ceiling.hip): the practical write ceiling of the step's store shape
  run obs_ceiling 200 ./scripts/bin/obs_ceiling || exit 1; cat $O/obs_ceiling.log
  ;;
s23)  # the N > 1 control flow of this round's bench.py (kernel sampled in the timed region, MAX over ranks) with ranks sharing one GPU over gloo
  TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 run n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 || exit 1; line n2; grep -h '^{' $O/n2.log | cut -c1-1500
  TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 run n8 400 python bench.py --gpus 8 --steps 20 --warmup 5 || exit 1; line n8; grep -h '^{' $O/n8.log | cut -c1-1500
  ;;
s24)  # the observation stream alone at 20x20 and 30x30 (16,384 boards)
  run obs_ceiling_20 200 ./scripts/bin/obs_ceiling 20 || exit 1; cat $O/obs_ceiling_20.log
  run obs_ceiling_30 200 ./scripts/bin/obs_ceiling 30 || exit 1; cat $O/obs_ceiling_30.log
  ;;
s25)  # phase stamps at 8,192 boards: the product vs the build without the observation writer (x1)
  for v in stamps x1stamps; do
    TD_PROBE_KERNEL=small TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run phases_${v}_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
    cat $O/phases_${v}_8192.log | grep -v amdgpu
  done
  ;;
s26)  # captured(): the HBM config load kept apart from the LDS one (no FLAT load, no vmcnt(0) behind the wave's stores) -- w1
  for r in 1 2; do
    for spec in 8192:2000 4096:2000 16384:1000 65536:300; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base w1; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  TD_PROBE_KERNEL=small TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_w1stamps.so run phases_w1_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
  grep -v amdgpu $O/phases_w1_8192.log
  ;;
s27)  # w2 = w1 + vmcnt(0) before the state stores (no wait on the wave's own stores in the late phases): A/B and phase stamps
  for r in 1 2; do
    for spec in 8192:2000 4096:2000 16384:1000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base w1 w2; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  TD_PROBE_KERNEL=small TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_w2stamps.so run phases_w2_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
  grep -v amdgpu $O/phases_w2_8192.log
  ;;
s28)  # issue sensitivity: +8 dependent SALU (ps) / VALU (pv) per observation window
  for r in 1 2; do
    for spec in 8192:2000 65536:300; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base ps pv; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s29)  # the class-by-class observation writer (write_obs_lean, one-wave kernels at 10x10): parity first, then A/B vs libtdstep_base.so
  run pytest_lean 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store_policy.py tests/test_gpu_envs.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_lean.log | head -20; tail -1 $O/pytest_lean.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    for spec in 8192:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base new; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = new ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s30)  # final-build validation and profiles (after the captured() change): GPU suite, smoke, the driver's command, every line, kernel traces, PMC bytes
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r
  done
  run line_65536 300 python bench.py --steps 300 --no-cpu-baseline || exit 1; line line_65536
  run line_32768 300 python bench.py --global-batch 32768 --steps 600 --no-cpu-baseline || exit 1; line line_32768
  run line_16384 300 python bench.py --global-batch 16384 --steps 1000 --no-cpu-baseline || exit 1; line line_16384
  run line_8192 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline || exit 1; line line_8192
  run line_4096 300 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline || exit 1; line line_4096
  run line_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline || exit 1; line line_l30
  kt() { local name=$1; shift; run kt_$name 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- "$@" || return 1; cp $(find $O/kt_$name -name "*kernel_stats.csv") $O/kt_${name}_kernel_stats.csv; rm -rf $O/kt_$name; grep -h td_step_kernel $O/kt_${name}_kernel_stats.csv | cut -c1-160; }
  kt drv python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  kt b8192 python bench.py --global-batch 8192 --steps 300 --no-cpu-baseline || exit 1
  kt b4096 python bench.py --global-batch 4096 --steps 300 --no-cpu-baseline || exit 1
  kt p2 python bench.py --workload 2p-middle-multi --steps 100 --no-cpu-baseline || exit 1
  kt l30 python bench.py --workload def-large --global-batch 16384 --steps 100 --no-cpu-baseline || exit 1
  for spec in def-small:65536 def-small:8192 def-small:4096 2p-middle-multi:16384 def-large:16384; do
    wl=${spec%%:*}; bb=${spec##*:}
    OUT=$O/pmc NAME=${wl}_$bb WL=$wl B=$bb timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
    rm -rf $O/pmc/${wl}_$bb/FETCH_SIZE $O/pmc/${wl}_$bb/WRITE_SIZE
  done
  ;;
s31)  # l2: class-by-class observation writer, 4 windows at a time (LDS reads first): parity on it, then A/B vs the product
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_l2.so run pytest_l2 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_store_policy.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_l2.log | head -20; tail -1 $O/pytest_l2.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    for spec in 8192:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base l2; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s32)  # the multi-action flag fold: 12 loads in flight at 6 waves per SIMD (f1), 4 at 8 (f2), vs the product (8 at 8)
  for r in 1 2; do
    for v in base f1 f2; do
      lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_p2_$r
    done
  done
  ;;
s33)  # kernel choice at the N = 2 / 4 shares: every step kernel at 16,384 and 32,768 boards (and 8,192)
  for r in 1 2; do
    for bb in 16384 32768 8192; do
      for k in auto large small small2; do
        run ${k}_${bb}_$r 300 python bench.py --global-batch $bb --steps 600 --no-cpu-baseline --timing none --step-kernel $k || exit 1; line ${k}_${bb}_$r
      done
    done
  done
  ;;
s34)  # the two-wave kernel over more rounds: 65,536 / 49,152 / 32,768 / 8,192 boards, large or small vs small2
  for r in 1 2 3; do
    for spec in 65536:large:300 49152:large:400 32768:large:600 8192:small:2000; do
      bb=${spec%%:*}; rest=${spec#*:}; k=${rest%%:*}; st=${rest##*:}
      for kk in $k small2; do
        run ${kk}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel $kk || exit 1; line ${kk}_${bb}_$r
      done
    done
  done
  ;;
s35)  # final-build validation and profiles (TD-def 10x10 on the two-wave kernel at every batch above one round): GPU suite, smoke, the driver's command, every line, kernel traces, PMC bytes
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r
  done
  run line_65536 300 python bench.py --steps 300 --no-cpu-baseline || exit 1; line line_65536
  run line_32768 300 python bench.py --global-batch 32768 --steps 600 --no-cpu-baseline || exit 1; line line_32768
  run line_16384 300 python bench.py --global-batch 16384 --steps 1000 --no-cpu-baseline || exit 1; line line_16384
  run line_8192 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline || exit 1; line line_8192
  run line_4096 300 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline || exit 1; line line_4096
  run line_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline || exit 1; line line_l30
  kt() { local name=$1; shift; run kt_$name 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- "$@" || return 1; cp $(find $O/kt_$name -name "*kernel_stats.csv") $O/kt_${name}_kernel_stats.csv; rm -rf $O/kt_$name; grep -h td_step_kernel $O/kt_${name}_kernel_stats.csv | cut -c1-160; }
  kt drv python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  kt b8192 python bench.py --global-batch 8192 --steps 300 --no-cpu-baseline || exit 1
  kt b4096 python bench.py --global-batch 4096 --steps 300 --no-cpu-baseline || exit 1
  kt p2 python bench.py --workload 2p-middle-multi --steps 100 --no-cpu-baseline || exit 1
  kt l30 python bench.py --workload def-large --global-batch 16384 --steps 100 --no-cpu-baseline || exit 1
  kt b32768 python bench.py --global-batch 32768 --steps 300 --no-cpu-baseline || exit 1
  for spec in def-small:65536 def-small:8192 def-small:4096 2p-middle-multi:16384 def-large:16384; do
    wl=${spec%%:*}; bb=${spec##*:}
    OUT=$O/pmc NAME=${wl}_$bb WL=$wl B=$bb timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
    rm -rf $O/pmc/${wl}_$bb/FETCH_SIZE $O/pmc/${wl}_$bb/WRITE_SIZE
  done
  ;;
s36)  # live-slot loads in the two-wave kernel (live) vs the speculative 16 + 16 slots: parity, A/B, PMC; launch ramp of multi-wave workgroups
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_live.so run pytest_live 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k small2 --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_live.log | head -20; tail -1 $O/pytest_live.log; [ $rc -eq 0 ] || exit $rc
  run ramp 120 scripts/bin/launch_ramp wg || exit 1; cat $O/ramp.log
  for r in 1 2; do
    for spec in 65536:300 32768:600 16384:1000 4096:2000; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base live; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_live.so OUT=$O/pmc NAME=live_65536 B=65536 timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_live.so OUT=$O/pmc NAME=live_4096 B=4096 timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
  rm -rf $O/pmc/*/FETCH_SIZE $O/pmc/*/WRITE_SIZE
  ;;
s37)  # the observation store stream in other shapes (scripts/obs_ceiling.hip shapes): waves per board, boards in flight
  run shapes 120 scripts/bin/obs_ceiling shapes || exit 1; cat $O/shapes.log
  ;;
s38)  # issue priority for the observation writer (s_setprio 1 / 3 inside write_obs_lines) vs the product
  for r in 1 2; do
    for spec in 65536:300 32768:600 8192:2000 4096:2000; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base p1 p3; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s39)  # td_step_kernel_group (16 / 8 boards per workgroup, the group's waves write its windows together): parity, A/B vs the product
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_g16.so run pytest_g16 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "large" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_g16.log | head -20; tail -1 $O/pytest_g16.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for spec in 65536:300 32768:600 16384:1000; do
      bb=${spec%%:*}; st=${spec##*:}
      run base_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line base_${bb}_$r
      for v in g16 g8; do
        TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s40)  # the group kernel's structure without the group writer (g16s: 16 boards per workgroup, each wave its own observation; g1s: one), and 4 boards per group
  for spec in 65536:300 16384:1000; do
    bb=${spec%%:*}; st=${spec##*:}
    run base_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line base_${bb}
    run large_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line large_${bb}
    for v in g1s g16s g4 g16; do
      TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run ${v}_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line ${v}_${bb}
    done
  done
  ;;
s41)  # final-build validation and profiles on the round's last sources (s35's steps): GPU suite, smoke, the driver's command, every line, kernel traces, PMC bytes
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r
  done
  run line_65536 300 python bench.py --steps 300 --no-cpu-baseline || exit 1; line line_65536
  run line_32768 300 python bench.py --global-batch 32768 --steps 600 --no-cpu-baseline || exit 1; line line_32768
  run line_16384 300 python bench.py --global-batch 16384 --steps 1000 --no-cpu-baseline || exit 1; line line_16384
  run line_8192 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline || exit 1; line line_8192
  run line_4096 300 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline || exit 1; line line_4096
  run line_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline || exit 1; line line_l30
  kt() { local name=$1; shift; run kt_$name 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- "$@" || return 1; cp $(find $O/kt_$name -name "*kernel_stats.csv") $O/kt_${name}_kernel_stats.csv; rm -rf $O/kt_$name; grep -h td_step_kernel $O/kt_${name}_kernel_stats.csv | cut -c1-160; }
  kt drv python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  kt b8192 python bench.py --global-batch 8192 --steps 300 --no-cpu-baseline || exit 1
  kt b4096 python bench.py --global-batch 4096 --steps 300 --no-cpu-baseline || exit 1
  kt p2 python bench.py --workload 2p-middle-multi --steps 100 --no-cpu-baseline || exit 1
  kt l30 python bench.py --workload def-large --global-batch 16384 --steps 100 --no-cpu-baseline || exit 1
  kt b32768 python bench.py --global-batch 32768 --steps 300 --no-cpu-baseline || exit 1
  for spec in def-small:65536 def-small:8192 def-small:4096 2p-middle-multi:16384 def-large:16384; do
    wl=${spec%%:*}; bb=${spec##*:}
    OUT=$O/pmc NAME=${wl}_$bb WL=$wl B=$bb timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
    rm -rf $O/pmc/${wl}_$bb/FETCH_SIZE $O/pmc/${wl}_$bb/WRITE_SIZE
  done
  ;;
s42)  # fewer boards per CU in the two-wave kernel (extra dynamic LDS per workgroup, TD_DYN_LDS in the dyn build): 10x10 65,536, 2p, 30x30
  L=$PWD/gym-td_amd/lib/libtdstep_dyn.so
  for r in 1 2; do
    for d in 0 7600 13200; do
      TD_DYN_LDS=$d TDSTEP_LIB=$L run d10_${d}_$r 300 python bench.py --steps 300 --no-cpu-baseline --timing none --step-kernel small2 || exit 1; line d10_${d}_$r
    done
    for d in 0 5200 10800; do
      TD_DYN_LDS=$d TDSTEP_LIB=$L run d20_${d}_$r 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none --step-kernel small2 || exit 1; line d20_${d}_$r
    done
    for d in 0 1200 3400; do
      TD_DYN_LDS=$d TDSTEP_LIB=$L run d30_${d}_$r 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline --timing none --step-kernel small2 || exit 1; line d30_${d}_$r
    done
  done
  ;;
s43)  # the two-wave kernel without the early binary-plane pass (ne: both waves write after the step, windows split at 9) vs the product
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_ne.so run pytest_ne 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k small2 --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_ne.log | head -20; tail -1 $O/pytest_ne.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for spec in 65536:300 32768:600 16384:1000 4096:2000; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base ne; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel small2 || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s44)  # td_step_kernel_wq (8 / 4 boards per workgroup + as many writer waves fed through an LDS queue): parity, A/B vs the product
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_wq8.so run pytest_wq8 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "large" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_wq8.log | head -20; tail -1 $O/pytest_wq8.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for spec in 65536:300 32768:600 16384:1000; do
      bb=${spec%%:*}; st=${spec##*:}
      run base_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line base_${bb}_$r
      for v in wq8 wq4; do
        TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s45)  # the round's closing check on the final tree: GPU suite, smoke, the driver's command twice
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do
    run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r
  done
  grep -h '"traffic"' $O/bench_driver_1.log | grep -o '"traffic": [^,]*' | head -1
  ;;
s46)  # the queue-fed writer kernel with 1 / 2 boards per workgroup (libs built from the s44 commit): does the per-workgroup max-of-boards cost explain s44?
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_wq1.so run pytest_wq1 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "large and batched" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -1 $O/pytest_wq1.log; [ $rc -le 1 ] || exit $rc
  for spec in 65536:300 16384:1000; do
    bb=${spec%%:*}; st=${spec##*:}
    run base_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line base_${bb}
    for v in wq1 wq2; do
      TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run ${v}_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line ${v}_${bb}
    done
  done
  ;;
s47)  # the queue-fed writer kernel without scratch (7 waves per SIMD: 67 VGPRs, no spill; 1 / 2 boards per workgroup) vs the product
  for spec in 65536:300 16384:1000; do
    bb=${spec%%:*}; st=${spec##*:}
    run base_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line base_${bb}
    for v in wq1w7 wq2w7; do
      TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_$v.so run ${v}_${bb} 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --step-kernel large || exit 1; line ${v}_${bb}
    done
  done
  ;;
*) echo "unknown session $S"; exit 2;;
esac
