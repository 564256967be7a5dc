#!/bin/bash
# Round-6 GPU sessions: bash scripts/r06.sh <session>.  Every GPU step runs under its own
# time limit; the session stops at the first crash / timeout (pytest's 1 = failures is
# reported and the session goes on only where noted).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=$1
O=gpurun_out/r06_$S
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -25 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', r['avg_kernel_us'] and round(r['avg_kernel_us'],2), 'frac', r['frac'] and round(r['frac'],3), r['kernel'], 'n', r['kernel_samples'], 'B/gpu', d['config']['boards_per_gpu'], 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'], 'ranks_us', [round(x*1e3,2) for x in d.get('per_rank_ms_per_step', [])], 'barrier_us', [round(x,1) for x in d.get('closing_barrier_us', [])])"; }
gpusuite() { run pytest_gpu ${1:-900} python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider ${2}; local rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; return $rc; }
case $S in
s1)  # round 6 first build: new steady-state test + claims, GPU suite, smoke, the driver's command, N>1 rehearsal on one GPU
  run pytest_new 600 python -u -m pytest tests/test_gpu_steady.py tests/test_gpu_claims.py tests/test_gpu_rccl.py -m gpu -v -x --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )|PASSED|passed|failed" $O/pytest_new.log | head -30; [ $rc -le 1 ] || exit $rc
  gpusuite 1000; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver
  grep -h '^{' $O/bench_driver.log | cut -c1-3000
  TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 run n8 400 python bench.py --gpus 8 --steps 20 --warmup 5 || exit 1; line n8
  TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 run n2 300 python bench.py --gpus 2 --steps 20 --warmup 5 || exit 1; line n2
  ;;
s2)  # placement probe (boards a CU writes at once contiguous?), kernel trace + PMC bytes of the driver's command on this round's sources
  run obs_place 180 ./scripts/bin/obs_place || exit 1; cat $O/obs_place.log
  kt() { local name=$1; shift; run kt_$name 300 timeout -s KILL 280 rocprofv3 --kernel-trace --stats -d $O/kt_$name -o kt --output-format csv -- "$@" || return 1; cp $(find $O/kt_$name -name "*kernel_stats.csv") $O/kt_${name}_kernel_stats.csv; rm -rf $O/kt_$name; grep -h td_step_kernel $O/kt_${name}_kernel_stats.csv | cut -c1-160; }
  kt drv python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1
  OUT=$O/pmc NAME=def-small_65536 WL=def-small B=65536 timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
  rm -rf $O/pmc/def-small_65536/FETCH_SIZE $O/pmc/def-small_65536/WRITE_SIZE
  ;;
s3)  # cooperative writer probe: the waves of a workgroup write the boards it finished together (no barrier)
  run coop 240 ./scripts/bin/coop_writer || exit 1; cat $O/coop.log
  ;;
s4)  # the store-shape probe again (does 16 waves per board still stream at 7 TB/s on this box?)
  run shapes 240 ./scripts/bin/obs_ceiling shapes || exit 1; cat $O/shapes.log
  ;;
s5)  # 4 prefetched enemy slots in the TD-def small kernels (pf) + the header's second half stored only when it changed (hh, product lib) vs r06 s1 (base): parity, A/B, PMC bytes; store-shape probe
  run pytest_pf 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady.py tests/test_gpu_deep.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_pf.log | head -20; tail -1 $O/pytest_pf.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2; do
    for spec in 65536:300 8192:2000 4096:2000; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base pf hh; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = hh ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  OUT=$O/pmc NAME=def-small_65536 WL=def-small B=65536 timeout -k 10 700 bash scripts/pmc_ab.sh || exit 1
  rm -rf $O/pmc/def-small_65536/FETCH_SIZE $O/pmc/def-small_65536/WRITE_SIZE
  run shapes 240 ./scripts/bin/obs_ceiling shapes || exit 1; cat $O/shapes.log
  ;;
s6)  # issue priority 2 for boards with enemies (the small-batch tail) vs the product (hh), 3 rounds
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base prio; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s7)  # the cleaned tree (no diagnostic paths, header half store): steady-state tests over the five configs, GPU suite, smoke, the driver's command twice
  run pytest_steady 900 python -u -m pytest tests/test_gpu_steady.py -m gpu -v -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )|PASSED|passed|failed" $O/pytest_steady.log | head -20; [ $rc -le 1 ] || exit $rc
  gpusuite 1100 "--deselect tests/test_gpu_steady.py"; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r; done
  ;;
s8)  # the final build: every line with the bench's defaults, kernel traces, PMC bytes of the five workloads (pmc_traffic.json records)
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
s9)  # bench.py --gpus 2 end to end (gloo, both ranks on cuda:0) as a GPU test
  run pytest_ranks 400 python -u -m pytest tests/test_gpu_bench_ranks.py -m gpu -v -x --timeout 350 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )|PASSED|passed|failed" $O/pytest_ranks.log | head -20; [ $rc -le 1 ] || exit $rc
  ;;
s10)  # the 7-TB/s shape: narrow address band or few boards per CU? (scripts/obs_span.hip)
  run span 240 ./scripts/bin/obs_span || exit 1; cat $O/span.log
  ;;
s11)  # closing check on the final tree: build() on the box (no recompile expected), GPU suite, smoke, the driver's command twice
  run build 400 python -c "import time, __graft_entry__ as g; t = time.time(); g.build(); print('build() %.1f s' % (time.time() - t))" || exit 1; grep -E "build\(\)|Nothing|hipcc" $O/build.log | head -5
  gpusuite 1100; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r; done
  grep -h '"traffic"' $O/bench_driver_1.log | grep -o '"traffic": [^,]*' | head -1
  ;;
s12)  # kernel choice at configs[1] (4,096 boards) and the N = 8 share (8,192) on the final build: small / small2 / large
  for r in 1 2; do
    for spec in 4096 8192; do
      for k in small small2 large; do
        run ${k}_${spec}_$r 300 python bench.py --global-batch $spec --steps 2000 --no-cpu-baseline --timing none --step-kernel $k || exit 1; line ${k}_${spec}_$r
      done
    done
  done
  ;;
s13)  # issue priority by launch order (the last-launched quarter of a one-round grid at 3; lp) vs the product, 3 rounds
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base lp; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = base ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s14)  # the constant block's load issued with the board's loads (one L2 round trip fewer in front of each board; product) vs base: parity, A/B 3 rounds
  run pytest_cf 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady.py tests/test_gpu_deep.py tests/test_gpu_envs.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_cf.log | head -20; tail -1 $O/pytest_cf.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in base cf; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = cf ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  for v in base cf; do
    lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = cf ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_p2
    TDSTEP_LIB=$lib run ${v}_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_l30
  done
  ;;
s15)  # the kernel arguments the prologue needs read in one scalar round trip (pa, product) vs cf: parity, A/B 3 rounds
  run pytest_pa 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady.py tests/test_gpu_deep.py tests/test_gpu_envs.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_pa.log | head -20; tail -1 $O/pytest_pa.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in cf pa; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = pa ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  for v in cf pa; do
    lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = pa ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_p2 300 python bench.py --workload 2p-middle-multi --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_p2
    TDSTEP_LIB=$lib run ${v}_l30 300 python bench.py --workload def-large --global-batch 16384 --steps 200 --no-cpu-baseline --timing none || exit 1; line ${v}_l30
  done
  ;;
s16)  # the output pointers read together before the outputs are stored (po, product) vs pa: parity, A/B 3 rounds
  run pytest_po 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady.py tests/test_gpu_envs.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_po.log | head -20; tail -1 $O/pytest_po.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in pa po; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = po ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s17)  # the final build (constant block + argument prologue): GPU suite, smoke, the driver's command twice, every line, kernel traces, PMC bytes
  gpusuite 1100; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r; done
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
s18)  # what do episode ends cost at small batches?  auto-reset on (the metric) vs off (diagnostic: finished boards keep stepping)
  for r in 1 2; do
    for bb in 8192 4096; do
      for ar in 1 0; do
        run ar${ar}_${bb}_$r 300 python bench.py --global-batch $bb --steps 2000 --no-cpu-baseline --timing none --autoreset $ar || exit 1; line ar${ar}_${bb}_$r
      done
    done
  done
  ;;
s19)  # early layout hand-off (el, product) vs pa: full GPU suite on it, then A/B 3 rounds; then the auto-reset cost probe on both
  gpusuite 1100; rc=$?; [ $rc -eq 0 ] || exit 1
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in pa el; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = el ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  for v in pa el; do
    lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = el ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_ar0_8192 300 python bench.py --global-batch 8192 --steps 2000 --no-cpu-baseline --timing none --autoreset 0 || exit 1; line ${v}_ar0_8192
    TDSTEP_LIB=$lib run ${v}_ar0_4096 300 python bench.py --global-batch 4096 --steps 2000 --no-cpu-baseline --timing none --autoreset 0 || exit 1; line ${v}_ar0_4096
  done
  ;;
s20)  # long runs on the final build: no board flag, no guard timeout over 20,000 steps (8,192 / 4,096) and 3,000 (65,536)
  run long_8192 400 python bench.py --global-batch 8192 --steps 20000 --no-cpu-baseline || exit 1; line long_8192
  run long_4096 400 python bench.py --global-batch 4096 --steps 20000 --no-cpu-baseline || exit 1; line long_4096
  run long_65536 400 python bench.py --steps 3000 --no-cpu-baseline || exit 1; line long_65536
  grep -ho '"board_flags_nonzero": [0-9]*, "guard_timeouts_rank0": [0-9]*' $O/long_*.log
  ;;
s21)  # steady-state every-board tests incl. TD-atk / TD-2p discrete at 10x10
  run pytest_steady 900 python -u -m pytest tests/test_gpu_steady.py -m gpu -v -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )|PASSED|passed|failed" $O/pytest_steady.log | head -20; [ $rc -le 1 ] || exit $rc
  ;;
s22)  # convergent f64 divisions in channel_scalars (cs, product) vs pa: parity subset, A/B 3 rounds
  run pytest_cs 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steady.py tests/test_gpu_envs.py -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_cs.log | head -20; tail -1 $O/pytest_cs.log; [ $rc -eq 0 ] || exit $rc
  for r in 1 2 3; do
    for spec in 8192:2000 4096:2000 65536:300 32768:600; do
      bb=${spec%%:*}; st=${spec##*:}
      for v in pa cs; do
        lib=$PWD/gym-td_amd/lib/libtdstep_$v.so; [ $v = cs ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
  done
  ;;
s23)  # closing check on the final tree: build() on the box, GPU suite, smoke, the driver's command twice, bench.py's defaults
  run build 400 python -c "import time, __graft_entry__ as g; t = time.time(); g.build(); print('build() %.1f s' % (time.time() - t))" || exit 1; grep -E "build\(\)|Nothing|hipcc" $O/build.log | head -5
  gpusuite 1100; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for r in 1 2; do run bench_driver_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver_$r; done
  run bench_default 400 python bench.py || exit 1; line bench_default
  grep -h '"traffic"' $O/bench_driver_1.log | grep -o '"traffic": [^,]*' | head -1
  ;;
s24)  # the placement-report test
  run pytest_alloc 300 python -u -m pytest tests/test_gpu_store_policy.py -m gpu -v -x --timeout 250 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )|PASSED|passed|failed" $O/pytest_alloc.log | head -20; [ $rc -le 1 ] || exit $rc
  ;;
s25)  # layout draws only in the ring guard on the step stream (refill interval 0 in the timed steps) vs side-stream refills every 64th step, 3 rounds
  for r in 1 2 3; do
    for spec in 8192:3000 4096:3000 65536:300 16384:1500; do
      bb=${spec%%:*}; st=${spec##*:}
      run ri64_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none || exit 1; line ri64_${bb}_$r
      run ri0_${bb}_$r 300 python bench.py --global-batch $bb --steps $st --no-cpu-baseline --timing none --refill-interval 0 || exit 1; line ri0_${bb}_$r
    done
  done
  grep -ho '"board_flags_nonzero": [0-9]*, "guard_timeouts_rank0": [0-9]*' $O/ri0_*.log | sort | uniq -c
  ;;
*) echo "unknown session $S"; exit 2 ;;
esac
