#!/bin/bash
# Round-4 GPU sessions: bash scripts/r04.sh <session>.  Every GPU step runs under its own
# time limit; the session stops at the first crash / timeout (pytest's 1 = failures is
# reported and the session goes on only where noted).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
S=$1
O=gpurun_out/r04_$S
mkdir -p $O
run() { local name=$1 secs=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -ne 0 ] && tail -25 "$O/$name.log"; return $rc; }
line() { grep -h '^{' "$O/$1.log" | python3 -c "import json,sys
for l in sys.stdin: d=json.loads(l); r=d['roofline']; print('   %-18s' % '$1', round(d['value']/1e6,1), 'M/s  step', round(d['ms_per_step']*1e3,2), 'us  kernel', round(r['avg_kernel_us'],2), 'frac', r['frac'] and round(r['frac'],3), r['kernel'], 'n', r['kernel_samples'], 'B/gpu', d['config']['boards_per_gpu'], 'flags', d.get('board_flags'), 'eps', d['episodes']['finished'])"; }
gpusuite() { run pytest_gpu ${1:-900} python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider; local rc=$?; grep -E "^(FAILED|E  )" $O/pytest_gpu.log | head -30; tail -1 $O/pytest_gpu.log; return $rc; }
case $S in
s1)  # host probe, the GPU suite on the ABI-3 build, smoke, the driver's command, the small shares
  (python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>&1; nproc) > $O/host.log 2>&1; cat $O/host.log
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
  grep '^{' $O/bench_driver.log; line bench_driver
  for bb in 8192 4096; do
    run b$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 || exit 1; line b$bb
  done
  ;;
s2)  # board order + XCD map: GPU suite (every kernel), A/B at 8,192 / 4,096 / 65,536, PMC bytes, phase stamps, timing-event flags
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for v in "1 1" "0 1" "0 0"; do set -- $v; for bb in 8192 4096; do
      TD_ORDER=$1 TD_XCD_MAP=$2 run o$1x$2_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line o$1x$2_${bb}_$r
    done; done
    for x in 1 0; do
      TD_XCD_MAP=$x run x${x}_65536_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line x${x}_65536_$r
    done
  done
  for x in 1 0; do for bb in 65536 8192; do
    OUT=$O/pmc NAME=x${x}_$bb B=$bb TD_XCD_MAP=$x run pmc_x${x}_$bb 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_x${x}_$bb.log
  done; done
  for o in 0 1; do
    TD_ORDER=$o TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_o${o}_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
    grep -E "rt |tail" $O/phases_o${o}_8192.log
  done
  run large30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line large30
  for f in 0 1; do for bb in 65536 4096; do
    TD_TEV_FLAGS=$f run tev${f}_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 10000 ? 200 : 2000)) || exit 1; line tev${f}_$bb
  done; done
  ;;
s3)  # A/B builds: boards per workgroup of the small kernel (TD_BPW), uniform channel divisions (chvu)
  for v in bpw2 bpw4; do
    TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so run pytest_$v 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envs.py -m gpu -q -k "small and not small2" --timeout 300 --timeout-method thread -p no:cacheprovider
    rc=$?; grep -E "^(FAILED|E  )" $O/pytest_$v.log | head -10; tail -1 $O/pytest_$v.log; [ $rc -le 1 ] || exit $rc
  done
  TDSTEP_LIB=$PWD/gym-td_amd/lib/variants/libtdstep_chvu.so run pytest_chvu 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_chvu.log | head -10; tail -1 $O/pytest_chvu.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for v in prod bpw2 bpw4 chvu; do for bb in 8192 4096; do
    lib=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    k=small; [ $v = chvu ] && k=auto
    TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none --step-kernel $k || exit 1; line ${v}_${bb}_$r
  done; done
  for v in prod chvu; do
    lib=$PWD/gym-td_amd/lib/variants/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_65536_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line ${v}_65536_$r
  done; done
  ;;
s4)  # XCD map x shared-line policy per workload, lazy opponent cache (hc16/hc28), BPW and uniform-division builds
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for v in hc28 hc16 bpw2 bpw4 chvu; do
    TDSTEP_LIB=$V/libtdstep_$v.so run pytest_$v 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
    rc=$?; grep -E "^(FAILED|E  )" $O/pytest_$v.log | head -10; tail -1 $O/pytest_$v.log; [ $rc -le 1 ] || exit $rc
  done
  for r in 1 2; do
    for xe in "1 1" "1 0" "0 1"; do set -- $xe
      TD_XCD_MAP=$1 TD_EDGE_WT=$2 run p_x$1e$2_65536_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line p_x$1e$2_65536_$r
    done
    for v in hc28 hc16; do
      TDSTEP_LIB=$V/libtdstep_$v.so TD_EDGE_WT=1 run ${v}_x1e1_65536_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line ${v}_x1e1_65536_$r
    done
    for xe in "1 1" "1 0" "0 1"; do set -- $xe
      TD_XCD_MAP=$1 TD_EDGE_WT=$2 run l30_x$1e$2_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line l30_x$1e$2_$r
      TD_XCD_MAP=$1 TD_EDGE_WT=$2 run p2_x$1e$2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line p2_x$1e$2_$r
    done
    for v in prod bpw2 bpw4 chvu; do for bb in 8192 4096; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      k=small; [ $v = chvu -o $v = prod ] && k=auto
      TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none --step-kernel $k || exit 1; line ${v}_${bb}_$r
    done; done
  done
  for v in prod hc28 hc16; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib TD_EDGE_WT=1 OUT=$O/pmc NAME=${v}_x1e1 B=65536 run pmc_${v} 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_${v}.log
  done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit 1; line bench_driver
  ;;
s5)  # board order in multi-round grids (small2 at 30x30 / 16,384 10x10; the large kernel: olarge build), driver command
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  TDSTEP_LIB=$V/libtdstep_olarge.so TD_ORDER=1 run pytest_olarge 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_envs.py -m gpu -q -k "large" --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; grep -E "^(FAILED|E  )" $O/pytest_olarge.log | head -10; tail -1 $O/pytest_olarge.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for o in 0 1; do
      TD_ORDER=$o run l30_o${o}_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line l30_o${o}_$r
      TD_ORDER=$o run s16k_o${o}_$r 200 python bench.py --global-batch 16384 --no-cpu-baseline --steps 1000 --timing none || exit 1; line s16k_o${o}_$r
      TDSTEP_LIB=$V/libtdstep_olarge.so TD_ORDER=$o run ol65_o${o}_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line ol65_o${o}_$r
      TDSTEP_LIB=$V/libtdstep_olarge.so TD_ORDER=$o run ol32_o${o}_$r 200 python bench.py --global-batch 32768 --no-cpu-baseline --steps 500 --timing none || exit 1; line ol32_o${o}_$r
      TDSTEP_LIB=$V/libtdstep_olarge.so TD_ORDER=$o run olp2_o${o}_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line olp2_o${o}_$r
    done
    run p65_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line p65_$r
  done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; line bench_driver
  ;;
s6)  # 30x30: reproduce r04/s2's 466-us line (timing mode, order, edge policy); refill waves at the small shares
  for r in 1 2; do
    for t in dispatch none; do for oe in "0 1" "1 0"; do set -- $oe
      TD_ORDER=$1 TD_EDGE_WT=$2 run l30_$t_o$1e$2_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing $t || exit 1; line l30_$t_o$1e$2_$r
    done; done
    for w in 1024 256 64; do for bb in 8192 4096; do
      TD_REFILL_WAVES=$w run rw${w}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line rw${w}_${bb}_$r
    done; done
    for bb in 8192 4096; do
      run norefill_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none --refill-interval 0 || exit 1; line norefill_${bb}_$r
    done
  done
  ;;
s7)  # block twist of the opponent stream (large kernel) vs lazy (nobt); lazy-hot small kernels (lhs) at 30x30; PMC
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  TDSTEP_LIB=$V/libtdstep_lhs.so run pytest_lhs 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider
  rc=$?; tail -1 $O/pytest_lhs.log; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do
    for v in prod nobt; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_65536_$r 200 python bench.py --no-cpu-baseline --steps 300 --timing none || exit 1; line ${v}_65536_$r
      TDSTEP_LIB=$lib run ${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_p2_$r
    done
    for v in prod lhs; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_l30_$r
      TDSTEP_LIB=$lib run ${v}_8192_$r 200 python bench.py --global-batch 8192 --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_8192_$r
    done
  done
  OUT=$O/pmc NAME=prod B=65536 run pmc_prod 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_prod.log
  ;;
s8)  # 30x30 bisect (builds of commits 9f7a2e2 / bf5cc12 vs current); summon-cost change at the small shares (vs nobt)
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do
    for v in prod c9f7 cbf5; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_l30_$r
    done
    for v in prod nobt; do for bb in 8192 4096; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
    done; done
  done
  ;;
s9)  # two-wave kernel: the second wave stores the board and the outputs (offload) vs the previous build (pre)
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do
    for v in prod pre; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      for bb in 4096 2048 16384; do
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
      done
      TDSTEP_LIB=$lib run ${v}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_l30_$r
    done
  done
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_4096 300 python scripts/probe_phases.py 4096 10 600 || exit 1
  grep -E "rt |tail|cycles/wave" $O/phases_4096.log
  ;;
s10)  # the profile of the current build: kernel trace + PMC per workload; smoke; driver command; small2 at 2p / 8,192
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  for r in 1 2; do
    run p2_small2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none --step-kernel small2 || exit 1; line p2_small2_$r
    run b8192_small2_$r 200 python bench.py --global-batch 8192 --no-cpu-baseline --steps 2000 --timing none --step-kernel small2 || exit 1; line b8192_small2_$r
  done
  ;;
s11)  # scalar-bitmap road generator in the refill kernel (prod) vs lane words (nosb): roadgen parity, draw cycles, small shares; 2p rule
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for v in sb nosb; do
    TDSTEP_LIB=$V/libtdstep_gs_$v.so run parts_${v} 300 python scripts/probe_draw_parts.py 1024 10 || exit 1; cat $O/parts_${v}.log | grep -v amdgpu
  done
  for r in 1 2; do
    for v in prod nosb; do
      lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
      for bb in 8192 4096; do
        TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
      done
    done
    run p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line p2_$r
  done
  # the profile of this build (kernel trace + PMC per workload) and the driver's command
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  run launch_ramp 120 ./scripts/bin/launch_ramp || exit 1; cat $O/launch_ramp.log
  ;;
s12)  # final build: GPU suite, scalar search in the refill kernel (draw cycles; small shares vs noproof), profiles, driver command
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  V=$PWD/gym-td_amd/lib/variants
  TDSTEP_LIB=$V/libtdstep_gs_hyb.so run parts_hyb 300 python scripts/probe_draw_parts.py 1024 10 || exit 1; grep -v amdgpu $O/parts_hyb.log
  for r in 1 2; do for v in prod noproof; do for bb in 8192 4096; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
  done; done; done
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  for bb in 65536 32768 16384 8192 4096; do
    run line_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) || exit 1; line line_$bb
  done
  run line_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line line_l30
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  ;;
s13)  # early opponent pre-draw (small kernels): GPU suite, A/B vs late (noearly) and consumed-at-end, phase stamps, launch ramp
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do for v in prod noearly early_end; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    for bb in 8192 4096 16384; do
      TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 2000 --timing none || exit 1; line ${v}_${bb}_$r
    done
    TDSTEP_LIB=$lib run ${v}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_l30_$r
  done; done
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
  grep -E "rt |tail" $O/phases_8192.log
  run launch_ramp 120 ./scripts/bin/launch_ramp || exit 1; cat $O/launch_ramp.log
  ;;
s14)  # early pre-draw consumed after the board step (default now); start priority A/B; phases; launch ramp with start priority
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do for v in prod sprio3 sprio1; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    for bb in 8192 4096 16384 65536; do
      TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) --timing none || exit 1; line ${v}_${bb}_$r
    done
  done; done
  TDSTEP_LIB=$PWD/gym-td_amd/lib/libtdstep_stamps.so run phases_8192 300 python scripts/probe_phases.py 8192 10 600 || exit 1
  grep -E "rt |tail" $O/phases_8192.log
  run launch_ramp 120 ./scripts/bin/launch_ramp || exit 1; cat $O/launch_ramp.log
  ;;
s15)  # launch ramp by work kind (SALU / LDS chain / VALU with sleeps); PMC bytes of the early-pre-draw build at 8,192 / 4,096
  run launch_ramp 120 ./scripts/bin/launch_ramp || exit 1; cat $O/launch_ramp.log
  for bb in 8192 4096; do
    OUT=$O/pmc NAME=prod_$bb B=$bb run pmc_$bb 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_$bb.log
  done
  ;;
s16)  # generator draw state uniform (SGPRs): GPU suite, draw cycles by part, the step rate beside the refills
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  TDSTEP_LIB=$V/libtdstep_gs.so run parts_gs 300 python scripts/probe_draw_parts.py 1024 10 || exit 1; grep -v amdgpu $O/parts_gs.log
  for r in 1 2; do for bb in 8192 4096 16384 65536; do
    run prod_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) --timing none || exit 1; line prod_${bb}_$r
  done; done
  run line_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line line_l30
  ;;
s17)  # 2p multi-action: the second wave folds the flags and writes the real actions (prod) vs the stepping wave (noss), 6 waves/SIMD (cap6)
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do for v in prod noss cap6; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib run ${v}_p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line ${v}_p2_$r
    TDSTEP_LIB=$lib run ${v}_p2_4096_$r 300 python bench.py --workload 2p-middle-multi --global-batch 4096 --no-cpu-baseline --steps 500 --timing none || exit 1; line ${v}_p2_4096_$r
  done; done
  run prod_8192 200 python bench.py --global-batch 8192 --no-cpu-baseline --steps 2000 --timing none || exit 1; line prod_8192
  ;;
s18)  # the early opponent window in the large kernel too (a refill every step) vs lazy refills: step time and bytes
  V=$PWD/gym-td_amd/lib/variants
  for r in 1 2; do for v in prod early_large; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    for bb in 65536 32768; do
      TDSTEP_LIB=$lib run ${v}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps 300 --timing none || exit 1; line ${v}_${bb}_$r
    done
  done; done
  for v in prod early_large; do
    lib=$V/libtdstep_$v.so; [ $v = prod ] && lib=$PWD/gym-td_amd/lib/libtdstep.so
    TDSTEP_LIB=$lib OUT=$O/pmc NAME=${v}_65536 B=65536 run pmc_$v 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_$v.log
  done
  ;;
s19)  # final build: GPU suite, smoke, profiles of five workloads (kernel trace, PMC bytes, SQ counters), bench lines, the driver's command
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  for bb in 65536 32768 16384 8192 4096; do
    run line_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) || exit 1; line line_$bb
  done
  run line_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line line_l30
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  ;;
s20)  # shared observation lines: write-through (TD_EDGE_WT=1, product) vs plain write-back stores merged in the XCD's L2 (2)
  for r in 1 2; do for e in 1 2; do
    for bb in 65536 32768 16384; do
      TD_EDGE_WT=$e run e${e}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 1000)) --timing none || exit 1; line e${e}_${bb}_$r
    done
    TD_EDGE_WT=$e run e${e}_p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line e${e}_p2_$r
    TD_EDGE_WT=$e run e${e}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line e${e}_l30_$r
  done; done
  TD_EDGE_WT=2 OUT=$O/pmc NAME=e2_65536 B=65536 run pmc_e2 600 bash scripts/pmc_ab.sh || exit 1; tail -1 $O/pmc_e2.log
  TD_EDGE_WT=2 run pytest_edge2 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 400 --timeout-method thread -p no:cacheprovider || exit 1; tail -1 $O/pytest_edge2.log
  ;;
s21)  # final build (plain shared observation lines): as s19
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  for bb in 65536 32768 16384 8192 4096; do
    run line_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) || exit 1; line line_$bb
  done
  run line_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line line_l30
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  ;;
s22)  # the 30x30 step time by buffer placement (probe_alloc), repeated 30x30 lines; store-policy parity test
  run alloc_l30 600 python scripts/probe_alloc.py 30 16384 3 6 || exit 1; grep -v amdgpu $O/alloc_l30.log
  for r in 1 2 3 4; do
    run l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line l30_$r
  done
  run pytest_store 600 python -u -m pytest tests/test_gpu_store_policy.py -m gpu -v -x --timeout 500 --timeout-method thread -p no:cacheprovider || exit 1; tail -4 $O/pytest_store.log
  ;;
s23)  # 30x30 step time over raw allocations: default vs contiguous (hipDeviceMallocContiguous)
  PROBE_MODE=hip run alloc_hip 600 python scripts/probe_alloc.py 30 16384 || exit 1; grep -v amdgpu $O/alloc_hip.log
  run alloc_l30 600 python scripts/probe_alloc.py 30 16384 2 6 || exit 1; grep -v amdgpu $O/alloc_l30.log
  ;;
s24)  # default vs contiguous observation allocations at 10x10 / 65,536 and 8,192, 20x20 / 16,384, 30x30 again
  for lb in "10 65536" "10 8192" "20 16384" "30 16384"; do set -- $lb
    PROBE_MODE=hip run alloc_hip_$1_$2 600 python scripts/probe_alloc.py $1 $2 || exit 1; grep -v amdgpu $O/alloc_hip_$1_$2.log
  done
  ;;
s25)  # contiguous device allocations (library state + the engine's observation): GPU suite, A/B vs TD_CONTIG=0
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for r in 1 2; do for c in 1 0; do
    for bb in 65536 32768 16384 8192 4096; do
      TD_CONTIG=$c run c${c}_${bb}_$r 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) --timing none || exit 1; line c${c}_${bb}_$r
    done
    TD_CONTIG=$c run c${c}_p2_$r 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line c${c}_p2_$r
    TD_CONTIG=$c run c${c}_l30_$r 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line c${c}_l30_$r
  done; done
  ;;
s26)  # plain state arrays; the engine's observation contiguous (TD_CONTIG_OBS=1, default) vs plain: GPU suite, A/B, final profiles
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  for c in 1 0; do
    for bb in 65536 32768 16384 8192 4096; do
      TD_CONTIG_OBS=$c run o${c}_${bb} 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) --timing none || exit 1; line o${c}_${bb}
    done
    TD_CONTIG_OBS=$c run o${c}_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 --timing none || exit 1; line o${c}_p2
    TD_CONTIG_OBS=$c run o${c}_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 --timing none || exit 1; line o${c}_l30
  done
  for wb in "def-small 65536" "def-small 8192" "def-small 4096" "2p-middle-multi 16384" "def-large 16384"; do set -- $wb
    NO_PHASES=1 PROF_DIR=$O/prof_$1_$2 WL=$1 B=$2 run prof_$1_$2 900 bash scripts/profile_session.sh || exit 1
  done
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  ;;
s27)  # the engine's observation contiguous from 512 MiB on (auto rule): GPU suite, smoke, bench lines, the driver's command
  gpusuite 900; rc=$?; [ $rc -le 1 ] || exit $rc
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
  for bb in 65536 32768 16384 8192 4096; do
    run line_$bb 200 python bench.py --global-batch $bb --no-cpu-baseline --steps $((bb > 20000 ? 300 : 2000)) || exit 1; line line_$bb
  done
  run line_p2 300 python bench.py --workload 2p-middle-multi --no-cpu-baseline --steps 200 || exit 1; line line_p2
  run line_l30 300 python bench.py --workload def-large --global-batch 16384 --no-cpu-baseline --steps 200 || exit 1; line line_l30
  run bench_driver 300 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1; grep '^{' $O/bench_driver.log; line bench_driver
  ;;
s28)  # observation allocation kinds: default 0, contiguous 4, fine-grained 1, uncached 3 (30x30 and 10x10 / 65,536)
  for lb in "30 16384" "10 65536"; do set -- $lb
    PROBE_MODE=hip PROBE_FLAGS=0,4,1,3 PROBE_REPS=2 run alloc_kinds_$1_$2 600 python scripts/probe_alloc.py $1 $2 || exit 1; grep -v amdgpu $O/alloc_kinds_$1_$2.log
  done
  ;;
*) echo "unknown session $S"; exit 2 ;;
esac
