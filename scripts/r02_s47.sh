#!/bin/bash
# Round-2 GPU session 47: the N > 1 control flow of bench.py on the final build, ranks
# sharing one GPU over gloo (the 8-GPU RCCL run is the driver's): N = 2 and N = 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/s47
mkdir -p $O
for n in 2 8; do
  echo "== n$n $(date +%T)"
  timeout -k 10 300 env TD_BENCH_DIST_BACKEND=gloo TD_BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 50 --warmup 5 > $O/bench_n${n}_rehearsal.log 2>&1 || { tail -5 $O/bench_n${n}_rehearsal.log; exit 1; }
  grep '^{' $O/bench_n${n}_rehearsal.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(' ', d['metric'], d['n_gpus'], d['config']['global_batch'], d['config']['boards_per_gpu'], d['scaling'], round(d['value']/1e6,1), 'M/s', d['board_flags'], d['episodes']['per_rank'])"
done
echo "session rc=0"
