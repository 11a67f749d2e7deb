#!/bin/bash
# Rehearse bench.py's N-rank path on ONE GPU (every rank on device 0, gloo
# collectives): exercises the stripe partition, weak-scaling frame counts, the
# max-over-ranks timing and the gather.  The driver's real N-GPU runs use RCCL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${RANKS:-2 8}; do
  RT_BENCH_BACKEND=gloo RT_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 \
    --warmup 1 --no-cpu-baseline > gpurun_out/bench_rehearse_n$n.log 2>&1
  rc=$?
  echo "ranks=$n rc=$rc"; tail -1 gpurun_out/bench_rehearse_n$n.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
